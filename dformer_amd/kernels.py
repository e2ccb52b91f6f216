"""Thin tensor-level wrappers over the C ABI (allocation of outputs / workspaces + launch).

All tensors are CUDA (HIP) tensors; 2-D operands are [rows, cols] views whose last stride is 1
(the row stride is passed through as `ld`, so column slices of wider buffers work in place).
Activations are float32 or bfloat16; statistics / params / param-grads are float32.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, dtype_code, lib, ptr, stream

_ws_cache = {}

# When set to a list, every GEMM launch appends its descriptor fields (tools/gemm_sweep.py)
GEMM_TRACE = None


# ---------------------------------------------------------------- accounting (bench.py)
# When ACCOUNT is a list, every wrapper appends (kernel funcs launched, algorithmic FLOPs, algorithmic
# HBM bytes, MFMA peak class) after its C call: the FLOPs/bytes an ideal kernel for that op must do
# (inputs read once, outputs written once; workspaces and split-K partials are not algorithmic).
# The library's launch tracer says which kernels the call enqueued; the first one is charged.
ACCOUNT = None
TAG = ""  # component label of the launches that follow (set by the modules; census breakdown)
_FUNCS = (ctypes.c_void_p * 64)()


def trace(flags, probe=None):
    """Launch tracer of the library: flags 0 off, 1 record launched kernels, 2 time (HIP events) the
    kernel(s) named `probe` (demangled, as rocprofv3 prints it; a name or a list of names; None = every
    kernel), 3 both."""
    if isinstance(probe, (list, tuple)):
        probe = "\n".join(probe)
    check(lib.dfm_trace_set(flags, probe.encode() if probe else None), "dfm_trace_set")


def trace_read():
    """[(kernel name, ms)] of the timed launches since the last read (synchronises on the last one)."""
    cap = 1 << 16
    funcs = (ctypes.c_void_p * cap)()
    ms = (ctypes.c_float * cap)()
    n = lib.dfm_trace_read(funcs, ms, cap)
    return [(kernel_name(funcs[i]), float(ms[i])) for i in range(min(n, cap))]


_NAMES = {}


def kernel_name(func):
    nm = _NAMES.get(func)
    if nm is None:
        nm = _NAMES[func] = lib.dfm_kernel_name(func).decode()
    return nm


def _acct(flops, nbytes, peak="bf16"):
    n = lib.dfm_trace_take(_FUNCS, 64)
    ACCOUNT.append((tuple(_FUNCS[i] for i in range(min(n, 64))), float(flops), float(nbytes), peak, TAG))


def _es(t):
    return t.element_size()


def _pref(ps):
    return None if ps is None else ctypes.byref(ps)


def _ws(nbytes, dev):
    """Scratch buffer per (device, stream) that only grows (the library never allocates); one per
    stream so kernels running concurrently on a side stream never share a workspace. A buffer that
    is outgrown is retired, not freed: a HIP graph captured earlier keeps using its pointer."""
    if nbytes == 0:
        return None
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None:  # a captured graph may still hold the old pointer: never free it
            _ws_retired.append(buf)
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
        _ws_cache[key] = buf
    return buf


_ws_retired = []


def ld(t):
    assert t.dim() >= 2 and t.stride(-1) == 1, "inner dimension must be contiguous"
    return t.stride(-2)


def rows_of(t):
    return t.numel() // t.shape[-1] if t.is_contiguous() else t.shape[0]


# ------------------------------------------------------------------------------------------ GEMM
# ------------------------------------------------------------------ grouped weight gradients
# Inside `with wgrad_group():` the weight-gradient GEMMs (linear_wgrad) are not launched one by one:
# they are queued and issued at the end of the block as grouped launches (dfm_gemm_group, up to 8
# problems each + one split-K combine), so the independent dW GEMMs of a Block's backward share the
# chip instead of each splitting K over all of it. Their outputs must not be read before the block
# ends (they only feed the optimizer).
# The second stages of the parameter-gradient reductions issued inside (LayerNorm dgamma / dbeta,
# layer-scale dscale, depthwise dw / db: fixed-order sums over per-block partials) are deferred the
# same way and issued as ONE dfm_partial_sum_group launch per block instead of one small launch each;
# every deferred reduction keeps its own partials buffer until then.
_WG_PENDING = None
_RED_PENDING = None


WG_STREAM_MIN_FLOPS = 4e9


class wgrad_group:
    """Queue the weight-gradient GEMMs and reduction second stages issued inside; at exit issue
    them (flush_wgrad, flush_reductions) on the current stream, or on `stream` (after it waits for
    the current one), so that the current stream's later work does not wait for them."""

    def __init__(self, stream=None):
        self.stream = stream

    def __enter__(self):
        global _WG_PENDING, _RED_PENDING
        self.prev = (_WG_PENDING, _RED_PENDING)
        _WG_PENDING, _RED_PENDING = [], []
        return self

    def __exit__(self, exc_type, exc, tb):
        global _WG_PENDING, _RED_PENDING
        pending, reds = _WG_PENDING, _RED_PENDING
        _WG_PENDING, _RED_PENDING = self.prev
        if exc_type is None and (pending or reds):
            # a group worth less than WG_STREAM_MIN_FLOPS stays on the current stream: its launches take
            # about as long as the two cross-stream edges cost. Every group on the stream: DFormer-Tiny bs 8
            # (~2.5 GFLOP groups) 628.1 / 625.0 vs 639.9 / 639.0 images/s with none; from 8 GFLOP up: Tiny
            # 642.4 / 639.8 vs 639.5 / 638.7, DFormer-B flat (its ~5 GFLOP depth-branch ConvFFN groups stay);
            # from 4 GFLOP up: Tiny 651.2 / 649.5 vs 640.4 / 639.2, DFormer-B 496.9 / 504.7 vs 496.4 / 495.0
            if self.stream is None or sum(it[5] for it in pending) < WG_STREAM_MIN_FLOPS:
                if pending:
                    flush_wgrad(pending)
                if reds:
                    flush_reductions(reds)
            else:
                self.stream.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.stream):
                    for item in pending:  # operands written on the current stream, read on this one
                        item[2].record_stream(self.stream)
                        item[3].record_stream(self.stream)
                    if pending:
                        flush_wgrad(pending)
                    if reds:
                        flush_reductions(reds)
        return False


def _red_ws(nbytes, dev):
    """(workspace, DfmPartialSum or None): inside a wgrad_group a reduction gets a partials buffer of
    its own and a descriptor its entry point fills instead of launching the second stage."""
    if _RED_PENDING is None or nbytes == 0:
        return _ws(nbytes, dev), None
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    ps = _lib.PartialSum()
    _RED_PENDING.append((ps, buf))
    return buf, ps


def flush_reductions(reds):
    """Issue deferred reduction second stages as one dfm_partial_sum_group launch (16 per launch)."""
    n = len(reds)
    arr = (_lib.PartialSum * n)(*[r[0] for r in reds])
    cur = torch.cuda.current_stream()
    for _, buf in reds:  # partials written on a side stream are read here: no reuse before that
        buf.record_stream(cur)
    check(lib.dfm_partial_sum_group(n, ctypes.cast(arr, ctypes.c_void_p), stream()), "dfm_partial_sum_group")
    if ACCOUNT is not None:  # second stages: no algorithmic bytes (the partials are not algorithmic)
        _acct(0, 0)


def flush_wgrad(pending):
    """Issue queued GEMMs as grouped launches: problems of one dtype / operand layout, 8 per launch."""
    classes = {}
    for item in pending:
        d, dt = item[0], item[1]
        classes.setdefault((dt, d.a_kcontig, d.b_kcontig), []).append(item)
    for (dt, _, _), items in classes.items():
        for i in range(0, len(items), 8):
            chunk = items[i:i + 8]
            n = len(chunk)
            descs = (_lib.GemmDesc * n)(*[c[0] for c in chunk])
            pa = (ctypes.c_void_p * n)(*[c[2].data_ptr() for c in chunk])
            pb = (ctypes.c_void_p * n)(*[c[3].data_ptr() for c in chunk])
            pc = (ctypes.c_void_p * n)(*[c[4].data_ptr() for c in chunk])
            dev = chunk[0][2].device
            ws = _ws(lib.dfm_gemm_group_workspace_size(n, descs), dev)
            descs[0].workspace_bytes = ws.numel() if ws is not None else 0
            check(lib.dfm_gemm_group(dt, n, descs, ctypes.cast(pa, ctypes.c_void_p), ctypes.cast(pb, ctypes.c_void_p),
                                     ctypes.cast(pc, ctypes.c_void_p), ptr(ws), stream()), "dfm_gemm_group")
            if ACCOUNT is not None:
                _acct(sum(c[5] for c in chunk), sum(c[6] for c in chunk), chunk[0][7])


def gemm(a, b, *, M, N, K, a_kcontig, b_kcontig, lda, ldb, out, ldc, batch=1, stride_a=0, stride_b=0,
         stride_c=0, alpha=1.0, beta=0.0, bias=None, act=0, preact=None, ldpre=0, mul=None, ldmul=0, res=None,
         ldres=0, colscale=None, rowscale=None, rows_per_scale=1, split_k=0, act_col0=0, colsum=None,
         colsum_accumulate=False, mul_gelu_grad=False, mul2=None, out2=None, defer=False, collect=None):
    """One dfm_gemm launch. defer=True (weight gradients) inside `with wgrad_group():` queues it for
    the block's grouped launch instead; `collect` (a list, from gemm_many) receives it unlaunched."""
    dt = dtype_code(a)
    assert b.dtype == a.dtype, (a.dtype, b.dtype)
    c_f32 = int(out.dtype == torch.float32 and a.dtype != torch.float32)
    if out.dtype != torch.float32:
        assert out.dtype == a.dtype
    d = _lib.GemmDesc(M, N, K, batch, int(a_kcontig), int(b_kcontig), lda, ldb, ldc, stride_a, stride_b, stride_c,
                      alpha, beta, c_f32, ptr(bias), act, ptr(preact), ldpre, ptr(mul), ldmul, ptr(res), ldres,
                      ptr(colscale), ptr(rowscale), rows_per_scale, split_k, act_col0, ptr(colsum),
                      int(colsum_accumulate), int(mul_gelu_grad), 0, ptr(mul2), ld(mul2) if mul2 is not None else 0,
                      ptr(out2), ld(out2) if out2 is not None else 0)
    if GEMM_TRACE is not None:
        GEMM_TRACE.append({f: getattr(d, f) for f, _ in d._fields_ if not f in ("alpha", "beta")} |
                          {"dtype": dt, "beta": d.beta, "out_f32": out.dtype == torch.float32})
    es, nb = _es(a), max(batch, 1)
    byt = es * (M * K * nb + N * K * (nb if stride_b else 1))
    byt += M * N * nb * (out.element_size() * (2 if beta != 0.0 else 1))
    byt += es * M * N * nb * ((preact is not None) + (mul is not None) + (res is not None) + 2 * (out2 is not None))
    byt += 4 * N * (bias is not None) + 4 * M * (colsum is not None)
    peak = "bf16" if a.dtype != torch.float32 else "f32"
    if collect is not None:
        collect.append((d, dt, a, b, out, 2.0 * M * N * K * nb, byt, peak))
        return out
    if defer and _WG_PENDING is not None and a.is_cuda:
        # queued for the block's grouped launch; the tensors stay referenced until it is issued
        _WG_PENDING.append((d, dt, a, b, out, 2.0 * M * N * K * nb, byt, peak, colsum, bias))
        return out
    nbytes = lib.dfm_gemm_workspace_size(d)
    ws = _ws(nbytes, a.device)
    d.workspace_bytes = ws.numel() if ws is not None else 0
    check(lib.dfm_gemm(dt, d, ptr(a), ptr(b), ptr(out), ptr(ws), stream()), "dfm_gemm")
    if ACCOUNT is not None:
        _acct(2.0 * M * N * K * nb, byt, peak)
    return out


def gemm_many(calls):
    """Run independent GEMMs (thunks that call linear / linear_dgrad with collect=lst) as ONE grouped
    launch (dfm_gemm_group: k-contiguous A problems go to the LDS-DMA ring kernel's grouped variant);
    a single call launches alone. The calls must not read each other's outputs."""
    items = []
    for c in calls:
        c(items)
    if len(items) == 1:
        for d, dt, a, b, out, fl, by, peak in items:
            ws = _ws(lib.dfm_gemm_workspace_size(d), a.device)
            d.workspace_bytes = ws.numel() if ws is not None else 0
            check(lib.dfm_gemm(dt, d, ptr(a), ptr(b), ptr(out), ptr(ws), stream()), "dfm_gemm")
            if ACCOUNT is not None:
                _acct(fl, by, peak)
        return
    for i in range(0, len(items), 8):
        chunk = items[i:i + 8]
        n = len(chunk)
        descs = (_lib.GemmDesc * n)(*[c[0] for c in chunk])
        pa = (ctypes.c_void_p * n)(*[c[2].data_ptr() for c in chunk])
        pb = (ctypes.c_void_p * n)(*[c[3].data_ptr() for c in chunk])
        pc = (ctypes.c_void_p * n)(*[c[4].data_ptr() for c in chunk])
        ws = _ws(lib.dfm_gemm_group_workspace_size(n, descs), chunk[0][2].device)
        descs[0].workspace_bytes = ws.numel() if ws is not None else 0
        check(lib.dfm_gemm_group(chunk[0][1], n, descs, ctypes.cast(pa, ctypes.c_void_p), ctypes.cast(pb, ctypes.c_void_p),
                                 ctypes.cast(pc, ctypes.c_void_p), ptr(ws), stream()), "dfm_gemm_group")
        if ACCOUNT is not None:
            _acct(sum(c[5] for c in chunk), sum(c[6] for c in chunk), chunk[0][7])


def linear(x, w, bias=None, *, act=0, preact=None, mul=None, res=None, colscale=None, rowscale=None,
           rows_per_scale=1, out=None, beta=0.0, act_col0=0, collect=None):
    """y[M,N] = epi(x[M,K] @ w[N,K]^T)  (nn.Linear forward)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    return gemm(x, w, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=ld(x), ldb=ld(w), out=out, ldc=ld(out),
                beta=beta, bias=bias, act=act, preact=preact, ldpre=ld(preact) if preact is not None else 0,
                mul=mul, ldmul=ld(mul) if mul is not None else 0, res=res, ldres=ld(res) if res is not None else 0,
                colscale=colscale, rowscale=rowscale, rows_per_scale=rows_per_scale, act_col0=act_col0,
                collect=collect)


def linear_dgrad(dy, w, out=None, accumulate=False, mul=None, gelu_grad_of=None, mul2=None, out2=None,
                 collect=None):
    """dx[M,K] (+)= dy[M,N] @ w[N,K]   (times `mul` elementwise, or times gelu'(gelu_grad_of)); with
    mul2 / out2 also out2 = (dy @ w) * mul2 from the same accumulator (an elementwise product's two
    input gradients in one pass: out = g * y, out2 = g * x for the product x * y)."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    if gelu_grad_of is not None:
        mul = gelu_grad_of
    return gemm(dy, w, M=M, N=K, K=N, a_kcontig=True, b_kcontig=False, lda=ld(dy), ldb=ld(w), out=out, ldc=ld(out),
                beta=1.0 if accumulate else 0.0, mul=mul, ldmul=ld(mul) if mul is not None else 0,
                mul_gelu_grad=gelu_grad_of is not None, mul2=mul2, out2=out2, collect=collect)


def linear_wgrad(dy, x, out=None, accumulate=False, bias_grad=False, bias_out=None):
    """dW[N,K] (+)= dy[M,N]^T @ x[M,K]  (float32 output, split-K over M).
    bias_grad=True also returns db[N] = sum_M dy (fused: virtual all-ones column of x), written
    into `bias_out` when given (e.g. a slot of the optimizer's flat gradient buffer)."""
    M, N = dy.shape
    K = x.shape[1]
    if out is None:
        out = torch.empty(N, K, device=dy.device, dtype=torch.float32)
    db = None
    if bias_grad:
        db = bias_out if bias_out is not None else torch.empty(N, device=dy.device, dtype=torch.float32)
    gemm(dy, x, M=N, N=K, K=M, a_kcontig=False, b_kcontig=False, lda=ld(dy), ldb=ld(x), out=out,
         ldc=ld(out), beta=1.0 if accumulate else 0.0, colsum=db, colsum_accumulate=accumulate, defer=True)
    return (out, db) if bias_grad else out


def bmm(a, b, *, a_t=False, b_t=False, out=None, alpha=1.0, beta=0.0):
    """Batched out[b] (= or +=) op(a[b]) @ op(b[b]) for contiguous 3-D tensors (op = transpose if *_t)."""
    B = a.shape[0]
    M = a.shape[2] if a_t else a.shape[1]
    K = a.shape[1] if a_t else a.shape[2]
    N = b.shape[1] if b_t else b.shape[2]
    assert (b.shape[2] if b_t else b.shape[1]) == K
    if out is None:
        out = torch.empty(B, M, N, device=a.device, dtype=a.dtype)
    # A(m,k): a[m][k] (k-contig, lda=K) or a[k][m] (a_t: row-contig, lda=M)
    # B(k,n): b[k][n] (row-contig, ldb=N) or b[n][k] (b_t: k-contig, ldb=K)
    return gemm(a, b, M=M, N=N, K=K, a_kcontig=not a_t, b_kcontig=b_t, lda=a.shape[2], ldb=b.shape[2], out=out,
                ldc=N, batch=B, stride_a=a.shape[1] * a.shape[2], stride_b=b.shape[1] * b.shape[2],
                stride_c=M * N, alpha=alpha, beta=beta)


# ------------------------------------------------------------------------------------ LayerNorm
def layernorm(x, gamma, beta, eps=1e-6, out=None):
    rows, C = x.shape
    if out is None:
        out = torch.empty(rows, C, device=x.device, dtype=x.dtype)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    check(lib.dfm_layernorm_fwd(dtype_code(x), rows, C, ptr(x), ld(x), ptr(gamma), ptr(beta), eps, ptr(out),
                                ld(out), ptr(mean), ptr(rstd), stream()), "dfm_layernorm_fwd")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * 2 + 8 * rows)
    return out, mean, rstd


def layernorm_bwd(x, dy, gamma, mean, rstd, dx=None, accumulate=False, dres=None):
    """dx = LN'(dy) [+ dres] [+ dx when accumulate]; returns (dx, dgamma, dbeta)."""
    rows, C = x.shape
    if dx is None:
        dx = torch.empty(rows, C, device=x.device, dtype=x.dtype)
        accumulate = False
    dg = torch.empty(C, device=x.device, dtype=torch.float32)
    db = torch.empty(C, device=x.device, dtype=torch.float32)
    ws, ps = _red_ws(lib.dfm_layernorm_bwd_workspace(rows, C), x.device)
    check(lib.dfm_layernorm_bwd(dtype_code(x), rows, C, ptr(x), ld(x), ptr(dy), ld(dy), ptr(gamma), ptr(mean),
                                ptr(rstd), ptr(dres), ld(dres) if dres is not None else 0, ptr(dx), ld(dx),
                                int(accumulate), ptr(dg), ptr(db), ptr(ws), _pref(ps), stream()), "dfm_layernorm_bwd")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * (3 + (dres is not None) + bool(accumulate)) + 8 * rows)
    return dx, dg, db


def residual_bwd(dout, f, colscale, rowscale=None, rows_per_scale=1, df=None):
    """Block residual x + rowscale*ls*f backward: returns (df = dout*ls*rowscale, dls = sum dout*f*rowscale)."""
    rows, C = dout.shape
    if df is None:
        df = torch.empty(rows, C, device=dout.device, dtype=dout.dtype)
    dls = torch.empty(C, device=dout.device, dtype=torch.float32)
    ws, ps = _red_ws(lib.dfm_residual_bwd_workspace(rows, C), dout.device)
    check(lib.dfm_residual_bwd(dtype_code(dout), rows, C, ptr(dout), ld(dout), ptr(f), ld(f), ptr(colscale),
                               ptr(rowscale), rows_per_scale, ptr(df), ld(df), ptr(dls), ptr(ws), _pref(ps), stream()),
          "dfm_residual_bwd")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(dout) * 3)
    return df, dls


# ----------------------------------------------------------------------------- fused ConvFFN (K4)
def _acct_named(parts, peak="bf16"):
    """Account one entry point that launched several kernels: parts = [(name substring, flops, bytes)];
    each launched kernel is charged the first unused part whose substring its name contains."""
    n = lib.dfm_trace_take(_FUNCS, 64)
    used = [False] * len(parts)
    for i in range(min(n, 64)):
        f = _FUNCS[i]
        nm = kernel_name(f)
        fl = by = 0.0
        for j, (sub, pf, pb) in enumerate(parts):
            if not used[j] and sub in nm:
                used[j], fl, by = True, pf, pb
                break
        ACCOUNT.append(((f,), float(fl), float(by), peak, TAG))


def _ffn_desc(shape, C, hidden, eps):
    B, H, W = shape
    return _lib.ConvFFNDesc(B, H, W, C, hidden, eps)


def convffn_supported(dtype, shape, C, hidden):
    if dtype not in (torch.bfloat16, torch.float16):
        return False
    d = _ffn_desc(shape, C, hidden, 1e-6)
    code = _lib.BF16 if dtype == torch.bfloat16 else _lib.F16
    return bool(lib.dfm_convffn_supported(code, ctypes.byref(d)))


def convffn_fwd(x, shape, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls, rowscale=None, eps=1e-6, save_gelu=False):
    """Fused ConvFFN + Block residual (DFormer.py:48-67, 176-179). Returns (out, f, h, xn, mean, rstd)
    (+ (g, gp) = GELU(hpre), GELU'(hpre) with save_gelu, the op-level backward's operands):
    out = x + rowscale * ls * f, f = fc2 pre-residual output, h = fc1 output, LN output / statistics."""
    P, C = x.shape
    R = w1.shape[0]
    d = _ffn_desc(shape, C, R, eps)
    out, f = torch.empty_like(x), torch.empty_like(x)
    h = torch.empty(P, R, device=x.device, dtype=x.dtype)
    xn = torch.empty_like(x)
    mean = torch.empty(P, device=x.device, dtype=torch.float32)
    rstd = torch.empty(P, device=x.device, dtype=torch.float32)
    g = gp = None
    if save_gelu:
        g, gp = torch.empty_like(h), torch.empty_like(h)
    check(lib.dfm_convffn_fwd(dtype_code(x), ctypes.byref(d), ptr(x), ptr(ln_w), ptr(ln_b), ptr(w1), ptr(b1),
                              ptr(wpos), ptr(bpos), ptr(w2), ptr(b2), ptr(ls), ptr(rowscale), ptr(out), ptr(f),
                              ptr(h), ptr(xn), ptr(mean), ptr(rstd), ptr(g), ptr(gp), stream()), "dfm_convffn_fwd")
    if ACCOUNT is not None:
        es = _es(x)
        _acct(4.0 * P * C * R + 18.0 * P * R, es * P * (4 * C + R * (3 if save_gelu else 1)) + 8 * P + es * 2 * C * R)
    if save_gelu:
        return out, f, h, xn, mean, rstd, g, gp
    return out, f, h, xn, mean, rstd


def convffn_bwd(dout, x, h, xn, f, mean, rstd, shape, ln_w, ln_b, w1, wpos, bpos, w2, ls, rowscale=None, eps=1e-6,
                grads=None):
    """Backward of convffn_fwd. Returns (dx, dln_w, dln_b, dw1, db1, dwpos, dbpos, dw2, db2, dls); the
    parameter gradients go to the tensors of `grads` (same order, None = allocate; float32, overwritten)."""
    P, C = x.shape
    R = w1.shape[0]
    d = _ffn_desc(shape, C, R, eps)
    code = dtype_code(x)
    dev = x.device
    shapes = [(C,), (C,), (R, C), (R,), (R, 9), (R,), (C, R), (C,), (C,)]
    grads = list(grads) if grads is not None else [None] * 9
    outs = [g if g is not None else torch.empty(sh, device=dev, dtype=torch.float32) for g, sh in zip(grads, shapes)]
    dx = torch.empty_like(x)
    nbytes = lib.dfm_convffn_bwd_workspace_size(code, ctypes.byref(d))
    ws = _ws(nbytes, dev)
    check(lib.dfm_convffn_bwd(code, ctypes.byref(d), ptr(dout), ptr(x), ptr(h), ptr(xn), ptr(f), ptr(mean), ptr(rstd),
                              ptr(ln_w), ptr(ln_b), ptr(w1), ptr(wpos), ptr(bpos), ptr(w2), ptr(ls), ptr(rowscale),
                              ptr(dx), *[ptr(o) for o in outs], ptr(ws), nbytes, stream()), "dfm_convffn_bwd")
    if ACCOUNT is not None:
        es = _es(x)
        _acct_named([("residual", 0.0, 3.0 * es * P * C),
                     ("ffn_bwd", 6.0 * P * C * R + 36.0 * P * R, es * P * (2 * R + 2 * C) + 8 * P),
                     ("ffn_dhpre", 4.0 * P * C * R + 18.0 * P * R, es * P * (2 * R + C)),
                     ("dw3", 36.0 * P * R, es * P * 3 * R),
                     ("gemm", 2.0 * P * C * R, es * (P * R + P * C + R * C)),
                     ("gemm", 2.0 * P * C * R, es * (P * R + P * C + R * C)),
                     ("ln_bwd", 0.0, es * P * C * 4 + 8 * P)])
    return (dx, *outs)


# ---------------------------------------------------------------------------- depthwise conv
def dwconv(x, shape, w, bias, k, add_identity=False, out=None, gelu_out=None, out_gelu_grad=False):
    """x: [B*H*W, C] view (NHWC rows); w float32 [C,1,k,k] or [C,k,k]. gelu_out: also GELU(y);
    out_gelu_grad (with gelu_out): `out` receives GELU'(y) instead of y."""
    B, H, W = shape
    C = x.shape[1]
    if out is None:
        out = torch.empty(x.shape[0], C, device=x.device, dtype=x.dtype)
    flags = int(bool(add_identity)) | (2 if out_gelu_grad and gelu_out is not None else 0)
    check(lib.dfm_dwconv_fwd(dtype_code(x), B, H, W, C, k, ptr(x), ld(x), ptr(w), ptr(bias), flags,
                             ptr(out), ld(out), ptr(gelu_out), ld(gelu_out) if gelu_out is not None else 0,
                             stream()), "dfm_dwconv_fwd")
    if ACCOUNT is not None:
        _acct(2 * k * k * C * x.shape[0], x.shape[0] * C * _es(x) * (2 + (gelu_out is not None)))
    return out


def dwconv_bwd_data(dy, shape, w, k, add_identity=False, dx=None, accumulate=False):
    B, H, W = shape
    C = dy.shape[1]
    if dx is None:
        dx = torch.empty(dy.shape[0], C, device=dy.device, dtype=dy.dtype)
        accumulate = False
    check(lib.dfm_dwconv_bwd_data(dtype_code(dy), B, H, W, C, k, ptr(dy), ld(dy), ptr(w), int(add_identity),
                                  ptr(dx), ld(dx), int(accumulate), stream()), "dfm_dwconv_bwd_data")
    if ACCOUNT is not None:
        _acct(2 * k * k * C * dy.shape[0], dy.shape[0] * C * _es(dy) * (2 + bool(accumulate)))
    return dx


def dwconv_bwd(x, dy, shape, w, k, add_identity=False, dx=None, accumulate=False, dw=None, db=None):
    """Input gradient and weight / bias gradient of a 3x3 depthwise conv in one pass (dfm_dwconv_bwd)."""
    B, H, W = shape
    C = x.shape[1]
    if dx is None:
        dx = torch.empty(dy.shape[0], C, device=dy.device, dtype=dy.dtype)
        accumulate = False
    if dw is None:
        dw = torch.empty(C, 1, k, k, device=x.device, dtype=torch.float32)
    if db is None:
        db = torch.empty(C, device=x.device, dtype=torch.float32)
    ws, ps = _red_ws(lib.dfm_dwconv_bwd_weight_workspace(B, H, W, C, k), x.device)
    check(lib.dfm_dwconv_bwd(dtype_code(x), B, H, W, C, k, ptr(x), ld(x), ptr(dy), ld(dy), ptr(w), int(add_identity),
                             ptr(dx), ld(dx), int(accumulate), ptr(dw), ptr(db), ptr(ws), _pref(ps), stream()),
          "dfm_dwconv_bwd")
    if ACCOUNT is not None:
        _acct(4 * k * k * C * x.shape[0], x.shape[0] * C * _es(x) * (3 + bool(accumulate)))
    return dx, dw, db


def dwconv_bwd_weight(x, dy, shape, k, dw=None, db=None):
    B, H, W = shape
    C = x.shape[1]
    if dw is None:
        dw = torch.empty(C, 1, k, k, device=x.device, dtype=torch.float32)
    if db is None:
        db = torch.empty(C, device=x.device, dtype=torch.float32)
    ws, ps = _red_ws(lib.dfm_dwconv_bwd_weight_workspace(B, H, W, C, k), x.device)
    check(lib.dfm_dwconv_bwd_weight(dtype_code(x), B, H, W, C, k, ptr(x), ld(x), ptr(dy), ld(dy), ptr(dw), ptr(db),
                                    ptr(ws), _pref(ps), stream()), "dfm_dwconv_bwd_weight")
    if ACCOUNT is not None:
        _acct(2 * k * k * C * x.shape[0], x.shape[0] * C * _es(x) * 2)
    return dw, db


# -------------------------------------------------------------------------- reductions / misc
def colsum(x, mul=None, rowscale=None, rows_per_scale=1, out=None, accumulate=False):
    rows, C = x.shape
    if out is None:
        out = torch.empty(C, device=x.device, dtype=torch.float32)
        accumulate = False
    ws = _ws(lib.dfm_colsum_workspace(rows, C), x.device)
    check(lib.dfm_colsum(dtype_code(x), rows, C, ptr(x), ld(x), ptr(mul), ld(mul) if mul is not None else 0,
                         ptr(rowscale), rows_per_scale, ptr(out), int(accumulate), ptr(ws), stream()), "dfm_colsum")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * (1 + (mul is not None)))
    return out


def cast(x, dtype, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype)
    assert x.is_contiguous() and out.is_contiguous()
    check(lib.dfm_cast(dtype_code(x), dtype_code(out), x.numel(), ptr(x), ptr(out), stream()), "dfm_cast")
    if ACCOUNT is not None:
        _acct(0, x.numel() * (_es(x) + _es(out)))
    return out


def pack_slices(srcs, out):
    """out [..., n * cols] <- the n tensors [..., cols] side by side (converted to out.dtype), one launch."""
    n, cols = len(srcs), srcs[0].shape[-1]
    rows = srcs[0].numel() // cols
    assert out.is_contiguous() and out.shape[-1] == n * cols and out.numel() == rows * n * cols
    for t in srcs:
        assert t.is_contiguous() and t.shape[-1] == cols and t.numel() == rows * cols
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    dts = (ctypes.c_int * n)(*[dtype_code(t) for t in srcs])
    check(lib.dfm_pack_slices(dtype_code(out), n, ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(dts, ctypes.c_void_p),
                              rows, cols, ptr(out), stream()), "dfm_pack_slices")
    if ACCOUNT is not None:
        _acct(0, sum(t.numel() * _es(t) for t in srcs) + out.numel() * _es(out))
    return out


def gelu_bwd(dy, pre, out=None, accumulate=False):
    rows, C = dy.shape
    if out is None:
        out = torch.empty(rows, C, device=dy.device, dtype=dy.dtype)
        accumulate = False
    check(lib.dfm_gelu_bwd(dtype_code(dy), rows, C, ptr(dy), ld(dy), ptr(pre), ld(pre), ptr(out), ld(out),
                           int(accumulate), stream()), "dfm_gelu_bwd")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(dy) * (3 + bool(accumulate)))
    return out


def relu_bwd(dy, y, out=None):
    rows, C = dy.shape
    if out is None:
        out = torch.empty(rows, C, device=dy.device, dtype=dy.dtype)
    check(lib.dfm_relu_bwd(dtype_code(dy), rows, C, ptr(dy), ld(dy), ptr(y), ld(y), ptr(out), ld(out), stream()),
          "dfm_relu_bwd")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(dy) * 3)
    return out


def scale_mul(src, mul=None, colscale=None, rowscale=None, rows_per_scale=1, alpha=1.0, out=None, accumulate=False):
    rows, C = src.shape
    if out is None:
        out = torch.empty(rows, C, device=src.device, dtype=src.dtype)
        accumulate = False
    check(lib.dfm_scale_mul(dtype_code(src), rows, C, ptr(src), ld(src), ptr(mul), ld(mul) if mul is not None else 0,
                            ptr(colscale), ptr(rowscale), rows_per_scale, alpha, ptr(out), ld(out), int(accumulate),
                            stream()), "dfm_scale_mul")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(src) * (2 + (mul is not None) + bool(accumulate)))
    return out


def group_scale(x, scale, rows_per_group, out=None):
    """out[r, c] = x[r, c] * scale[r // rows_per_group, c] (float32 scale [groups, C]); out may be x."""
    rows, C = x.shape
    if out is None:
        out = torch.empty_like(x)
    assert scale.dtype == torch.float32 and scale.is_contiguous() and scale.numel() >= -(-rows // rows_per_group) * C
    check(lib.dfm_group_scale(dtype_code(x), rows, C, ptr(x), ld(x), ptr(scale), rows_per_group, ptr(out), ld(out),
                              stream()), "dfm_group_scale")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * 2)
    return out


def dual_mul(src, m1, m2, out1=None, out2=None):
    """(src * m1, src * m2) in one pass over src (the two gradients of an elementwise product)."""
    rows, C = src.shape
    if out1 is None:
        out1 = torch.empty(rows, C, device=src.device, dtype=src.dtype)
    if out2 is None:
        out2 = torch.empty(rows, C, device=src.device, dtype=src.dtype)
    check(lib.dfm_dual_mul(dtype_code(src), rows, C, ptr(src), ld(src), ptr(m1), ld(m1), ptr(m2), ld(m2), ptr(out1),
                           ld(out1), ptr(out2), ld(out2), stream()), "dfm_dual_mul")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(src) * 5)
    return out1, out2


# ---------------------------------------------------------------------- pool / bilinear / attn
def pool7(x, shape, out=None):
    B, H, W = shape
    C = x.shape[1]
    if out is None:
        out = torch.empty(B * 49, C, device=x.device, dtype=x.dtype)
    check(lib.dfm_adaptive_pool7_fwd(dtype_code(x), B, H, W, C, ptr(x), ld(x), ptr(out), ld(out), stream()),
          "dfm_adaptive_pool7_fwd")
    if ACCOUNT is not None:
        _acct(0, (B * H * W + B * 49) * C * _es(x))
    return out


def pool7_bwd(dy, shape, dx=None, accumulate=False):
    B, H, W = shape
    C = dy.shape[1]
    if dx is None:
        dx = torch.empty(B * H * W, C, device=dy.device, dtype=dy.dtype)
        accumulate = False
    check(lib.dfm_adaptive_pool7_bwd(dtype_code(dy), B, H, W, C, ptr(dy), ld(dy), ptr(dx), ld(dx), int(accumulate),
                                     stream()), "dfm_adaptive_pool7_bwd")
    if ACCOUNT is not None:
        _acct(0, (B * H * W * (1 + bool(accumulate)) + B * 49) * C * _es(dy))
    return dx


def bilinear(x, in_hw, out_hw, B, out=None, accumulate=False):
    (Hi, Wi), (Ho, Wo) = in_hw, out_hw
    C = x.shape[1]
    if out is None:
        out = torch.empty(B * Ho * Wo, C, device=x.device, dtype=x.dtype)
        accumulate = False
    check(lib.dfm_bilinear_fwd(dtype_code(x), B, Hi, Wi, Ho, Wo, C, ptr(x), ld(x), ptr(out), ld(out),
                               int(accumulate), stream()), "dfm_bilinear_fwd")
    if ACCOUNT is not None:
        _acct(0, (B * Hi * Wi + B * Ho * Wo * (1 + bool(accumulate))) * C * _es(x))
    return out


def bilinear_bwd(dy, in_hw, out_hw, B, dx=None, accumulate=False):
    (Hi, Wi), (Ho, Wo) = in_hw, out_hw
    C = dy.shape[1]
    if dx is None:
        dx = torch.empty(B * Hi * Wi, C, device=dy.device, dtype=dy.dtype)
        accumulate = False
    check(lib.dfm_bilinear_bwd(dtype_code(dy), B, Hi, Wi, Ho, Wo, C, ptr(dy), ld(dy), ptr(dx), ld(dx),
                               int(accumulate), stream()), "dfm_bilinear_bwd")
    if ACCOUNT is not None:
        _acct(0, (B * Hi * Wi * (1 + bool(accumulate)) + B * Ho * Wo) * C * _es(dy))
    return dx


def pooled_attn(q, k, v, B, heads, N, dh, scale, out=None):
    """q: [B*49, >=heads*dh] view, k/v: [B*N, ...] views (head h at cols h*dh)."""
    if out is None:
        out = torch.empty(B * 49, heads * dh, device=q.device, dtype=q.dtype)
    lse = torch.empty(B * heads * 49, device=q.device, dtype=torch.float32)
    ws = _ws(lib.dfm_pooled_attn_workspace(B, heads, N, dh), q.device)
    assert ld(k) == ld(v)
    check(lib.dfm_pooled_attn_fwd(dtype_code(q), B, heads, N, dh, ptr(q), ld(q), ptr(k), ptr(v), ld(k), scale,
                                  ptr(out), ld(out), ptr(lse), ptr(ws), stream()), "dfm_pooled_attn_fwd")
    if ACCOUNT is not None:
        _acct(4.0 * B * heads * 49 * N * dh, _es(q) * (2 * B * 49 * heads * dh + 2 * B * N * heads * dh))
    return out, lse


def pooled_attn_bwd(q, k, v, o, dout, lse, B, heads, N, dh, scale, dq, dk, dv):
    ws = _ws(lib.dfm_pooled_attn_workspace(B, heads, N, dh), q.device)
    assert ld(dk) == ld(dv) and ld(dq) == ld(q)
    check(lib.dfm_pooled_attn_bwd(dtype_code(q), B, heads, N, dh, ptr(q), ld(q), ptr(k), ptr(v), ld(k), scale,
                                  ptr(o), ld(o), ptr(dout), ld(dout), ptr(lse), ptr(dq), ptr(dk), ptr(dv), ld(dk),
                                  ptr(ws), stream()), "dfm_pooled_attn_bwd")
    if ACCOUNT is not None:
        hd = heads * dh
        _acct(10.0 * B * heads * 49 * N * dh, _es(q) * (4 * B * 49 * hd + 4 * B * N * hd))


# ---------------------------------------------------------------------------------- BatchNorm
def bn_stats(x):
    """float32 [3, C]: (sum (x-K), sum (x-K)^2, K) with the per-column shift K = x[0]."""
    rows, C = x.shape
    st = torch.empty(3, C, device=x.device, dtype=torch.float32)
    ws = _ws(lib.dfm_bn_workspace(rows, C), x.device)
    check(lib.dfm_bn_stats(dtype_code(x), rows, C, ptr(x), ld(x), ptr(st), ptr(ws), stream()), "dfm_bn_stats")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x))
    return st


def bn_finalize(stats, count, eps, momentum, running_mean=None, running_var=None):
    C = stats.shape[1]
    mean = torch.empty(C, device=stats.device, dtype=torch.float32)
    rstd = torch.empty(C, device=stats.device, dtype=torch.float32)
    check(lib.dfm_bn_finalize(C, ptr(stats), float(count), eps, momentum, ptr(mean), ptr(rstd), ptr(running_mean),
                              ptr(running_var), stream()), "dfm_bn_finalize")
    if ACCOUNT is not None:
        _acct(0, C * 4 * (3 + 4 * (running_mean is not None)))
    return mean, rstd


def bn_merge(parts, counts):
    """SyncBN: all-gathered per-rank bn_stats triples [S, 3, C] + per-rank rows [S] (float32) -> the
    union's triple [3, C], shifted by rank 0's K (fixed order; identity for S = 1)."""
    S, three, C = parts.shape
    if three != 3 or counts.shape != (S,) or parts.dtype != torch.float32 or counts.dtype != torch.float32:
        raise ValueError(f"bn_merge: parts {tuple(parts.shape)} {parts.dtype}, counts {tuple(counts.shape)}")
    parts, counts = parts.contiguous(), counts.contiguous()
    st = torch.empty(3, C, device=parts.device, dtype=torch.float32)
    check(lib.dfm_bn_merge(S, C, ptr(parts), ptr(counts), ptr(st), stream()), "dfm_bn_merge")
    return st


def bn_apply(x, mean, rstd, gamma, beta, res=None, act=0, out=None):
    rows, C = x.shape
    if out is None:
        out = torch.empty(rows, C, device=x.device, dtype=x.dtype)
    check(lib.dfm_bn_apply(dtype_code(x), rows, C, ptr(x), ld(x), ptr(mean), ptr(rstd), ptr(gamma), ptr(beta),
                           ptr(res), ld(res) if res is not None else 0, act, ptr(out), ld(out), stream()),
          "dfm_bn_apply")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * (2 + (res is not None)))
    return out


def bn_bwd_stats(x, dy, mean, rstd, out=None):
    rows, C = x.shape
    st = torch.empty(2, C, device=x.device, dtype=torch.float32) if out is None else out
    ws = _ws(lib.dfm_bn_workspace(rows, C), x.device)
    check(lib.dfm_bn_bwd_stats(dtype_code(x), rows, C, ptr(x), ld(x), ptr(dy), ld(dy), ptr(mean), ptr(rstd),
                               ptr(st), ptr(ws), stream()), "dfm_bn_bwd_stats")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * 2)
    return st


def bn_bwd_apply(x, dy, mean, rstd, gamma, stats2, count, dx=None, accumulate=False):
    rows, C = x.shape
    if dx is None:
        dx = torch.empty(rows, C, device=x.device, dtype=x.dtype)
        accumulate = False
    check(lib.dfm_bn_bwd_apply(dtype_code(x), rows, C, ptr(x), ld(x), ptr(dy), ld(dy), ptr(mean), ptr(rstd),
                               ptr(gamma), ptr(stats2), float(count), ptr(dx), ld(dx), int(accumulate), stream()),
          "dfm_bn_bwd_apply")
    if ACCOUNT is not None:
        _acct(0, rows * C * _es(x) * (3 + bool(accumulate)))
    return dx


# ------------------------------------------------------------------- dense 3x3 stride-2 conv
def conv3s2_kp(cin):
    """Packed K (columns of the gathered operand): 9*cin rounded up to a multiple of 8."""
    return (9 * cin + 7) // 8 * 8


def conv3s2_im2col(x, dtype, bn=None, gelu=False, out=None):
    """Gather of nn.Conv2d(cin, cout, 3, 2, 1)'s operand from an NCHW-logical tensor x (any strides),
    with an optional folded BatchNorm affine bn = (mean, rstd, gamma, beta) and exact GELU.
    Returns cols [B*Ho*Wo, Kp] in `dtype` (columns (kh, kw, c))."""
    B, C, H, W = x.shape
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    kp = conv3s2_kp(C)
    if out is None:
        out = torch.empty(B * Ho * Wo, kp, device=x.device, dtype=dtype)
    mean, rstd, gamma, beta = bn if bn is not None else (None,) * 4
    sb, sc, sh, sw = x.stride()
    check(lib.dfm_conv3s2_im2col(dtype_code(x), dtype_code(out), B, H, W, C, sb, sc, sh, sw, ptr(x), ptr(mean),
                                 ptr(rstd), ptr(gamma), ptr(beta), int(gelu), kp, ptr(out), stream()),
          "dfm_conv3s2_im2col")
    if ACCOUNT is not None:
        _acct(0, B * C * H * W * _es(x) + out.numel() * _es(out))
    return out


def conv3s2_col2im(dcols, shape, cin, x=None, bn=None, gelu=False, dx=None, accumulate=False):
    """Backward of conv3s2_im2col w.r.t. the BN output (rows [B*H*W, cin]); x: the rows the gather
    read (needed with gelu, to recompute GELU' of the folded BN output)."""
    B, H, W = shape
    if dx is None:
        dx = torch.empty(B * H * W, cin, device=dcols.device, dtype=dcols.dtype)
        accumulate = False
    mean, rstd, gamma, beta = bn if bn is not None else (None,) * 4
    check(lib.dfm_conv3s2_col2im(dtype_code(dcols), B, H, W, cin, ptr(dcols), ld(dcols), ptr(x),
                                 ld(x) if x is not None else 0, ptr(mean), ptr(rstd), ptr(gamma), ptr(beta),
                                 int(gelu), ptr(dx), ld(dx), int(accumulate), stream()), "dfm_conv3s2_col2im")
    if ACCOUNT is not None:
        _acct(0, dcols.shape[0] * 9 * cin * _es(dcols) + dx.numel() * _es(dx) * (1 + bool(accumulate) + bool(gelu)))
    return dx


def conv3s2_col2im_nchw(dcols, shape, cin, dtype):
    """Input gradient of a conv with no folded BN: contiguous NCHW [B, cin, H, W] in `dtype`."""
    B, H, W = shape
    dx = torch.empty(B, cin, H, W, device=dcols.device, dtype=dtype)
    sb, sc, sh, sw = dx.stride()
    check(lib.dfm_conv3s2_col2im_nchw(dtype_code(dcols), dtype_code(dx), B, H, W, cin, ptr(dcols), ld(dcols),
                                      ptr(dx), sb, sc, sh, sw, stream()), "dfm_conv3s2_col2im_nchw")
    if ACCOUNT is not None:
        _acct(0, dcols.shape[0] * 9 * cin * _es(dcols) + dx.numel() * _es(dx))
    return dx


def conv3_weight_pack(w, dtype, kp):
    cout, cin = w.shape[:2]
    out = torch.empty(cout, kp, device=w.device, dtype=dtype)
    check(lib.dfm_conv3_weight_pack(dtype_code(out), cout, cin, kp, ptr(w), ptr(out), stream()),
          "dfm_conv3_weight_pack")
    if ACCOUNT is not None:
        _acct(0, w.numel() * 4 + out.numel() * _es(out))
    return out


def conv3_weight_unpack(dwp, cin, dw=None, accumulate=False):
    cout, kp = dwp.shape
    if dw is None:
        dw = torch.empty(cout, cin, 3, 3, device=dwp.device, dtype=torch.float32)
        accumulate = False
    check(lib.dfm_conv3_weight_unpack(cout, cin, kp, ptr(dwp), ptr(dw), int(accumulate), stream()),
          "dfm_conv3_weight_unpack")
    if ACCOUNT is not None:
        _acct(0, dwp.numel() * 4 + dw.numel() * 4)
    return dw


# ------------------------------------------------------------------ multi-scale + flip eval
def resize_nchw(x, size, align_corners, flip=False, dtype=torch.float32):
    """F.interpolate(x, size, 'bilinear', align_corners) [then torch.flip(dims=(3,))], x any strides."""
    B, C, Hi, Wi = x.shape
    Ho, Wo = size
    y = torch.empty(B, C, Ho, Wo, device=x.device, dtype=dtype)
    sb, sc, sh, sw = x.stride()
    check(lib.dfm_resize_nchw(dtype_code(x), dtype_code(y), B, C, Hi, Wi, sb, sc, sh, sw, ptr(x), Ho, Wo,
                              int(align_corners), int(flip), ptr(y), stream()), "dfm_resize_nchw")
    return y


def msf_accumulate(low_rows, B, h, w, ncls, scaled_hw, out_hw, flip, acc):
    """acc [B*H*W, ncls] float32 += softmax(resize_ac(flip?(upsample(low -> scaled_hw))))."""
    (Hs, Ws), (H, W) = scaled_hw, out_hw
    check(lib.dfm_msf_accumulate(dtype_code(low_rows), B, h, w, ncls, ptr(low_rows), ld(low_rows), Hs, Ws, H, W,
                                 int(flip), ptr(acc), stream()), "dfm_msf_accumulate")
    return acc


def seg_confusion(acc, label, ncls, ignore, hist):
    """hist [ncls*ncls] int64 += bincount(label*ncls + argmax(acc rows)) over label != ignore."""
    assert label.dtype == torch.int64 and hist.dtype == torch.int64 and acc.is_contiguous()
    assert label.is_contiguous()
    if acc.dim() != 2 or acc.shape[1] != ncls or acc.shape[0] != label.numel():
        raise ValueError(f"seg_confusion: scores {tuple(acc.shape)} do not match {label.numel()} labels x {ncls}")
    check(lib.dfm_seg_confusion(label.numel(), ncls, ptr(acc), ptr(label), ignore, ptr(hist), stream()),
          "dfm_seg_confusion")
    return hist


# ---------------------------------------------------------------------------------------- NMF
def _copy_dtype(flag):
    """bf16_copy argument: False / None (no copy), True (bf16) or a 16-bit torch dtype."""
    if not flag:
        return None
    return torch.bfloat16 if flag is True else flag


def nmf_update(a, num, den, eps=1e-6, out=None, bf16_copy=False):
    """out = a * num / (den + eps) (float32); with bf16_copy (True = bf16, or a 16-bit dtype) also
    returns a 16-bit copy of out."""
    if out is None:
        out = torch.empty_like(a)
    cdt = _copy_dtype(bf16_copy)
    o16 = torch.empty(a.shape, device=a.device, dtype=cdt) if cdt is not None else None
    check(lib.dfm_nmf_update(a.numel(), ptr(a), ptr(num), ptr(den), eps, ptr(out), ptr(o16),
                             dtype_code(o16) if o16 is not None else 0, stream()), "dfm_nmf_update")
    if ACCOUNT is not None:
        _acct(0, a.numel() * (16 + 2 * bool(bf16_copy)))
    return (out, o16) if bf16_copy else out


def nmf_update_bwd(g, a, num, den, out, ga=None, accumulate=False, eps=1e-6, bf16_copy=False):
    """-> ga, gnum, gden (float32) [, bf16 copy of gnum]."""
    if ga is None:
        ga = torch.empty_like(a)
        accumulate = False
    gnum = torch.empty_like(a)
    gden = torch.empty_like(a)
    cdt = _copy_dtype(bf16_copy)
    g16 = torch.empty(a.shape, device=a.device, dtype=cdt) if cdt is not None else None
    check(lib.dfm_nmf_update_bwd(a.numel(), ptr(g), ptr(a), ptr(num), ptr(den), ptr(out), eps, ptr(ga),
                                 int(accumulate), ptr(gnum), ptr(gden), ptr(g16),
                                 dtype_code(g16) if g16 is not None else 0, stream()), "dfm_nmf_update_bwd")
    if ACCOUNT is not None:
        _acct(0, a.numel() * (4 * (8 + bool(accumulate)) + 2 * bool(bf16_copy)))
    return (ga, gnum, gden, g16) if bf16_copy else (ga, gnum, gden)


def nmf_update_mm(a, num, M, eps=1e-6, bf16_copy=False):
    """Batched [B, rows, 64] update with its denominator product fused: den = a M, out = a * num /
    (den + eps). Returns (out, den[, 16-bit copy of out])."""
    Bb, rows, R = a.shape
    out, den = torch.empty_like(a), torch.empty_like(a)
    cdt = _copy_dtype(bf16_copy)
    o16 = torch.empty(a.shape, device=a.device, dtype=cdt) if cdt is not None else None
    check(lib.dfm_nmf_update_mm(Bb, rows, R, ptr(a), ptr(num), ptr(M), eps, ptr(den), ptr(out), ptr(o16),
                                dtype_code(o16) if o16 is not None else 0, stream()), "dfm_nmf_update_mm")
    if ACCOUNT is not None:
        _acct(2.0 * a.numel() * R, a.numel() * (16 + 2 * bool(bf16_copy)) + M.numel() * 4)
    return (out, den, o16) if bf16_copy else (out, den)


def nmf_update_bwd_mm(g, a, num, den, out, A2=None, S=None, Mg=None, eps=1e-6, bf16_copy=False):
    """Backward of nmf_update_mm with g' = g + A2 (S + S^T) and ga = g' num / (den+eps) + gden Mg.
    Returns (ga, gnum, gden[, 16-bit copy of gnum])."""
    Bb, rows, R = a.shape
    ga, gnum, gden = torch.empty_like(a), torch.empty_like(a), torch.empty_like(a)
    cdt = _copy_dtype(bf16_copy)
    g16 = torch.empty(a.shape, device=a.device, dtype=cdt) if cdt is not None else None
    check(lib.dfm_nmf_update_bwd_mm(Bb, rows, R, ptr(g), ptr(A2), ptr(S), ptr(a), ptr(num), ptr(den), ptr(out), eps,
                                    ptr(Mg), ptr(ga), 0, ptr(gnum), ptr(gden), ptr(g16),
                                    dtype_code(g16) if g16 is not None else 0, stream()), "dfm_nmf_update_bwd_mm")
    if ACCOUNT is not None:
        _acct(2.0 * a.numel() * R * ((A2 is not None) + (Mg is not None)),
              a.numel() * (4 * (8 + (A2 is not None)) + 2 * bool(bf16_copy)))
    return (ga, gnum, gden, g16) if bf16_copy else (ga, gnum, gden)


def nmf_fwd(x, bases, steps, eps=1e-6, keep=False):
    """NMF2D forward in one library call (dfm_nmf_fwd): x [B, N, D], bases [B, D, 64] float32 -> y
    [B, N, D]; keep=True also returns the saved factors for nmf_bwd (a uint8 buffer)."""
    Bb, N, D = x.shape
    R = bases.shape[2]
    assert x.is_contiguous() and bases.is_contiguous() and bases.dtype == torch.float32
    dt = dtype_code(x)
    nbytes = lib.dfm_nmf_fwd_workspace_size(dt, Bb, N, D, R, steps)
    assert nbytes > 0, "dfm_nmf_fwd: unsupported shape / rank"
    saved = None
    if keep:
        sb = lib.dfm_nmf_saved_size(dt, Bb, N, D, R, steps)
        saved = torch.empty(sb, device=x.device, dtype=torch.uint8)
    ws = _ws(nbytes, x.device)
    y = torch.empty_like(x)
    check(lib.dfm_nmf_fwd(dt, Bb, N, D, R, steps, eps, ptr(x), ptr(bases), ptr(y), ptr(saved),
                          saved.numel() if keep else 0, ptr(ws), nbytes, stream()), "dfm_nmf_fwd")
    return (y, saved) if keep else y


def nmf_bwd(x, bases, saved, gy, steps, eps=1e-6):
    """Gradient of nmf_fwd's y w.r.t. x (dfm_nmf_bwd) from the factors nmf_fwd(keep=True) saved."""
    Bb, N, D = x.shape
    R = bases.shape[2]
    assert gy.is_contiguous() and gy.dtype == x.dtype
    dt = dtype_code(x)
    nbytes = lib.dfm_nmf_bwd_workspace_size(dt, Bb, N, D, R, steps)
    ws = _ws(nbytes, x.device)
    gx = torch.empty_like(x)
    check(lib.dfm_nmf_bwd(dt, Bb, N, D, R, steps, eps, ptr(x), ptr(bases), ptr(saved), saved.numel(), ptr(gy),
                          ptr(gx), ptr(ws), nbytes, stream()), "dfm_nmf_bwd")
    return gx


def softmax_rows(x):
    y = torch.empty_like(x)
    check(lib.dfm_softmax_rows(x.numel() // x.shape[-1], x.shape[-1], ptr(x), ptr(y), stream()), "dfm_softmax_rows")
    if ACCOUNT is not None:
        _acct(0, x.numel() * 8)
    return y


def softmax_rows_bwd(y, dy, dx=None, accumulate=False):
    if dx is None:
        dx = torch.empty_like(y)
        accumulate = False
    check(lib.dfm_softmax_rows_bwd(y.numel() // y.shape[-1], y.shape[-1], ptr(y), ptr(dy), ptr(dx), int(accumulate),
                                   stream()), "dfm_softmax_rows_bwd")
    if ACCOUNT is not None:
        _acct(0, y.numel() * 4 * (3 + bool(accumulate)))
    return dx


# --------------------------------------------------------------------------------------- loss
def seg_loss_fwd(logits, B, h, w, ncls, label, ignore=255):
    H, W = label.shape[-2:]
    out = torch.empty(2, device=logits.device, dtype=torch.float32)
    ws = _ws(lib.dfm_seg_loss_workspace(B, H, W), logits.device)
    check(lib.dfm_seg_loss_fwd(dtype_code(logits), B, h, w, ncls, ptr(logits), H, W, ptr(label), ignore, None,
                               ptr(out), ptr(ws), stream()), "dfm_seg_loss_fwd")
    if ACCOUNT is not None:
        _acct(0, logits.numel() * _es(logits) + label.numel() * 8)
    return out


def seg_loss_bwd(logits, B, h, w, ncls, label, loss_out, gscale=None, ignore=255):
    H, W = label.shape[-2:]
    dl = torch.empty(B * h * w, ncls, device=logits.device, dtype=torch.float32)
    ws = _ws(lib.dfm_seg_loss_bwd_workspace(B, h, w, ncls, H, W), logits.device)
    check(lib.dfm_seg_loss_bwd(dtype_code(logits), B, h, w, ncls, ptr(logits), H, W, ptr(label), ignore, None,
                               ptr(loss_out), ptr(gscale), ptr(dl), ptr(ws), stream()), "dfm_seg_loss_bwd")
    if ACCOUNT is not None:
        _acct(0, logits.numel() * (_es(logits) + 4) + label.numel() * 8)
    return dl


def seg_loss_grad_partials_size(B, h, w, ncls, H, W):
    return lib.dfm_seg_loss_grad_partials_size(B, h, w, ncls, H, W)


def seg_loss_fwd_grad(logits, B, h, w, ncls, label, ignore=255):
    """Training loss + its gradient's unscaled per-tile partials in one pass -> (loss_out, partials)."""
    H, W = label.shape[-2:]
    out = torch.empty(2, device=logits.device, dtype=torch.float32)
    nb = seg_loss_grad_partials_size(B, h, w, ncls, H, W)
    part = torch.empty(nb // 4, device=logits.device, dtype=torch.float32)
    check(lib.dfm_seg_loss_fwd_grad(dtype_code(logits), B, h, w, ncls, ptr(logits), H, W, ptr(label), ignore,
                                    ptr(out), ptr(part), stream()), "dfm_seg_loss_fwd_grad")
    if ACCOUNT is not None:
        _acct(0, logits.numel() * _es(logits) + label.numel() * 8)
    return out, part


def seg_loss_bwd_gather(part, B, h, w, ncls, loss_out, gscale, dtype):
    dl = torch.empty(B * h * w, ncls, device=part.device, dtype=dtype)
    check(lib.dfm_seg_loss_bwd_gather(dtype_code(dl), B, h, w, ncls, ptr(part), ptr(loss_out), ptr(gscale), ptr(dl),
                                      stream()), "dfm_seg_loss_bwd_gather")
    if ACCOUNT is not None:
        _acct(0, dl.numel() * _es(dl))
    return dl


# -------------------------------------------------------------------------------------- AdamW
def loss_scale_update(amp, flag, growth, backoff, interval):
    check(lib.dfm_loss_scale_update(ptr(amp), ptr(flag), growth, backoff, interval, stream()),
          "dfm_loss_scale_update")


def grad_nonfinite(g, flag):
    """flag (int32 [1], zeroed by the caller) := 1 if any element of g is inf / nan."""
    check(lib.dfm_grad_nonfinite(g.numel(), ptr(g), ptr(flag), stream()), "dfm_grad_nonfinite")
    return flag


def adamw(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0, bf16_copy=None, hyper=None,
          amp=None, flag=None):
    """AdamW step; with `hyper` (device float32 [lr, step]) lr and step are read on the device
    (lr / step arguments ignored) so the launch can live in a replayed HIP graph. With the loss
    scaler's device state `amp` and overflow `flag` the step is skipped / unscaled on the device."""
    cdt = dtype_code(bf16_copy) if bf16_copy is not None else 0
    if amp is not None:
        check(lib.dfm_adamw_amp(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(hyper), ptr(amp), ptr(flag), beta1,
                                beta2, eps, weight_decay, grad_scale, ptr(bf16_copy), cdt, stream()), "dfm_adamw_amp")
    elif hyper is not None:
        check(lib.dfm_adamw_dev(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), ptr(hyper), beta1, beta2, eps,
                                weight_decay, grad_scale, ptr(bf16_copy), cdt, stream()), "dfm_adamw_dev")
    else:
        check(lib.dfm_adamw(p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), lr, beta1, beta2, eps, weight_decay, step,
                            grad_scale, ptr(bf16_copy), cdt, stream()), "dfm_adamw")
    if ACCOUNT is not None:
        _acct(0, p.numel() * (28 + (2 if bf16_copy is not None else 0)))
