"""autograd.Functions of DFormer's encoder Block with hand-written backward passes.

Every tensor op inside these Functions is a libdformer_hip.so kernel (dformer_amd.kernels);
torch provides allocation, views and the autograd tape only. Activations are NHWC rows [P, C]
in the compute dtype (float32 for parity runs, bfloat16 for training); parameters and their
gradients are float32 (GEMM operands use cached compute-dtype copies of the weights).

Reference semantics (file:line in Originofamonia/DFormer):
  ConvFFNFn     MLP.forward + Block residual/layer-scale/DropPath   DFormer.py:48-67, 173-179
  AttentionFn   Attention.forward + Block residuals                 DFormer.py:70-145, 168-179
"""
import os
import weakref

import torch

from . import kernels as K

# ---------------------------------------------------------------- compute-dtype weight cache
_EPOCH = [0]
_WCACHE = {}


def invalidate_weights():
    """Call after parameters change outside dformer_amd's optimizer (load_state_dict, manual edits)."""
    _EPOCH[0] += 1
    _WCACHE.clear()


def register_shadow(p, shadow):
    """The fused optimizer keeps `shadow` (bf16 copy of p) up to date itself."""
    _WCACHE[(id(p), shadow.dtype)] = (_EPOCH[0], shadow, (p.data_ptr(),), (weakref.ref(p),))


def _adjacent_rows(ts):
    """One [sum of rows, cols] view over 2-D tensors that lie back to back in one storage (the
    optimizer's flat buffers place q | q_cut | l and proj | proj_e so), or None."""
    t0 = ts[0]
    cols = t0.shape[1]
    off = t0.storage_offset()
    for t in ts:
        if (t.dim() != 2 or t.shape[1] != cols or not t.is_contiguous() or t.dtype != t0.dtype or
                t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or t.storage_offset() != off):
            return None
        off += t.numel()
    rows = sum(t.shape[0] for t in ts)
    return t0.new_empty(0).set_(t0.untyped_storage(), t0.storage_offset(), (rows, cols))


def wcast(dtype, *params):
    """Compute-dtype 2-D copy of one parameter (or the row-concatenation of several), cached per epoch.
    Parameters re-homed by FusedAdamW are views of its flat buffers: the concatenation of adjacent
    ones is a view of the flat compute-dtype shadow (no per-step copy)."""
    if dtype == torch.float32 and len(params) == 1:
        p = params[0].detach()
        return p if p.dim() == 2 else p.reshape(p.shape[0], -1)
    key = tuple(id(p) for p in params) + (dtype,)
    ptrs = tuple(p.data_ptr() for p in params)
    hit = _WCACHE.get(key)
    # valid while the same parameter objects are alive (a new tensor may reuse a freed one's id() and
    # address) at the same addresses, in the same epoch
    if (hit is not None and hit[0] == _EPOCH[0] and hit[2] == ptrs and
            all(r() is p for r, p in zip(hit[3], params))):
        return hit[1]
    w = None
    if len(params) > 1:
        parts = [wcast(dtype, p) for p in params]
        w = _adjacent_rows(parts)
    if w is None:
        src = params[0].detach().reshape(params[0].shape[0], -1) if len(params) == 1 else \
            torch.cat([p.detach().reshape(p.shape[0], -1) for p in params], 0)
        src = src.contiguous()
        w = src if dtype == torch.float32 else K.cast(src, dtype)
    _WCACHE[key] = (_EPOCH[0], w, ptrs, tuple(weakref.ref(p) for p in params))
    return w


_GSLOT = {}


def register_grad_slot(p, flat, offset):
    """Weight gradients of `p` are written straight into flat[offset:offset+numel] (the optimizer's
    flat gradient buffer); autograd then adopts that view as p.grad without a copy. The entry holds
    a weak reference so a recycled id() of a dead parameter never aliases a live slot."""
    _GSLOT[id(p)] = (flat, offset, tuple(p.shape), weakref.ref(p))


def clear_grad_slots():
    _GSLOT.clear()


def _slot(p):
    s = _GSLOT.get(id(p))
    if s is None or s[3]() is not p:
        return None
    return s


def has_grad_slot(p):
    """True while `p` belongs to a live FusedAdamW flat group (its gradients go to a flat slot)."""
    return _slot(p) is not None


def gslot(p):
    s = _slot(p)
    if s is None:
        return None
    flat, off, shape, _ = s
    n = 1
    for d in shape:
        n *= d
    return flat[off:off + n].view(shape)


def gslot2(p):
    t = gslot(p)
    return None if t is None else t.view(t.shape[0], -1)


def gslot_rows(*ps):
    """One [sum of rows, cols] view over the flat-gradient slots of parameters whose slots are
    adjacent in that order (e.g. proj.weight, proj_e.weight), or None."""
    ss = [_slot(p) for p in ps]
    if any(s is None for s in ss) or any(s[0] is not ss[0][0] for s in ss):
        return None
    cols = ss[0][2][1:] if len(ss[0][2]) > 1 else ()
    off = ss[0][1]
    rows = 0
    for s in ss:
        if s[1] != off or tuple(s[2][1:]) != tuple(cols):
            return None
        n = 1
        for d in s[2]:
            n *= d
        off += n
        rows += s[2][0]
    return ss[0][0][ss[0][1]:off].view(rows, *cols) if cols else ss[0][0][ss[0][1]:off]


# The grouped weight gradients (and deferred reduction second stages) of every Block backward -- the
# attention's and both ConvFFNs' -- are issued on a stream of their own, after that stream waits for
# the block's data gradients: nothing downstream reads them before the optimizer (join_streams), so the
# next block's backward no longer waits for them. Measured (alternating runs): 492.2-495.9 vs
# 499.1-501.9 images/s; the ConvFFNs' groups alone (490.6 / 492.2) or the attention's alone (486.5 /
# 488.1) were slower. Groups under kernels.WG_STREAM_MIN_FLOPS stay on the current stream.
_WG_STREAM = {}


def _wg_stream(dev):
    st = _WG_STREAM.get(dev)
    if st is None:
        st = _WG_STREAM[dev] = torch.cuda.Stream(device=dev)
        register_side_stream(st)
    return st


def wgrad_group(dev=None):
    """The weight-gradient queue of one Block backward (kernels.wgrad_group), flushed on the
    weight-gradient stream for CUDA tensors."""
    if dev is not None and dev.type == "cuda":
        return K.wgrad_group(stream=_wg_stream(dev))
    return K.wgrad_group()


_SIDE_STREAMS = []


def register_side_stream(s):
    """Streams besides the step's own on which this package issues gradient-writing kernels (the
    encoder's RGB ConvFFN stream, the attention-backward and weight-gradient streams)."""
    if all(s is not t for t in _SIDE_STREAMS):
        _SIDE_STREAMS.append(s)


def join_streams(main=None):
    """The current stream waits for everything issued so far on `main` (the stream the step's
    backward was started from) and on every side stream of this package, so a collective enqueued
    next sees every gradient slot complete whichever stream autograd ran its last hook on."""
    streams = ([main] if main is not None else []) + _SIDE_STREAMS
    if not streams:  # CPU tensors / nothing issued off the current stream
        return
    cur = torch.cuda.current_stream()
    for s in streams:
        if s is not None and s.device == cur.device and s != cur:
            cur.wait_stream(s)


def _cat1(*vs):
    """Concatenate float32 vectors (bias concat for fused GEMMs); cached like weights (a view when
    the vectors are adjacent in the optimizer's flat buffer)."""
    key = tuple(id(v) for v in vs) + ("bias",)
    ptrs = tuple(v.data_ptr() for v in vs)
    hit = _WCACHE.get(key)
    if (hit is not None and hit[0] == _EPOCH[0] and hit[2] == ptrs and
            all(r() is v for r, v in zip(hit[3], vs))):
        return hit[1]
    out = _adjacent_rows([v.detach().view(-1, 1) for v in vs])
    out = out.view(-1) if out is not None else torch.cat([v.detach() for v in vs])
    _WCACHE[key] = (_EPOCH[0], out, ptrs, tuple(weakref.ref(v) for v in vs))
    return out


# ====================================================================== ConvFFN (+ residual)
# FUSED_FFN: True runs bf16 / fp16 ConvFFNs whose shape has fused kernels through dfm_convffn_fwd / _bwd
# (csrc/convffn.hip); "fwd" runs only the forward fused (it also stores GELU(hpre) / GELU'(hpre)) and the
# op-level backward; "auto" does that on planes of >= FUSED_FWD_MIN_PLANE pixels (stage 0 at 480 x 640,
# where the fused forward wins: 431 vs 526 us at 512 hidden channels, 210 vs 229 at 256; it loses from
# stage 1 on, tools/ffn_kernels_bench.py); False routes every ConvFFN through the op-level chain below
# (tests compare them; DFM_FUSED_FFN=0|1|fwd|auto sets the default for A/B runs)
FUSED_FWD_MIN_PLANE = 16384
_FUSED_FFN_MODES = {"0": False, "1": True, "fwd": "fwd", "auto": "auto"}


def _fused_ffn_mode(v):
    if v not in _FUSED_FFN_MODES:
        raise ValueError(f"DFM_FUSED_FFN={v!r}: expected one of {sorted(_FUSED_FFN_MODES)}")
    return _FUSED_FFN_MODES[v]


FUSED_FFN = _fused_ffn_mode(os.environ.get("DFM_FUSED_FFN", "auto"))


class ConvFFNFn(torch.autograd.Function):
    """out = x + rowscale * ls * fc2(GELU(DW3x3(h) + h)),  h = fc1(LN(x))   on [P, C] rows.

    forward: LN, GEMM fc1(+bias), DW3x3(+bias+identity) writing GELU'(hpre) and GELU(hpre) from one
    erf evaluation, GEMM fc2(+bias, preact f, residual/layer-scale/DropPath epilogue).
    backward: residual chain rule, fc2 input gradient times the stored GELU', the DW3x3 input and
    weight gradients in one pass, fc1 input gradient, LN backward; the fc2 / fc1 weight gradients
    as one grouped launch at the end."""

    @staticmethod
    def forward(ctx, x, shape, rowscale, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls):
        B, H, W = shape
        P, C = x.shape
        dt = x.dtype
        W1, W2 = wcast(dt, w1), wcast(dt, w2)
        ctx.tag = K.TAG
        fused = bool(FUSED_FFN) and K.convffn_supported(dt, shape, C, w1.shape[0])
        if FUSED_FFN == "auto":
            fused = fused and shape[1] * shape[2] >= FUSED_FWD_MIN_PLANE
        ctx.fused = fused and FUSED_FFN is True
        ctx.shape = shape
        if ctx.fused:  # one kernel: LN, fc1, DW3x3 + identity, GELU, fc2, residual; h is the saved hidden
            out, f, h, xn, mu, rs = K.convffn_fwd(x, shape, ln_w, ln_b, W1, b1, wpos, bpos, W2, b2, ls, rowscale)
            ctx.save_for_backward(x, h, xn, f, mu, rs, rowscale, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls)
            return out
        if fused:  # the fused forward also storing the op-level backward's operands
            out, f, h, xn, mu, rs, g, gp = K.convffn_fwd(x, shape, ln_w, ln_b, W1, b1, wpos, bpos, W2, b2, ls,
                                                         rowscale, save_gelu=True)
            ctx.save_for_backward(x, xn, mu, rs, h, gp, g, f, rowscale, ln_w, w1, b1, wpos, bpos, w2, b2, ls)
            return out
        xn, mu, rs = K.layernorm(x, ln_w, ln_b, 1e-6)
        h = K.linear(xn, W1, b1)
        g = torch.empty_like(h)
        # the DW kernel writes GELU'(hpre) instead of hpre (GELU and its derivative share one erf):
        # the backward's fc2 input gradient then multiplies instead of re-evaluating GELU'
        gp = K.dwconv(h, shape, wpos, bpos, 3, add_identity=True, gelu_out=g, out_gelu_grad=True)
        f = torch.empty(P, C, device=x.device, dtype=dt)
        out = K.linear(g, W2, b2, preact=f, res=x, colscale=ls, rowscale=rowscale, rows_per_scale=H * W)
        ctx.save_for_backward(x, xn, mu, rs, h, gp, g, f, rowscale, ln_w, w1, b1, wpos, bpos, w2, b2, ls)
        return out

    @staticmethod
    def backward(ctx, dout):
        K.TAG = ctx.tag + ".bwd"
        if ctx.fused:
            x, h, xn, f, mu, rs, rowscale, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls = ctx.saved_tensors
            dt = x.dtype
            slots = [gslot(ln_w), gslot(ln_b), gslot2(w1), gslot(b1), gslot(wpos), gslot(bpos), gslot2(w2), gslot(b2),
                     gslot(ls)]
            slots = [None if t is None else t.view(sh) for t, sh in
                     zip(slots, [(-1,), (-1,), tuple(w1.shape), (-1,), (w1.shape[0], 9), (-1,), tuple(w2.shape), (-1,),
                                 (-1,)])]
            dx, dlnw, dlnb, dW1, db1, dwpos, dbpos, dW2, db2, dls = K.convffn_bwd(
                dout.contiguous(), x, h, xn, f, mu, rs, ctx.shape, ln_w, ln_b, wcast(dt, w1), wpos, bpos, wcast(dt, w2), ls,
                rowscale, grads=slots)
            return (dx, None, None, dlnw, dlnb, dW1.view_as(w1), db1, dwpos.view_as(wpos), dbpos, dW2.view_as(w2), db2,
                    dls)
        with wgrad_group(dout.device):  # the fc2 and fc1 weight gradients as one grouped launch at the end
            x, xn, mu, rs, h, gp, g, f, rowscale, ln_w, w1, b1, wpos, bpos, w2, b2, ls = ctx.saved_tensors
            B, H, W = ctx.shape
            dt = x.dtype
            dout = dout.contiguous()
            W1, W2 = wcast(dt, w1), wcast(dt, w2)
            df, dls = K.residual_bwd(dout, f, ls, rowscale, H * W)
            dW2, db2 = K.linear_wgrad(df, g, out=gslot2(w2), bias_grad=True, bias_out=gslot(b2))
            dhpre = K.linear_dgrad(df, W2, mul=gp)  # GELU backward: times the stored GELU'(hpre)
            # input and weight gradients of DW3x3 + identity in one pass over dhpre, h
            dh, dwpos, dbpos = K.dwconv_bwd(h, dhpre, ctx.shape, wpos, 3, add_identity=True, dw=gslot(wpos),
                                            db=gslot(bpos))
            dW1, db1 = K.linear_wgrad(dh, xn, out=gslot2(w1), bias_grad=True, bias_out=gslot(b1))
            dxn = K.linear_dgrad(dh, W1)
            dx, dlnw, dlnb = K.layernorm_bwd(x, dxn, ln_w, mu, rs, dres=dout)
        return (dx, None, None, dlnw, dlnb, dW1.view_as(w1), db1, dwpos.view_as(wpos), dbpos, dW2.view_as(w2), db2,
                dls)


# ====================================================================== Attention (+ residuals)
# The depth branch of the attention BACKWARD (dual product -> e_back -> DW7x7 -> e_fore gradients,
# DFormer.py:84-88, 133) is independent of the RGB branch (pooled attention, q * a, the 7x7
# modulation) until the q|q_cut|l gradients, so the two overlap on two streams (round 6: the RGB part
# on the side stream, the depth branch on the step's own). Measured on MI355X, DFormer-B bf16
# bs 16 graph replay: 407.4-408.0 vs 386.9-387.5 images/s on one stream. (The forward's depth
# branch on a side stream measured 381.6 vs 383.4 images/s and was dropped: it is short and the
# fork / join costs what the overlap gains; a second backward stream for the pooled-attention
# branch gained nothing either.)
_ATTN_BWD_SIDE = {}


def _attn_bwd_side(dev):
    st = _ATTN_BWD_SIDE.get(dev)
    if st is None:
        st = _ATTN_BWD_SIDE[dev] = torch.cuda.Stream(device=dev)
        register_side_stream(st)
    return st


class AttentionFn(torch.autograd.Function):
    """(x1, xe1) = (x + rs*ls1*proj(f), xe + rs*ls1e*proj_e(f)),  f = cat(q*a, attn, cx*xe')

    Parameter order (`params`): see ATTN_PARAM_NAMES. Window 0 (stage 0) has no kv / pooled
    attention (f = cat(q*a, cx*xe')); drop_depth (last block) has no proj_e, xe passes through.
    """

    @staticmethod
    def forward(ctx, x, xe, shape, heads, window, drop_depth, rowscale, rowscale_e, *params):
        (n_w, n_b, ne_w, ne_b, wq, bq, wqc, bqc, wl, bl, wconv, bconv, wa, ba, wef, bef, wec, bec, web, beb,
         wkv, bkv, wsc, bsc, wp, bp, wpe, bpe, ls1, ls1e) = params
        B, H, W = shape
        P, C = x.shape
        Ch = C // 2
        dt = x.dtype
        dev = x.device
        rps = H * W
        ctx.tag = K.TAG
        fw = 2 * C if window else C + Ch
        f = torch.empty(P, fw, device=dev, dtype=dt)
        xen, mu2, rs2 = K.layernorm(xe, ne_w, ne_b, 1e-6)
        xn, mu1, rs1 = K.layernorm(x, n_w, n_b, 1e-6)
        # q | q_cut | l in one GEMM; GELU only on the l columns, whose derivative (act 3) is stored
        # for the backward
        Wqcl = wcast(dt, wq, wqc, wl)
        bqcl = _cat1(bq, bqc, bl)
        qcl = torch.empty(P, 2 * C + Ch, device=dev, dtype=dt)
        lpre = torch.empty(P, C, device=dev, dtype=dt)
        e1 = torch.empty(P, Ch, device=dev, dtype=dt)
        # independent GEMMs of one phase run as one grouped launch (K.gemm_many): q | q_cut | l with e_fore
        K.gemm_many([lambda c: K.linear(xn, Wqcl, bqcl, act=3, preact=lpre, act_col0=C + Ch, out=qcl, collect=c),
                     lambda c: K.linear(xen, wcast(dt, wef), bef, out=e1, collect=c)])
        q, cx, g = qcl[:, :C], qcl[:, C:C + Ch], qcl[:, C + Ch:]
        xep = torch.empty(P, Ch, device=dev, dtype=dt)
        # a = Linear_a(DW7(g)); f[:, :C] = q * a   (a kept for backward)
        apre = K.dwconv(g, shape, wconv, bconv, 7)
        e2 = K.dwconv(e1, shape, wec, bec, 7)
        a = torch.empty(P, C, device=dev, dtype=dt)
        kv = torch.empty(P, C, device=dev, dtype=dt) if window else None
        # a with kv and e_back; depth branch: xe' = e_back(DW7(e_fore(LN xe))); f[:, -Ch:] = cx * xe'
        calls = [lambda c: K.linear(apre, wcast(dt, wa), ba, mul=q, preact=a, out=f[:, :C], collect=c),
                 lambda c: K.linear(e2, wcast(dt, web), beb, mul=cx, preact=xep, out=f[:, fw - Ch:], collect=c)]
        if window:
            calls.append(lambda c: K.linear(g, wcast(dt, wkv), bkv, out=kv, collect=c))
        K.gemm_many(calls)
        saved_attn = ()
        if window:
            dh = C // heads // 2
            pooled = torch.empty(B * 49, C + Ch, device=dev, dtype=dt)
            K.pool7(xn, shape, out=pooled[:, :C])
            K.pool7(xen, shape, out=pooled[:, C:])
            m = K.linear(pooled, wcast(dt, wsc), bsc)
            o, lse = K.pooled_attn(m, kv[:, :Ch], kv[:, Ch:], B, heads, P // B, dh, dh ** -0.5)
            K.bilinear(o, (7, 7), (H, W), B, out=f[:, C:C + Ch])
            saved_attn = (kv, pooled, m, o, lse)
        # projections with the Block's residual / layer-scale / DropPath epilogue
        p1 = torch.empty(P, C, device=dev, dtype=dt)
        x1 = torch.empty(P, C, device=dev, dtype=dt)
        calls = [lambda c: K.linear(f, wcast(dt, wp), bp, preact=p1, res=x, colscale=ls1, rowscale=rowscale,
                                    rows_per_scale=rps, out=x1, collect=c)]
        if drop_depth:  # DFormer.py:133, 141-145: x_e leaves the Block as e_back's output (no proj_e)
            xe1, p1e = xep, None
            ctx.set_materialize_grads(False)  # the encoder discards it: no zero-filled gradient pass
        else:
            p1e = torch.empty(P, Ch, device=dev, dtype=dt)
            xe1 = torch.empty(P, Ch, device=dev, dtype=dt)
            calls.append(lambda c: K.linear(f, wcast(dt, wpe), bpe, preact=p1e, res=xe, colscale=ls1e,
                                            rowscale=rowscale_e, rows_per_scale=rps, out=xe1, collect=c))
        K.gemm_many(calls)  # proj with proj_e
        ctx.shape, ctx.heads, ctx.window, ctx.drop_depth = shape, heads, window, drop_depth
        ctx.n_attn = len(saved_attn)
        ctx.save_for_backward(x, xe, xn, mu1, rs1, xen, mu2, rs2, qcl, lpre, apre, a, e1, e2, xep, f, p1,
                              p1e if p1e is not None else x.new_empty(0), rowscale, rowscale_e, *params,
                              *saved_attn)
        return x1, xe1

    @staticmethod
    def backward(ctx, dx1, dxe1):
        K.TAG = ctx.tag + ".bwd"
        g0 = dx1 if dx1 is not None else dxe1
        with wgrad_group(g0.device if g0 is not None else None):  # the Block attention's weight gradients
            return AttentionFn._backward(ctx, dx1, dxe1)                 # as grouped launches at the end

    @staticmethod
    def _backward(ctx, dx1, dxe1):
        sv = ctx.saved_tensors
        (x, xe, xn, mu1, rs1, xen, mu2, rs2, qcl, lpre, apre, a, e1, e2, xep, f, p1, p1e, rowscale,
         rowscale_e) = sv[:20]
        params = sv[20:20 + 30]
        (n_w, n_b, ne_w, ne_b, wq, bq, wqc, bqc, wl, bl, wconv, bconv, wa, ba, wef, bef, wec, bec, web, beb,
         wkv, bkv, wsc, bsc, wp, bp, wpe, bpe, ls1, ls1e) = params
        saved_attn = sv[50:]
        shape, heads, window, drop_depth = ctx.shape, ctx.heads, ctx.window, ctx.drop_depth
        B, H, W = shape
        P, C = x.shape
        Ch = C // 2
        dt = x.dtype
        dev = x.device
        rps = H * W
        fw = f.shape[1]
        grads = {}
        dx1 = dx1.contiguous() if dx1 is not None else torch.zeros_like(x)
        # projections: proj and proj_e read the same f, so their backward runs as ONE weight-gradient
        # GEMM and ONE input-gradient GEMM over [dp1 | dp1e] (K = C + C/2) against [Wp; Wpe]
        if drop_depth:
            dp1, grads["ls1"] = K.residual_bwd(dx1, p1, ls1, rowscale, rps)
            grads["wp"], grads["bp"] = K.linear_wgrad(dp1, f, out=gslot2(wp), bias_grad=True, bias_out=gslot(bp))
            dpc, Wc = dp1, wcast(dt, wp)
            dxe_res = None  # x_e's output is xe' (no identity path), its gradient joins dxe' below
        else:
            dxe1 = dxe1.contiguous()
            dpc = torch.empty(P, C + Ch, device=dev, dtype=dt)
            _, grads["ls1"] = K.residual_bwd(dx1, p1, ls1, rowscale, rps, df=dpc[:, :C])
            _, grads["ls1e"] = K.residual_bwd(dxe1, p1e, ls1e, rowscale_e, rps, df=dpc[:, C:])
            ow, ob = gslot_rows(wp, wpe), gslot_rows(bp, bpe)
            dWc, dbc = K.linear_wgrad(dpc, f, out=ow, bias_grad=True, bias_out=ob)
            grads["wp"], grads["wpe"] = dWc[:C], dWc[C:]
            grads["bp"], grads["bpe"] = dbc[:C], dbc[C:]
            Wc = wcast(dt, wp, wpe)
            dxe_res = dxe1
        q, cx, g = qcl[:, :C], qcl[:, C:C + Ch], qcl[:, C + Ch:]
        dqcl = torch.empty(P, 2 * C + Ch, device=dev, dtype=dt)
        dq, dcx, dl = dqcl[:, :C], dqcl[:, C:C + Ch], dqcl[:, C + Ch:]
        # df = dpc [Wp; Wpe] by its column blocks f = cat(q*a, attn, cx*xe') in one grouped launch; the two
        # products' backward rides in the epilogues (second output): dq = df_q * a, da = df_q * q;
        # dcx = df_e * xe', dxe' = df_e * cx -- df itself is only materialised for the attention block
        da = torch.empty(P, C, device=dev, dtype=dt)
        dxep = torch.empty(P, Ch, device=dev, dtype=dt)
        dfa = torch.empty(P, Ch, device=dev, dtype=dt) if window else None
        calls = [lambda c: K.linear_dgrad(dpc, Wc[:, :C], out=dq, mul=a, mul2=q, out2=da, collect=c),
                 lambda c: K.linear_dgrad(dpc, Wc[:, fw - Ch:], out=dcx, mul=xep, mul2=cx, out2=dxep, collect=c)]
        if window:
            calls.append(lambda c: K.linear_dgrad(dpc, Wc[:, C:C + Ch], out=dfa, collect=c))
        # (measured on the step against df + two dual_mul passes: 478.3 / 480.8 vs 475.0 / 476.7 images/s)
        K.gemm_many(calls)
        side = _attn_bwd_side(dev) if x.is_cuda else None
        main = torch.cuda.current_stream(dev) if side is not None else None

        def depth_branch():  # cxe = cx * xe',  xe' = e_back(DW7(e_fore(LN_e xe)))
            if drop_depth and dxe1 is not None:  # the Block's x_e output is xe' itself
                K.scale_mul(dxe1.contiguous(), out=dxep, accumulate=True)
            ow, ob = gslot2(web), gslot(beb)
            grads["web"], grads["beb"] = K.linear_wgrad(dxep, e2, out=ow, bias_grad=True, bias_out=ob)
            de2 = K.linear_dgrad(dxep, wcast(dt, web))
            ow, ob = gslot(wec), gslot(bec)
            # (the one-pass 7x7 backward, dfm_dwconv_bwd k = 7, is 4-15 % faster alone but measured slower on the
            # step: 477.0 / 477.4 vs 479.3 / 478.4 images/s; its 65 KB of LDS per block keeps the two streams'
            # 7x7 backwards from sharing a CU)
            grads["wec"], grads["bec"] = K.dwconv_bwd_weight(e1, de2, shape, 7, dw=ow, db=ob)
            de1 = K.dwconv_bwd_data(de2, shape, wec, 7)
            ow, ob = gslot2(wef), gslot(bef)
            grads["wef"], grads["bef"] = K.linear_wgrad(de1, xen, out=ow, bias_grad=True, bias_out=ob)
            return K.linear_dgrad(de1, wcast(dt, wef)), (dxep, de2, de1)

        def rgb_part():  # the pooled attention, q * a and the 7x7 modulation branch
            dg = torch.empty(P, C, device=dev, dtype=dt)
            dxn = dpooled = dkv = None

            def pooled_branch():  # softmax(q_pool k^T) v over the pooled queries, DFormer.py:119-131
                kv, pooled, m, o, lse = saved_attn
                dh = C // heads // 2
                do = K.bilinear_bwd(dfa, (7, 7), (H, W), B)
                dm = torch.empty_like(m)
                dkv = torch.empty(P, C, device=dev, dtype=dt)
                K.pooled_attn_bwd(m, kv[:, :Ch], kv[:, Ch:], o, do, lse, B, heads, P // B, dh, dh ** -0.5, dm,
                                  dkv[:, :Ch], dkv[:, Ch:])
                ow, ob = gslot2(wsc), gslot(bsc)
                grads["wsc"], grads["bsc"] = K.linear_wgrad(dm, pooled, out=ow, bias_grad=True, bias_out=ob)
                dpooled = K.linear_dgrad(dm, wcast(dt, wsc))
                dxn = K.pool7_bwd(dpooled[:, :C], shape)
                ow, ob = gslot2(wkv), gslot(bkv)
                grads["wkv"], grads["bkv"] = K.linear_wgrad(dkv, g, out=ow, bias_grad=True, bias_out=ob)
                return dxn, dpooled, dkv, (do, dm)

            tmp = ()
            if window:
                dxn, dpooled, dkv, tmp = pooled_branch()
            # q * a (dq, da came out of the projection's input-gradient epilogue)
            ow, ob = gslot2(wa), gslot(ba)
            grads["wa"], grads["ba"] = K.linear_wgrad(da, apre, out=ow, bias_grad=True, bias_out=ob)
            dapre = torch.empty(P, C, device=dev, dtype=dt)
            # the a and kv input gradients as one grouped launch
            calls = [lambda c: K.linear_dgrad(da, wcast(dt, wa), out=dapre, collect=c)]
            if window:
                calls.append(lambda c: K.linear_dgrad(dkv, wcast(dt, wkv), out=dg, collect=c))
            K.gemm_many(calls)
            ow, ob = gslot(wconv), gslot(bconv)
            grads["wconv"], grads["bconv"] = K.dwconv_bwd_weight(g, dapre, shape, 7, dw=ow, db=ob)
            K.dwconv_bwd_data(dapre, shape, wconv, 7, dx=dg, accumulate=bool(window))
            K.scale_mul(dg, mul=lpre, out=dl)  # lpre holds GELU'(l pre-activation)
            made = tuple(t for t in (dg, dapre, dkv, dpooled, dxn) + tuple(tmp) if t is not None)
            return dxn, (dpooled[:, C:] if dpooled is not None else None), made

        # The RGB part runs on the side stream and the depth branch on the step's stream: the side stream's
        # kernels get the smaller share of the CUs, and with the depth branch there the join waited ~2 ms per
        # step for it (profiles/r06_queue_analysis.txt); swapped: 495.7 / 495.1 vs 491.3 / 492.6 images/s
        if side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                dxn, dpooled_e, made = rgb_part()
            dxen, _ = depth_branch()
            main.wait_stream(side)
            for t in made:  # side allocations read here or by the block's queued weight gradients
                t.record_stream(main)
        else:
            dxen, _ = depth_branch()
            dxn, dpooled_e, _ = rgb_part()
        if dpooled_e is not None:
            K.pool7_bwd(dpooled_e, shape, dx=dxen, accumulate=True)
        # q | q_cut | l
        dWqcl, dbqcl = K.linear_wgrad(dqcl, xn, bias_grad=True, out=gslot_rows(wq, wqc, wl),
                                      bias_out=gslot_rows(bq, bqc, bl))
        grads["bq"], grads["bqc"], grads["bl"] = dbqcl[:C], dbqcl[C:C + Ch], dbqcl[C + Ch:]
        grads["wq"], grads["wqc"], grads["wl"] = dWqcl[:C], dWqcl[C:C + Ch], dWqcl[C + Ch:]
        Wqcl = wcast(dt, wq, wqc, wl)
        if dxn is None:
            dxn = K.linear_dgrad(dqcl, Wqcl)
        else:
            K.linear_dgrad(dqcl, Wqcl, out=dxn, accumulate=True)
        dx, grads["n_w"], grads["n_b"] = K.layernorm_bwd(x, dxn, n_w, mu1, rs1, dres=dx1)
        dxe, grads["ne_w"], grads["ne_b"] = K.layernorm_bwd(xe, dxen, ne_w, mu2, rs2, dres=dxe_res)
        out = []
        for name, p in zip(ATTN_PARAM_NAMES, params):
            gr = grads.get(name)
            if gr is not None and p.numel() > 0:
                gr = gr.reshape(p.shape)
            out.append(gr if p.numel() > 0 else None)
        return (dx, dxe, None, None, None, None, None, None, *out)


ATTN_PARAM_NAMES = ("n_w", "n_b", "ne_w", "ne_b", "wq", "bq", "wqc", "bqc", "wl", "bl", "wconv", "bconv", "wa", "ba",
                    "wef", "bef", "wec", "bec", "web", "beb", "wkv", "bkv", "wsc", "bsc", "wp", "bp", "wpe", "bpe",
                    "ls1", "ls1e")
