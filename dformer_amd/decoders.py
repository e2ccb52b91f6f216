"""Segmentation decoders on HIP kernels with the reference's module tree / state_dict keys.

  LightHamHead (+ Hamburger, NMF2D)   models/decoders/ham_head.py:11-240, decode_head.py:55-231
  DecoderHead (MLPDecoder)            models/decoders/MLPDecoder.py:8-81
  seg_loss                            models/builder.py:203,230

Feature maps are NHWC rows [B*h*w, C] in the compute dtype. BatchNorm runs in training mode on
batch statistics; with a multi-rank process group and SyncBN, the (sum, sumsq) and the backward
(sum dy, sum dy*xhat) statistics are all-reduced (SyncBatchNorm semantics).
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from . import kernels as K
from .functional import gslot, gslot2, gslot_rows, wcast


# Test-only: with an initialised one-rank process group, take every collective branch (SyncBN
# all-gather / all-reduce, bucketed gradient all-reduce, loss all-reduce) as if world > 1, so the
# multi-rank code runs (and is captured into HIP graphs) on a single GPU (tests/test_graph_gpu.py).
FORCE_COLLECTIVES = False


def collectives_on(world=None):
    """True when the data-parallel collective branches run: world > 1, or FORCE_COLLECTIVES with an
    initialised process group."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    w = dist.get_world_size() if world is None else world
    return w > 1 or FORCE_COLLECTIVES


def _world(sync):
    if sync and dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


# Per-rank row counts of a SyncBN batch, keyed by (local rows, world): data-parallel ranks see the
# same batch shape every step, so the counts are exchanged (and read on the host) once per shape.
_GLOBAL_ROWS = {}
_GLOBAL_TOTAL = {}


def bn_batch_stats(x, bn, sync):
    """Train-mode BatchNorm / SyncBatchNorm statistics of NHWC rows x: (mean, rstd, count), with the
    running statistics updated like torch (momentum, unbiased variance). With SyncBN over a
    multi-rank group the per-rank shifted sums are all-gathered into one [world, 3, C] buffer and
    merged on the device (K.bn_merge; torch SyncBatchNorm all-gathers (mean, invstd, count) the
    same way, torch/nn/modules/_functions.py)."""
    st = K.bn_stats(x)
    rows = x.shape[0]
    world = _world(sync)
    count = rows
    if sync and collectives_on(world):
        # gathered along dim 0 as [world * 3, C] (gloo splits the output along its first dim and
        # requires each piece to have the input's shape; RCCL takes either form)
        gathered = torch.empty((world * st.shape[0],) + tuple(st.shape[1:]), device=st.device, dtype=st.dtype)
        dist.all_gather_into_tensor(gathered, st)
        gathered = gathered.view((world,) + tuple(st.shape))
        counts = _GLOBAL_ROWS.get((rows, world))
        if counts is None:  # first batch of this shape: exchange the per-rank row counts once
            cnt = torch.tensor([float(rows)], device=x.device)
            counts = torch.empty(world, device=x.device)
            dist.all_gather_into_tensor(counts, cnt)
            _GLOBAL_ROWS[(rows, world)] = counts
        st = K.bn_merge(gathered, counts)
        total = _GLOBAL_TOTAL.get((rows, world))
        if total is None:  # one host read per batch shape, not one per BN layer per step
            total = _GLOBAL_TOTAL[(rows, world)] = int(counts.sum().item())
        count = total
    mean, rstd = K.bn_finalize(st, count, bn.eps, bn.momentum if bn.momentum is not None else 0.1, bn.running_mean,
                               bn.running_var)
    bn.num_batches_tracked.add_(1)
    return mean, rstd, count


# test-only probe (tests/test_dp_gpu.py): when a dict, bn_grad_stats records per BN layer (by id) the
# float64 sums [sum dy*xhat, sum dy, sum |dy*xhat|, sum |dy|] of the rows it reduces, from the same
# dy / x / mean / rstd its kernel reads
BN_PROBE = None


def bn_grad_stats(x, dy, mean, rstd, bn, sync):
    """BatchNorm backward statistics st2 = (sum dy, sum dy * xhat) of NHWC rows. Returns (st2 for the
    input gradient, dgamma, dbeta). The local statistics ARE this rank's beta / gamma gradients
    (SyncBatchNorm's backward forms grad_weight / grad_bias before its all-reduce,
    torch/nn/modules/_functions.py; DDP then averages them like every gradient) and are written
    straight into the flat gradient slots, laid out [beta | gamma] by train.fused_chains; under
    SyncBN an all-reduced copy feeds the input gradient."""
    out = gslot_rows(bn.bias, bn.weight) if bn is not None and bn.affine else None
    if BN_PROBE is not None and bn is not None:
        dyd = dy.double()
        t = dyd * ((x.double() - mean.double()) * rstd.double())
        BN_PROBE[id(bn)] = torch.stack([t.sum(0), dyd.sum(0), t.abs().sum(0), dyd.abs().sum(0)])
    st = K.bn_bwd_stats(x, dy, mean, rstd, out=out.view(2, -1) if out is not None else None)
    stg = st
    if sync and collectives_on():
        stg = st.clone()
        dist.all_reduce(stg)
    return stg, st[1], st[0]


# ============================================================================ building blocks
class ConvBNActFn(torch.autograd.Function):
    """y = act(BN(x @ W^T) [+ res])  — mmcv ConvModule(1x1 conv, BN, ReLU) (ham_head.py:204-220)."""

    @staticmethod
    def forward(ctx, x, res, w, gamma, beta, bn, act, sync):
        dt = x.dtype
        Wc = wcast(dt, w)
        y0 = K.linear(x, Wc)
        rows = x.shape[0]
        if bn.training:
            mean, rstd, count = bn_batch_stats(y0, bn, sync)
        else:
            mean = bn.running_mean
            rstd = torch.rsqrt(bn.running_var + bn.eps)
            count = rows
        y = K.bn_apply(y0, mean, rstd, gamma, beta, res=res, act=act)
        ctx.save_for_backward(x, w, y0, y, mean, rstd, gamma)
        ctx.act, ctx.sync, ctx.count, ctx.has_res, ctx.bn = act, sync, count, res is not None, bn
        return y

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "decoder.bwd"
        x, w, y0, y, mean, rstd, gamma = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == 2:
            dy = K.relu_bwd(dy, y)
        st2, dgamma, dbeta = bn_grad_stats(y0, dy, mean, rstd, ctx.bn, ctx.sync)
        dy0 = K.bn_bwd_apply(y0, dy, mean, rstd, gamma, st2, ctx.count)
        dW = K.linear_wgrad(dy0, x, out=gslot2(w))
        dx = K.linear_dgrad(dy0, wcast(x.dtype, w))
        dres = dy if ctx.has_res else None
        return dx, dres, dW.view_as(w), dgamma, dbeta, None, None, None


class LinearActFn(torch.autograd.Function):
    """y = act(x @ W^T + b), optional float32 output (ham_in: ConvModule(bias, no norm) + ReLU)."""

    @staticmethod
    def forward(ctx, x, w, b, act, out_f32):
        Wc = wcast(x.dtype, w)
        out = torch.empty(x.shape[0], w.shape[0], device=x.device,
                          dtype=torch.float32 if out_f32 else x.dtype)
        K.linear(x, Wc, b, act=act, out=out)
        ctx.save_for_backward(x, w, b, out)
        ctx.act = act
        return out

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "decoder.bwd"
        x, w, b, y = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == 2:
            dy = K.relu_bwd(dy, y)
        if dy.dtype != x.dtype:
            dy = K.cast(dy, x.dtype)
        dW, db = K.linear_wgrad(dy, x, out=gslot2(w), bias_grad=True, bias_out=gslot(b))
        dx = K.linear_dgrad(dy, wcast(x.dtype, w))
        return dx, dW.view_as(w), db, None, None


class CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return x if x.dtype == dtype else K.cast(x.contiguous(), dtype)

    @staticmethod
    def backward(ctx, g):
        K.TAG = "decoder.bwd"
        g = g.contiguous()
        return (g if g.dtype == ctx.src else K.cast(g, ctx.src)), None


class ResizeCatFn(torch.autograd.Function):
    """cat([resize(f_i, size of f_0, bilinear, align_corners=False)], channels)  (ham_head.py:226-233,
    MLPDecoder.py:67-77). feats: NHWC rows; hw: list of (h, w)."""

    @staticmethod
    def forward(ctx, B, hw, *feats):
        H0, W0 = hw[0]
        widths = [f.shape[1] for f in feats]
        out = torch.empty(B * H0 * W0, sum(widths), device=feats[0].device, dtype=feats[0].dtype)
        c = 0
        for f, (h, w), cw in zip(feats, hw, widths):
            if (h, w) == (H0, W0):
                K.scale_mul(f, out=out[:, c:c + cw])
            else:
                K.bilinear(f, (h, w), (H0, W0), B, out=out[:, c:c + cw])
            c += cw
        ctx.B, ctx.hw, ctx.widths = B, hw, widths
        return out

    @staticmethod
    def backward(ctx, dout):
        K.TAG = "decoder.bwd"
        dout = dout.contiguous()
        H0, W0 = ctx.hw[0]
        grads = []
        c = 0
        for (h, w), cw in zip(ctx.hw, ctx.widths):
            sl = dout[:, c:c + cw]
            if (h, w) == (H0, W0):
                grads.append(K.scale_mul(sl))
            else:
                grads.append(K.bilinear_bwd(sl, (h, w), (H0, W0), ctx.B))
            c += cw
        return (None, None, *grads)


class SqueezeFoldFn(torch.autograd.Function):
    """LightHamHead's resize + cat + squeeze ConvModule (1x1 conv, BN, ReLU; ham_head.py:226-234),
    folded like MLPFoldFn: bilinear upsampling (align_corners=False) commutes with the 1x1 conv, so

        W cat[c_0, up(c_1), up(c_2)] = W_0 c_0 + up(W_1 c_1) + up(W_2 c_2)

    with W_i the column block of the squeeze weight that the cat order (in_index order, finest
    first) gives level i. Each level's product runs at its own resolution with K = C_i instead of
    one K = sum C_i GEMM over the concatenated map. Backward: G_i = up_i^T(dy0), dW_i = G_i^T c_i
    (column block i of the weight gradient), dc_i = G_i W_i."""

    @staticmethod
    def forward(ctx, B, hw, bn, sync, w, gamma, beta, *rows):
        dt = rows[0].dtype
        H0, W0 = hw[0]
        E = w.shape[0]
        Wc = wcast(dt, w).view(E, -1)
        offs = [0]
        for r in rows:
            offs.append(offs[-1] + r.shape[1])
        assert offs[-1] == Wc.shape[1], "squeeze weight / concatenated channels mismatch"
        y0 = None
        for i, r in enumerate(rows):
            Wi = Wc[:, offs[i]:offs[i + 1]]
            h, wd = hw[i]
            if (h, wd) == (H0, W0):
                y0 = K.linear(r, Wi) if y0 is None else K.linear(r, Wi, out=y0, beta=1.0)
            else:  # at the level's own resolution, then upsampled into the sum
                t = K.linear(r, Wi)
                if y0 is None:
                    y0 = K.bilinear(t, (h, wd), (H0, W0), B)
                else:
                    K.bilinear(t, (h, wd), (H0, W0), B, out=y0, accumulate=True)
        count = y0.shape[0]
        if bn.training:
            mean, rstd, count = bn_batch_stats(y0, bn, sync)
        else:
            mean, rstd = bn.running_mean, torch.rsqrt(bn.running_var + bn.eps)
        y = K.bn_apply(y0, mean, rstd, gamma, beta, act=2)
        ctx.save_for_backward(y0, y, mean, rstd, gamma, w, *rows)
        ctx.meta = (B, hw, count, sync, bn, offs)
        return y

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "decoder.bwd"
        y0, y, mean, rstd, gamma, w = ctx.saved_tensors[:6]
        rows = ctx.saved_tensors[6:]
        B, hw, count, sync, bn, offs = ctx.meta
        H0, W0 = hw[0]
        E = w.shape[0]
        dy = K.relu_bwd(dy.contiguous(), y)
        st2, dgamma, dbeta = bn_grad_stats(y0, dy, mean, rstd, bn, sync)
        dy0 = K.bn_bwd_apply(y0, dy, mean, rstd, gamma, st2, count)
        dW = gslot2(w)
        if dW is None:
            dW = torch.empty(E, offs[-1], device=y0.device, dtype=torch.float32)
        dW = dW.view(E, -1)
        Wc = wcast(y0.dtype, w).view(E, -1)
        drows = []
        with K.wgrad_group():  # the per-level dW_i as one grouped launch
            for i, r in enumerate(rows):
                h, wd = hw[i]
                G = dy0 if (h, wd) == (H0, W0) else K.bilinear_bwd(dy0, (h, wd), (H0, W0), B)
                K.linear_wgrad(G, r, out=dW[:, offs[i]:offs[i + 1]])
                drows.append(K.linear_dgrad(G, Wc[:, offs[i]:offs[i + 1]]))
        return (None, None, None, None, dW.view_as(w), dgamma, dbeta, *drows)


class ChannelDropoutLinearFn(torch.autograd.Function):
    """logits = (x * mask[b, c] / keep) @ W^T + b   — Dropout2d + 1x1 conv (decode_head.py:226-231)."""

    @staticmethod
    def forward(ctx, x, scale, B, w, b):
        dt = x.dtype
        xs = x
        if scale is not None:  # [B, C] per-image channel scale, one launch
            xs = K.group_scale(x, scale.contiguous(), x.shape[0] // B)
        y = K.linear(xs, wcast(dt, w), b)
        ctx.save_for_backward(xs, w, b, scale)
        ctx.B = B
        return y

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "decoder.bwd"
        xs, w, b, scale = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != xs.dtype:
            dy = K.cast(dy, xs.dtype)
        dW, db = K.linear_wgrad(dy, xs, out=gslot2(w), bias_grad=True, bias_out=gslot(b))
        dx = K.linear_dgrad(dy, wcast(xs.dtype, w))
        if scale is not None:
            K.group_scale(dx, scale.contiguous(), dx.shape[0] // ctx.B, out=dx)
        return dx, None, None, dW.view_as(w), db


# ======================================================================================= NMF
class NMF2DFn(torch.autograd.Function):
    """NMF2D.forward (ham_head.py:60-145) on NHWC: x [B, N, D] (= the reference's x^T), bases
    [B, D, R] injected or freshly drawn; gradients flow through every multiplicative step.

    x float32: every product in float32. x bfloat16 (the bf16 model; the reference's autocast runs
    these bmm in bf16): the products that stream x (x B, x^T C and their backward twins) and the
    output B C^T take bf16 operands with float32 accumulation; coef / bases, the small R x R
    products and every multiplicative update stay float32 (nmf_update emits the bf16 operand copy).

    Rank 64 runs as two library calls (dfm_nmf_fwd keeping every step's factors, dfm_nmf_bwd);
    entry=False issues the same launches one by one from here (the bit-identity reference of
    tests/test_kernels_gpu.py::test_nmf_entry_points, and the path for other ranks)."""

    @staticmethod
    def forward(ctx, x, bases, steps, eps, entry=True):
        x = x.contiguous()
        lp = x.dtype in (torch.bfloat16, torch.float16)
        B0 = bases.contiguous()
        if entry and B0.shape[2] == 64 and K.ACCOUNT is None:
            # rank 64 (the config's MD_R): the whole loop and its backward are library entry points
            # (dfm_nmf_fwd / dfm_nmf_bwd) issuing the launches below in the same order. bench.py's
            # census step (K.ACCOUNT set) takes the launch-by-launch path instead: the same kernels,
            # each charged its own algorithmic FLOPs / bytes
            B0 = B0.float()
            y, saved = K.nmf_fwd(x, B0, steps, eps, keep=True)
            ctx.entry, ctx.steps, ctx.eps = True, steps, eps
            ctx.save_for_backward(x, B0, saved)
            return y
        ctx.entry = False
        f32 = dict(device=x.device, dtype=torch.float32)

        def xmm(b16, a_t=False):  # x-streaming product, float32 out
            Bb, N, D = x.shape
            R = b16.shape[2]
            return K.bmm(x, b16, a_t=a_t, out=torch.empty(Bb, D if a_t else N, R, **f32))

        num0 = xmm(K.cast(B0, x.dtype) if lp else B0)
        coef = K.softmax_rows(num0)                                      # softmax(x^T B)
        hist = []
        Bt, Ct = B0, coef
        Bt16 = K.cast(B0, x.dtype) if lp else B0
        fused = B0.shape[2] == 64  # rank 64 (the config's MD_R): the den products fused into the updates
        ctx.fused = fused

        def update(a, num, G):  # a * num / (a G + eps) -> (out, den, 16-bit copy)
            if fused:
                r = K.nmf_update_mm(a, num, G, eps, bf16_copy=x.dtype if lp else False)
                return r if lp else (r[0], r[1], r[0])
            den = K.bmm(a, G)
            o = K.nmf_update(a, num, den, eps, bf16_copy=x.dtype) if lp else (K.nmf_update(a, num, den, eps),) * 2
            return o[0], den, o[1]

        for s in range(steps):
            num1 = num0 if s == 0 else xmm(Bt16)                  # x^T B        [N,R]
            M = K.bmm(Bt, Bt, a_t=True)                           # B^T B        [R,R]
            Cn, den1, Cn16 = update(Ct, num1, M)                  # den1 = C (B^T B)
            num2 = xmm(Cn16, a_t=True)                            # x C          [D,R]
            Q = K.bmm(Cn, Cn, a_t=True)                           # C^T C        [R,R]
            Bn, den2, Bn16 = update(Bt, num2, Q)                  # den2 = B (C^T C)
            hist.append((Bt, Ct, num1, M, den1, Cn, Cn16, num2, Q, den2, Bn))
            Bt, Ct, Bt16 = Bn, Cn, Bn16
        num = xmm(Bt16)
        M = K.bmm(Bt, Bt, a_t=True)
        Cf, den, Cf16 = update(Ct, num, M)
        y = K.bmm(Cf16, Bt16, b_t=True)                           # (B C^T)^T    [N,D], x.dtype
        ctx.hist = hist
        ctx.final = (Bt, Bt16, Ct, num, M, den, Cf, Cf16)
        ctx.eps = eps
        ctx.save_for_backward(x, B0, coef)
        return y

    @staticmethod
    def backward(ctx, gy):
        K.TAG = "decoder.bwd"
        if ctx.entry:
            x, B0, saved = ctx.saved_tensors
            gx = K.nmf_bwd(x, B0, saved, gy.contiguous(), ctx.steps, ctx.eps)
            return gx, None, None, None, None
        x, B0, coef0 = ctx.saved_tensors
        eps = ctx.eps
        lp = x.dtype in (torch.bfloat16, torch.float16)
        gy = gy.contiguous()
        Bb, N, D = x.shape
        R = B0.shape[2]
        f32 = dict(device=x.device, dtype=torch.float32)
        Bt, Bt16, Ct, num, M, den, Cf, Cf16 = ctx.final
        gC = K.bmm(gy, Bt16, out=torch.empty(Bb, N, R, **f32))   # gy B         [N,R]
        gB = K.bmm(gy, Cf16, a_t=True, out=torch.empty(Bb, D, R, **f32))  # gy^T C  [D,R]

        def upd_bwd(g, a, nm, dn, out):  # -> ga, gnum, gden, gnum operand for the x products
            r = K.nmf_update_bwd(g, a, nm, dn, out, eps=eps, bf16_copy=x.dtype if lp else None)
            return r if lp else (*r, r[1])

        # Every contribution to gx is a rank-R product P Q^T (P [N,R], Q [D,R]); they are gathered
        # side by side and applied by ONE GEMM over the concatenated K = T*R at the end, instead of
        # T read-modify-write passes over the [N, D] gradient.
        T = 2 * len(ctx.hist) + 2
        Ps, Qs = [], []

        def gx_term(P, Q):  # packed side by side at the end, one launch per operand (K.pack_slices)
            Ps.append(P)
            Qs.append(Q)

        if ctx.fused:
            # the den products' gradients ride in the fused update kernels: each C / B update's
            # gden M (gden Q) is added to its ga in place, and the symmetric Gram gradients
            # B (gM + gM^T) / C (gQ + gQ^T) are folded into the g of the update that consumes them
            def upd_mm(g, a, nm, dn, out, A2=None, S=None, Mg=None):
                r = K.nmf_update_bwd_mm(g, a, nm, dn, out, A2=A2, S=S, Mg=Mg, eps=eps,
                                        bf16_copy=x.dtype if lp else False)
                return r if lp else (*r, r[1])

            gCt, gnum, gden, gnum16 = upd_mm(gC, Ct, num, den, Cf, Mg=M)   # + gden M
            gx_term(gnum, Bt)                                             # gx += gnum B^T
            K.bmm(x, gnum16, a_t=True, out=gB, beta=1.0)                  # gB += x^T gnum
            pend = (Bt, K.bmm(Ct, gden, a_t=True))                        # gB += Bt (gM + gM^T)
            gC = gCt
            for (Bp, Cp, num1, M1, den1, Cn, Cn16, num2, Q, den2, Bn) in reversed(ctx.hist):
                assert pend[0] is Bn
                gBp, gnum2, gden2, gnum2_16 = upd_mm(gB, Bp, num2, den2, Bn, A2=pend[0], S=pend[1], Mg=Q)
                gx_term(Cn, gnum2)                                        # gx += Cn gnum2^T
                K.bmm(x, gnum2_16, out=gC, beta=1.0)                      # gCn += x gnum2
                gQ = K.bmm(Bp, gden2, a_t=True)                           # Bp^T gden2
                gCp, gnum1, gden1, gnum1_16 = upd_mm(gC, Cp, num1, den1, Cn, A2=Cn, S=gQ, Mg=M1)
                gx_term(gnum1, Bp)                                        # gx += gnum1 Bp^T
                K.bmm(x, gnum1_16, a_t=True, out=gBp, beta=1.0)           # gBp += x^T gnum1
                pend = (Bp, K.bmm(Cp, gden1, a_t=True))
                gB, gC = gBp, gCp
            # (the pending Gram term belongs to the random bases B0: no gradient)
        else:
            gC = NMF2DFn._backward_unfused(ctx, x, gy, gC, gB, upd_bwd, gx_term)
        gS = K.softmax_rows_bwd(coef0, gC)
        gx_term(gS, B0)                                           # gx += gS B0^T
        assert len(Ps) == T
        Pc = K.pack_slices(Ps, torch.empty(Bb, N, T * R, device=x.device, dtype=x.dtype))
        Qc = K.pack_slices(Qs, torch.empty(Bb, D, T * R, device=x.device, dtype=x.dtype))
        gx = K.bmm(Pc, Qc, b_t=True)                              # sum_i P_i Q_i^T, x.dtype
        ctx.hist = ctx.final = None
        return gx, None, None, None, None

    @staticmethod
    def _backward_unfused(ctx, x, gy, gC, gB, upd_bwd, gx_term):
        """Backward with every den product a separate batched GEMM (ranks other than 64)."""
        Bt, Bt16, Ct, num, M, den, Cf, Cf16 = ctx.final
        # final coef update: Cf = Ct * num / (Ct M + eps), num = x B, M = B^T B
        gCt, gnum, gden, gnum16 = upd_bwd(gC, Ct, num, den, Cf)
        gx_term(gnum, Bt)                                         # gx += gnum B^T
        K.bmm(x, gnum16, a_t=True, out=gB, beta=1.0)              # gB += x^T gnum
        _acc_CM(gCt, gB, Ct, Bt, M, gden)
        gC = gCt
        for (Bp, Cp, num1, M1, den1, Cn, Cn16, num2, Q, den2, Bn) in reversed(ctx.hist):
            # B-update: Bn = Bp * num2 / (Bp Q + eps), num2 = x^T-side (x C_n), Q = Cn^T Cn
            gBp, gnum2, gden2, gnum2_16 = upd_bwd(gB, Bp, num2, den2, Bn)
            gx_term(Cn, gnum2)                                    # gx += Cn gnum2^T
            K.bmm(x, gnum2_16, out=gC, beta=1.0)                  # gCn += x gnum2
            K.bmm(gden2, Q, out=gBp, beta=1.0)                    # gBp += gden2 Q
            gQ = K.bmm(Bp, gden2, a_t=True)                       # Bp^T gden2
            K.bmm(Cn, gQ, out=gC, beta=1.0)
            K.bmm(Cn, gQ, b_t=True, out=gC, beta=1.0)
            # C-update: Cn = Cp * num1 / (Cp M1 + eps), num1 = x B_p, M1 = Bp^T Bp
            gCp, gnum1, gden1, gnum1_16 = upd_bwd(gC, Cp, num1, den1, Cn)
            gx_term(gnum1, Bp)                                    # gx += gnum1 Bp^T
            K.bmm(x, gnum1_16, a_t=True, out=gBp, beta=1.0)       # gBp += x^T gnum1
            _acc_CM(gCp, gBp, Cp, Bp, M1, gden1)
            gB, gC = gBp, gCp
        return gC  # coef0 = softmax(x B0)  (B0 is a random constant)


def _acc_CM(gC, gB, C, Bt, M, gden):
    """den = C M, M = B^T B (symmetric):  gC += gden M ; gB += B (gM + gM^T), gM = C^T gden."""
    K.bmm(gden, M, out=gC, beta=1.0)
    gM = K.bmm(C, gden, a_t=True)
    K.bmm(Bt, gM, out=gB, beta=1.0)
    K.bmm(Bt, gM, b_t=True, out=gB, beta=1.0)


# ============================================================================ mmcv-like modules
class ConvModule(nn.Module):
    """1x1 ConvModule parameter container: `conv` (+ `bn`), keys as mmcv (ham_head.py:156-220)."""

    def __init__(self, cin, cout, norm=True, bias=None, bn_eps=1e-5):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 1, bias=(not norm) if bias is None else bias)
        if norm:
            self.bn = nn.BatchNorm2d(cout, eps=bn_eps)

    def fused(self, x, act, res=None, sync=False):
        return ConvBNActFn.apply(x, res, self.conv.weight, self.bn.weight, self.bn.bias, self.bn, act, sync)


class NMF2D(nn.Module):
    """NMF2D (ham_head.py:103-145): S=1, D=C, R=64, 6 train / 7 eval steps, inv_t=1, eps 1e-6."""

    def __init__(self, args=None):
        super().__init__()
        args = dict(args or {})
        self.S = args.get("MD_S", 1)
        self.R = args.get("MD_R", 64)
        self.train_steps = args.get("TRAIN_STEPS", 6)
        self.eval_steps = args.get("EVAL_STEPS", 7)
        self.injected_bases = None  # parity runs inject the reference's random bases
        self.generator = None

    def _build_bases(self, B, D, device):
        if self.injected_bases is not None:
            return self.injected_bases.to(device=device, dtype=torch.float32)
        b = torch.rand(B * self.S, D, self.R, device=device, generator=self.generator)
        return b / b.norm(dim=1, keepdim=True).clamp_min(1e-12)  # F.normalize(dim=1)

    def fused(self, x, B, N):
        """x: [B*N, D] rows (float32, or bf16 for the bf16 model) -> [B*N, D] rows of x.dtype."""
        D = x.shape[1]
        bases = self._build_bases(B, D, x.device)
        steps = self.train_steps if self.training else self.eval_steps
        if not torch.is_grad_enabled() and bases.shape[2] == 64 and K.ACCOUNT is None:  # inference
            return K.nmf_fwd(x.view(B, N, D).contiguous(), bases.float().contiguous(), steps, 1e-6).view(B * N, D)
        y = NMF2DFn.apply(x.view(B, N, D), bases, steps, 1e-6)
        return y.view(B * N, D)


class Hamburger(nn.Module):
    def __init__(self, ham_channels=512, ham_kwargs=None, norm_cfg=None, bn_eps=1e-5, **kwargs):
        super().__init__()
        self.ham_in = ConvModule(ham_channels, ham_channels, norm=False)
        self.ham = NMF2D(ham_kwargs)
        self.ham_out = ConvModule(ham_channels, ham_channels, norm=True, bn_eps=bn_eps)

    def fused(self, x, B, N, sync):
        enjoy = LinearActFn.apply(x, self.ham_in.conv.weight, self.ham_in.conv.bias, 2, False)
        enjoy = self.ham.fused(enjoy, B, N)
        enjoy = CastFn.apply(enjoy, x.dtype)
        return self.ham_out.fused(enjoy, act=2, res=x, sync=sync)  # relu(x + BN(conv(enjoy)))


def _nhwc_rows(t):
    """NCHW view of a channels-last buffer (or NHWC tensor) -> ([B*H*W, C] rows, (B, H, W))."""
    if t.dim() == 4 and t.shape[1] != t.shape[-1] and t.permute(0, 2, 3, 1).is_contiguous():
        B, C, H, W = t.shape
        return t.permute(0, 2, 3, 1).reshape(B * H * W, C), (B, H, W)
    B, C, H, W = t.shape
    return t.permute(0, 2, 3, 1).contiguous().view(B * H * W, C), (B, H, W)


class LightHamHead(nn.Module):
    """LightHamHead (ham_head.py:184-240) + BaseDecodeHead pieces (decode_head.py:55-231).
    forward(list of 4 NCHW maps) -> logits NCHW view of NHWC rows [B, ncls, H/8, W/8]."""

    def __init__(self, ham_channels=512, ham_kwargs=None, in_channels=(128, 256, 512), channels=512, num_classes=40,
                 dropout_ratio=0.1, norm_cfg=None, in_index=(1, 2, 3), align_corners=False, bn_eps=1e-3,
                 bn_momentum=0.1, device=None, **kwargs):
        super().__init__()
        self.in_channels = list(in_channels)
        self.in_index = list(in_index)
        self.channels = channels
        self.num_classes = num_classes
        self.dropout_ratio = dropout_ratio
        self.ham_channels = ham_channels
        self.syncbn = bool(norm_cfg) and norm_cfg.get("type") == "SyncBN"
        self.squeeze = ConvModule(sum(self.in_channels), ham_channels, norm=True, bn_eps=bn_eps)
        self.hamburger = Hamburger(ham_channels, ham_kwargs, bn_eps=bn_eps)
        self.align = ConvModule(ham_channels, channels, norm=True, bn_eps=bn_eps)
        self.conv_seg = nn.Conv2d(channels, num_classes, kernel_size=1)
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.momentum = bn_momentum
        self.dropout_masks = None  # tests may inject Dropout2d keep masks [B, channels]

    def forward(self, inputs):
        feats = [inputs[i] for i in self.in_index]
        rows, hw = [], []
        B = feats[0].shape[0]
        for f in feats:
            r, (b, h, w) = _nhwc_rows(f)
            rows.append(r)
            hw.append((h, w))
        sq = self.squeeze
        x = SqueezeFoldFn.apply(B, hw, sq.bn, self.syncbn, sq.conv.weight, sq.bn.weight, sq.bn.bias, *rows)
        H, W = hw[0]
        x = self.hamburger.fused(x, B, H * W, self.syncbn)
        x = self.align.fused(x, act=2, sync=self.syncbn)
        scale = None
        if self.training and self.dropout_ratio > 0:
            keep = 1.0 - self.dropout_ratio
            mask = self.dropout_masks if self.dropout_masks is not None else \
                (torch.rand(B, self.channels, device=x.device) < keep)
            scale = mask.to(device=x.device, dtype=torch.float32) / keep
        logits = ChannelDropoutLinearFn.apply(x, scale, B, self.conv_seg.weight, self.conv_seg.bias)
        return logits.view(B, H, W, self.num_classes).permute(0, 3, 1, 2)


class _Proj(nn.Module):
    """MLPDecoder.MLP: Linear embedding (MLPDecoder.py:8-19), key `proj`."""

    def __init__(self, input_dim, embed_dim):
        super().__init__()
        self.proj = nn.Linear(input_dim, embed_dim)


class DecoderHead(nn.Module):
    """SegFormer-style all-MLP head (MLPDecoder.py:22-81) -> logits at 1/4 resolution."""

    def __init__(self, in_channels=(64, 128, 320, 512), num_classes=40, dropout_ratio=0.1, norm_layer=nn.BatchNorm2d,
                 embed_dim=768, align_corners=False, bn_eps=1e-3, bn_momentum=0.1, syncbn=False):
        super().__init__()
        self.num_classes = num_classes
        self.dropout_ratio = dropout_ratio
        self.in_channels = list(in_channels)
        self.embed_dim = embed_dim
        self.syncbn = syncbn
        c1, c2, c3, c4 = self.in_channels
        self.linear_c4 = _Proj(c4, embed_dim)
        self.linear_c3 = _Proj(c3, embed_dim)
        self.linear_c2 = _Proj(c2, embed_dim)
        self.linear_c1 = _Proj(c1, embed_dim)
        self.linear_fuse = nn.Sequential(nn.Conv2d(embed_dim * 4, embed_dim, kernel_size=1),
                                         nn.BatchNorm2d(embed_dim, eps=bn_eps, momentum=bn_momentum),
                                         nn.ReLU(inplace=True))
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, kernel_size=1)
        self.dropout_masks = None

    def forward(self, inputs):
        B = inputs[0].shape[0]
        lvl, hw = [], []
        for i in range(4):  # c1 (finest, the output resolution) .. c4
            r, (b, h, w) = _nhwc_rows(inputs[i])
            lin = getattr(self, f"linear_c{i + 1}").proj
            lvl += [r, lin.weight, lin.bias]
            hw.append((h, w))
        H, W = hw[0]
        E = self.embed_dim
        fuse, bn = self.linear_fuse[0], self.linear_fuse[1]
        x = MLPFoldFn.apply(B, hw, E, bn, self.syncbn, fuse.weight, fuse.bias, bn.weight, bn.bias, *lvl)
        scale = None
        if self.training and self.dropout_ratio > 0:
            keep = 1.0 - self.dropout_ratio
            mask = self.dropout_masks if self.dropout_masks is not None else \
                (torch.rand(B, E, device=x.device) < keep)
            scale = mask.to(device=x.device, dtype=torch.float32) / keep
        logits = ChannelDropoutLinearFn.apply(x, scale, B, self.linear_pred.weight, self.linear_pred.bias)
        return logits.view(B, H, W, self.num_classes).permute(0, 3, 1, 2)


def _mm32(a, b, out, a_t=False, b_t=False, beta=0.0):
    """out (+)= op(a) @ op(b) for float32 2-D views (weight algebra of the folded decoder)."""
    M = a.shape[1] if a_t else a.shape[0]
    Kd = a.shape[0] if a_t else a.shape[1]
    N = b.shape[0] if b_t else b.shape[1]
    return K.gemm(a, b, M=M, N=N, K=Kd, a_kcontig=not a_t, b_kcontig=b_t, lda=K.ld(a), ldb=K.ld(b), out=out,
                  ldc=K.ld(out), beta=beta)


class MLPFoldFn(torch.autograd.Function):
    """DecoderHead's linear_c1..c4 + bilinear resize + cat + linear_fuse + BN + ReLU
    (MLPDecoder.py:59-81), folded: bilinear upsampling (align_corners=False, weights
    summing to one) commutes with 1x1 channel mixing, so

        W_f cat[up(L_4 c_4 + b_4), .., L_1 c_1 + b_1] + b_f = sum_i up((F_i L_i) c_i) + (b_f + sum_i F_i b_i)

    with F_i the column block of W_f that the reference's cat order [c4 | c3 | c2 | c1] gives level i.
    Each level's product W'_i = F_i L_i runs at that level's own resolution with K = C_i, instead of
    a K = 4E GEMM over the concatenated 1/4-resolution map (config 5: 51 GF per image). Gradients of
    the original parameters: G_i = up_i^T(dy0), dW'_i = G_i^T c_i, dc_i = G_i W'_i, dL_i = F_i^T dW'_i,
    dF_i = dW'_i L_i^T + (sum dy0) b_i^T, db_i = F_i^T sum dy0, db_f = sum dy0.
    lvl = (rows_1, L_1, b_1, .., rows_4, L_4, b_4), level 1 the finest."""

    @staticmethod
    def forward(ctx, B, hw, E, bn, sync, wf, bf, gamma, beta, *lvl):
        rows = lvl[0::3]
        Ls, bs = lvl[1::3], lvl[2::3]
        dt = rows[0].dtype
        dev = rows[0].device
        H0, W0 = hw[0]
        wf2 = wf.detach().view(E, 4 * E)
        Fs = [wf2[:, (3 - i) * E:(4 - i) * E] for i in range(4)]
        # W'_i = F_i L_i (float32), b' = b_f + sum_i F_i b_i
        Wp32 = [_mm32(Fs[i], Ls[i].detach(), torch.empty(E, Ls[i].shape[1], device=dev, dtype=torch.float32))
                for i in range(4)]
        bp = torch.empty(1, E, device=dev, dtype=torch.float32)
        for i in range(4):
            K.linear(bs[i].detach().view(1, E), Fs[i], bf.detach() if i == 0 else None, out=bp,
                     beta=0.0 if i == 0 else 1.0)
        Wpc = [w if dt == torch.float32 else K.cast(w, dt) for w in Wp32]
        y0 = K.linear(rows[0], Wpc[0], bp.view(E))
        for i in range(1, 4):
            h, w = hw[i]
            if (h, w) == (H0, W0):
                K.linear(rows[i], Wpc[i], out=y0, beta=1.0)
            else:  # at the level's own resolution, then upsampled into the sum
                K.bilinear(K.linear(rows[i], Wpc[i]), (h, w), (H0, W0), B, out=y0, accumulate=True)
        count = y0.shape[0]
        if bn.training:
            mean, rstd, count = bn_batch_stats(y0, bn, sync)
        else:
            mean, rstd = bn.running_mean, torch.rsqrt(bn.running_var + bn.eps)
        y = K.bn_apply(y0, mean, rstd, gamma, beta, act=2)
        ctx.save_for_backward(y0, y, mean, rstd, gamma, wf, bf, *rows, *Ls, *bs, *Wpc)
        ctx.meta = (B, hw, E, count, sync, bn)
        return y

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "decoder.bwd"
        sv = ctx.saved_tensors
        y0, y, mean, rstd, gamma, wf, bf = sv[:7]
        rows, Ls, bs, Wpc = sv[7:11], sv[11:15], sv[15:19], sv[19:23]
        B, hw, E, count, sync, bn = ctx.meta
        H0, W0 = hw[0]
        dev = y0.device
        dy = K.relu_bwd(dy.contiguous(), y)
        st2, dgamma, dbeta = bn_grad_stats(y0, dy, mean, rstd, bn, sync)
        dy0 = K.bn_bwd_apply(y0, dy, mean, rstd, gamma, st2, count)
        f32 = dict(device=dev, dtype=torch.float32)
        dbf = gslot(bf)
        if dbf is None:
            dbf = torch.empty(E, **f32)
        dWp, drows = [], []
        with K.wgrad_group():  # the four dW'_i as one grouped launch
            for i in range(4):
                h, w = hw[i]
                G = dy0 if (h, w) == (H0, W0) else K.bilinear_bwd(dy0, (h, w), (H0, W0), B)
                if i == 0:  # sum dy0 rides along as the bias gradient of level 1's product
                    dWp.append(K.linear_wgrad(G, rows[i], bias_grad=True, bias_out=dbf)[0])
                else:
                    dWp.append(K.linear_wgrad(G, rows[i]))
                drows.append(K.linear_dgrad(G, Wpc[i]))
        wf2 = wf.detach().view(E, 4 * E)
        dWf = gslot2(wf)
        if dWf is None:
            dWf = torch.empty(E, 4 * E, **f32)
        dLs, dbs = [], []
        for i in range(4):
            Fi = wf2[:, (3 - i) * E:(4 - i) * E]
            L = Ls[i].detach()
            dL = gslot2(Ls[i])
            dLs.append(_mm32(Fi, dWp[i], dL if dL is not None else torch.empty(E, L.shape[1], **f32), a_t=True))
            dFi = dWf[:, (3 - i) * E:(4 - i) * E]
            _mm32(dWp[i], L, dFi, b_t=True)                                 # dW'_i L_i^T
            _mm32(dbf.view(E, 1), bs[i].detach().view(1, E), dFi, beta=1.0)  # + (sum dy0) b_i^T
            dbi = gslot(bs[i])
            dbi = dbi if dbi is not None else torch.empty(E, **f32)
            K.linear_dgrad(dbf.view(1, E), Fi, out=dbi.view(1, E))           # F_i^T sum dy0
            dbs.append(dbi)
        grads = []
        for i in range(4):
            grads += [drows[i], dLs[i].view_as(Ls[i]), dbs[i]]
        return (None, None, None, None, None, dWf.view_as(wf), dbf, dgamma, dbeta, *grads)


# ========================================================================================== loss
class SegLossFn(torch.autograd.Function):
    """CE(bilinear_up(logits), label, ignore_index)[valid].mean() (builder.py:203,230), fused."""

    @staticmethod
    def forward(ctx, logits_rows, B, h, w, label, ignore):
        ncls = logits_rows.shape[1]
        label = label.contiguous()
        H, W = label.shape[-2:]
        ctx.meta = (B, h, w, ncls, ignore)
        if ctx.needs_input_grad[0] and K.seg_loss_grad_partials_size(B, h, w, ncls, H, W):
            # training at an integer factor (4, 8): the gradient's partials come out of the same pass
            out, part = K.seg_loss_fwd_grad(logits_rows, B, h, w, ncls, label, ignore)
            ctx.save_for_backward(part, out)
            ctx.fused, ctx.dtype = True, logits_rows.dtype
        else:
            out = K.seg_loss_fwd(logits_rows, B, h, w, ncls, label, ignore)
            ctx.save_for_backward(logits_rows, label, out)
            ctx.fused = False
        return out[0] / out[1].clamp_min(1.0)

    @staticmethod
    def backward(ctx, g):
        K.TAG = "loss.bwd"
        B, h, w, ncls, ignore = ctx.meta
        gs = g.reshape(1).float().contiguous()
        if ctx.fused:
            part, out = ctx.saved_tensors
            return K.seg_loss_bwd_gather(part, B, h, w, ncls, out, gs, ctx.dtype), None, None, None, None, None
        logits_rows, label, out = ctx.saved_tensors
        dl = K.seg_loss_bwd(logits_rows, B, h, w, ncls, label, out, gscale=gs, ignore=ignore)
        if logits_rows.dtype != torch.float32:
            dl = K.cast(dl, logits_rows.dtype)
        return dl, None, None, None, None, None
