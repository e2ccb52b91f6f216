"""DFormer RGB-D encoder with the reference's module tree, constructor arguments and state_dict
keys (Originofamonia/DFormer models/encoders/DFormer.py), computed by HIP kernels.

Layout: inside a stage the activations are NHWC rows in the compute dtype; the reference's
Block.forward(x [B,H,W,C], x_e [B,H,W,C/2]) -> (x, x_e) surface is kept. nn.Linear / nn.Conv2d
children are parameter containers only (their forward is never called on the hot path).
The stems / stage downsampling (BN + conv3x3 s2, DFormer.py:194-228) run on ConvS2Fn: the BN
statistics on the library's shifted-sum BN kernels, then one gather that folds the BN affine (and
the stem's GELU) into the convolution operand and one MFMA GEMM (csrc/conv.hip), reading the raw
input image and the previous stage's NHWC rows in place (no NCHW<->NHWC permute copies).
"""

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import kernels as K
from .decoders import bn_batch_stats, bn_grad_stats, collectives_on
from .functional import ATTN_PARAM_NAMES, AttentionFn, ConvFFNFn, gslot, invalidate_weights, register_side_stream

_EMPTY = {}


def _empty(dev):
    t = _EMPTY.get(dev)
    if t is None:
        t = _EMPTY[dev] = torch.empty(0, device=dev)
    return t


class LayerNorm(nn.Module):
    """channels_last LayerNorm parameters (DFormer.py:21-45); compute happens inside the fused ops."""

    def __init__(self, normalized_shape, eps=1e-6, data_format="channels_last"):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape))
        self.eps = eps
        self.data_format = data_format
        self.normalized_shape = (normalized_shape,)

    def forward(self, x):  # standalone use (not on the fused path)
        return F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)


class MLP(nn.Module):
    """ConvFFN: LN -> fc1 -> DW3x3 + identity -> GELU -> fc2 (DFormer.py:48-67)."""

    def __init__(self, dim, mlp_ratio=4, norm_cfg=None):
        super().__init__()
        self.norm = LayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, dim * mlp_ratio)
        self.pos = nn.Conv2d(dim * mlp_ratio, dim * mlp_ratio, 3, padding=1, groups=dim * mlp_ratio)
        self.fc2 = nn.Linear(dim * mlp_ratio, dim)
        self.act = nn.GELU()

    def fused(self, x2d, shape, rowscale, layer_scale):
        return ConvFFNFn.apply(x2d, shape, rowscale, self.norm.weight, self.norm.bias, self.fc1.weight,
                               self.fc1.bias, self.pos.weight, self.pos.bias, self.fc2.weight, self.fc2.bias,
                               layer_scale)


class Attention(nn.Module):
    """RGB-D attention (DFormer.py:70-145): conv modulation, pooled-query attention, depth branch."""

    def __init__(self, dim, num_head=8, window=7, norm_cfg=None, drop_depth=False):
        super().__init__()
        self.num_head = num_head
        self.window = window
        self.q = nn.Linear(dim, dim)
        self.q_cut = nn.Linear(dim, dim // 2)
        self.a = nn.Linear(dim, dim)
        self.l = nn.Linear(dim, dim)
        self.conv = nn.Conv2d(dim, dim, 7, padding=3, groups=dim)
        self.e_conv = nn.Conv2d(dim // 2, dim // 2, 7, padding=3, groups=dim // 2)
        self.e_fore = nn.Linear(dim // 2, dim // 2)
        self.e_back = nn.Linear(dim // 2, dim // 2)
        kin = dim * 2 if window != 0 else dim // 2 * 3
        self.proj = nn.Linear(kin, dim)
        if not drop_depth:
            self.proj_e = nn.Linear(kin, dim // 2)
        if window != 0:
            self.short_cut_linear = nn.Linear(dim // 2 * 3, dim // 2)
            self.kv = nn.Linear(dim, dim)
            self.pool = nn.AdaptiveAvgPool2d(output_size=(7, 7))
        self.act = nn.GELU()
        self.norm = LayerNorm(dim, eps=1e-6)
        self.norm_e = LayerNorm(dim // 2, eps=1e-6)
        self.drop_depth = drop_depth

    def fused_params(self, ls1, ls1e):
        e = _empty(self.q.weight.device)
        w = self.window != 0
        d = not self.drop_depth
        vals = dict(n_w=self.norm.weight, n_b=self.norm.bias, ne_w=self.norm_e.weight, ne_b=self.norm_e.bias,
                    wq=self.q.weight, bq=self.q.bias, wqc=self.q_cut.weight, bqc=self.q_cut.bias, wl=self.l.weight,
                    bl=self.l.bias, wconv=self.conv.weight, bconv=self.conv.bias, wa=self.a.weight, ba=self.a.bias,
                    wef=self.e_fore.weight, bef=self.e_fore.bias, wec=self.e_conv.weight, bec=self.e_conv.bias,
                    web=self.e_back.weight, beb=self.e_back.bias,
                    wkv=self.kv.weight if w else e, bkv=self.kv.bias if w else e,
                    wsc=self.short_cut_linear.weight if w else e, bsc=self.short_cut_linear.bias if w else e,
                    wp=self.proj.weight, bp=self.proj.bias,
                    wpe=self.proj_e.weight if d else e, bpe=self.proj_e.bias if d else e,
                    ls1=ls1, ls1e=ls1e if ls1e is not None else e)
        return [vals[n] for n in ATTN_PARAM_NAMES]


_SIDE = {}


def _side_stream(dev):
    """The RGB ConvFFN's stream: independent of the depth branch's ConvFFN (mlp_e2) within a Block, so
    the two overlap (the stage-2/3 kernels alone leave most CUs idle)."""
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
        register_side_stream(s)
    return s


def _drop_path_scale(B, drop_prob, training, dev):
    """mmcv DropPath as a per-sample row scale: floor(keep + U[0,1)) / keep, or None."""
    if drop_prob == 0.0 or not training:
        return None
    keep = 1.0 - drop_prob
    return (keep + torch.rand(B, device=dev)).floor_().div_(keep)


class Block(nn.Module):
    """DFormer Block (DFormer.py:147-181): x + DropPath(ls1 * attn), + DropPath(ls2 * MLP), both branches."""

    def __init__(self, index, dim, num_head, norm_cfg=None, mlp_ratio=4.0, block_index=0, last_block_index=50,
                 window=7, dropout_layer=None, drop_depth=False):
        super().__init__()
        self.index = index
        layer_scale_init_value = 1e-6
        if block_index > last_block_index:
            window = 0
        self.attn = Attention(dim, num_head, window=window, norm_cfg=norm_cfg, drop_depth=drop_depth)
        self.mlp = MLP(dim, int(mlp_ratio), norm_cfg=norm_cfg)
        self.drop_prob = float(dropout_layer.get("drop_prob", 0.0)) if dropout_layer else 0.0
        self.layer_scale_1 = nn.Parameter(layer_scale_init_value * torch.ones(dim))
        self.layer_scale_2 = nn.Parameter(layer_scale_init_value * torch.ones(dim))
        if not drop_depth:
            self.layer_scale_1_e = nn.Parameter(layer_scale_init_value * torch.ones(dim // 2))
            self.layer_scale_2_e = nn.Parameter(layer_scale_init_value * torch.ones(dim // 2))
            self.mlp_e2 = MLP(dim // 2, int(mlp_ratio))
        self.drop_depth = drop_depth
        self.drop_path_masks = None  # tests may inject the 4 per-sample keep masks (mmcv call order)
        self._row_scales = None  # [4, B] DropPath scales drawn for the whole backbone by DFormer.forward

    def forward(self, x, x_e):
        B, H, W, C = x.shape
        shape = (B, H, W)
        xr = x.reshape(B * H * W, C)
        xer = x_e.reshape(B * H * W, C // 2)
        if self.drop_path_masks is not None and self.training and self.drop_prob > 0:
            keep = 1.0 - self.drop_prob
            rs = [m.to(device=x.device, dtype=torch.float32) / keep for m in self.drop_path_masks]
        elif self._row_scales is not None:
            rs = list(self._row_scales.unbind(0))
            self._row_scales = None
        else:
            rs = [_drop_path_scale(B, self.drop_prob, self.training, x.device) for _ in range(4)]
        ls1e = self.layer_scale_1_e if not self.drop_depth else None
        st = getattr(self, "stage", "s?")
        K.TAG = st + ".attn"
        x1, xe1 = AttentionFn.apply(xr, xer, shape, self.attn.num_head, self.attn.window, self.drop_depth, rs[0],
                                    rs[2], *self.attn.fused_params(self.layer_scale_1, ls1e))
        if self.drop_depth:
            K.TAG = st + ".mlp"
            x2 = self.mlp.fused(x1, shape, rs[1], self.layer_scale_2)
            return x2.view(B, H, W, C), xe1.view(B, H, W, C // 2)  # DFormer.py:177-181: e_back's output
        # the RGB and depth ConvFFNs are independent: the RGB one runs on a side stream (and so does its
        # backward: autograd replays a node on its forward's stream) while the depth one runs on the
        # step's stream; the overlap fills the GPU at the late stages where each kernel alone is
        # latency-bound. (RGB on the side: 491.8 / 491.0 vs 488.2 / 487.8 images/s with the depth
        # ConvFFN there — the side stream's kernels get the smaller share of the CUs, and the join waited
        # 2.3 ms per step on the depth ConvFFN finishing after the RGB one, profiles/r06_queue_analysis.txt)
        side = _side_stream(x.device) if x1.is_cuda else None
        if side is not None:
            main = torch.cuda.current_stream(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                K.TAG = st + ".mlp"
                x2 = self.mlp.fused(x1, shape, rs[1], self.layer_scale_2)
            x1.record_stream(side)
            K.TAG = st + ".mlp_e2"
            xe2 = self.mlp_e2.fused(xe1, shape, rs[3], self.layer_scale_2_e)
            main.wait_stream(side)
            x2.record_stream(main)
        else:
            K.TAG = st + ".mlp"
            x2 = self.mlp.fused(x1, shape, rs[1], self.layer_scale_2)
            K.TAG = st + ".mlp_e2"
            xe2 = self.mlp_e2.fused(xe1, shape, rs[3], self.layer_scale_2_e)
        return x2.view(B, H, W, C), xe2.view(B, H, W, C // 2)


def _bn(c, syncbn):
    return nn.SyncBatchNorm(c) if syncbn else nn.BatchNorm2d(c)


class BNRowsFn(torch.autograd.Function):
    """BatchNorm2d / SyncBatchNorm (DFormer.py:219-228 stems and downsample layers) on a
    channels-last NCHW tensor, computed as [B*H*W, C] rows by the library's BN kernels: batch
    statistics + running-stat update in training (all-reduced for SyncBN), running stats in eval."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn, sync):
        B, C, H, W = x.shape
        xr = x.permute(0, 2, 3, 1).contiguous().view(-1, C)
        rows = xr.shape[0]
        if bn.training:
            mean, rstd, count = bn_batch_stats(xr, bn, sync)
        else:
            mean = bn.running_mean
            rstd = torch.rsqrt(bn.running_var + bn.eps)
            count = rows
        y = K.bn_apply(xr, mean, rstd, gamma, beta)
        ctx.save_for_backward(xr, mean, rstd, gamma)
        ctx.sync, ctx.count, ctx.shape, ctx.bn = sync, count, (B, C, H, W), bn
        ctx.training = bn.training
        return y.view(B, H, W, C).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        K.TAG = "down.bwd"
        xr, mean, rstd, gamma = ctx.saved_tensors
        B, C, H, W = ctx.shape
        dyr = dy.permute(0, 2, 3, 1).contiguous().view(-1, C)
        st2, dgamma, dbeta = bn_grad_stats(xr, dyr, mean, rstd, ctx.bn, ctx.sync)
        if ctx.training:
            dx = K.bn_bwd_apply(xr, dyr, mean, rstd, gamma, st2, ctx.count)
        else:  # running statistics: BN is a fixed per-channel affine
            dx = K.scale_mul(dyr, colscale=rstd * gamma)
        return dx.view(B, H, W, C).permute(0, 3, 1, 2), dgamma, dbeta, None, None


class ConvS2Fn(torch.autograd.Function):
    """nn.Conv2d(cin, cout, 3, stride 2, pad 1) [preceded by BatchNorm / SyncBatchNorm [+ GELU]]
    (DFormer.py:194-228: stem conv -> BN -> GELU -> conv; stage i>0: BN -> conv) on the library's
    kernels: the BN statistics over the input rows, then ONE gather that applies the BN affine and
    GELU on the fly (csrc/conv.hip) and ONE MFMA GEMM with the conv bias in its epilogue. x is any
    NCHW-logical tensor (raw image, the depth-channel view, or the previous stage's NHWC rows);
    returns NHWC rows [B*Ho*Wo, cout] in the compute dtype. Backward: weight / bias gradients
    from the saved gathered operand, input gradient by the transposed GEMM + deterministic
    col2im with GELU' recomputed, then the BN backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, bn_w, bn_b, bn, sync, gelu, dt):
        B, C, H, W = x.shape
        cout = weight.shape[0]
        kp = K.conv3s2_kp(C)
        aff = None
        count = None
        xr = None
        if bn is not None:
            xr = x.permute(0, 2, 3, 1).reshape(B * H * W, C)  # the NHWC rows (a view for channels-last x)
            if bn.training:
                mean, rstd, count = bn_batch_stats(xr, bn, sync)
            else:
                mean = bn.running_mean
                rstd = torch.rsqrt(bn.running_var + bn.eps)
                count = xr.shape[0]
            aff = (mean, rstd, bn_w.detach(), bn_b.detach())
        cols = K.conv3s2_im2col(x, dt, bn=aff, gelu=gelu)
        wp = K.conv3_weight_pack(weight.detach(), dt, kp)
        y = K.linear(cols, wp, bias.detach())
        ctx.shape, ctx.cin, ctx.sync, ctx.gelu, ctx.count = (B, H, W), C, sync, gelu, count
        ctx.has_bn = bn is not None
        ctx.bn = bn
        ctx.training = bn is not None and bn.training
        ctx.x_dtype = x.dtype
        ctx.tag = K.TAG
        ctx.save_for_backward(cols, wp, weight, bias, xr if xr is not None else x.new_empty(0),
                              *(aff if aff is not None else ()))
        return y

    @staticmethod
    def backward(ctx, dy):
        K.TAG = ctx.tag + ".bwd"
        cols, wp, weight, bias, xr, *aff = ctx.saved_tensors
        dy = dy.contiguous()
        cin = ctx.cin
        dwp, db = K.linear_wgrad(dy, cols, bias_grad=True, bias_out=gslot(bias))
        dw = K.conv3_weight_unpack(dwp, cin, dw=gslot(weight))
        dx = dgamma = dbeta = None
        if not ctx.has_bn:
            if ctx.needs_input_grad[0]:  # gradient w.r.t. the image (parity tests); not on the training path
                dx = K.conv3s2_col2im_nchw(K.linear_dgrad(dy, wp), ctx.shape, cin, ctx.x_dtype)
        elif ctx.needs_input_grad[0] or ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
            dcols = K.linear_dgrad(dy, wp)
            mean, rstd, gamma, beta = aff
            dz = K.conv3s2_col2im(dcols, ctx.shape, cin, x=xr, bn=aff if ctx.gelu else None, gelu=ctx.gelu)
            st2, dgamma, dbeta = bn_grad_stats(xr, dz, mean, rstd, ctx.bn, ctx.sync)
            if ctx.needs_input_grad[0]:
                B, H, W = ctx.shape
                if ctx.training:
                    dx = K.bn_bwd_apply(xr, dz, mean, rstd, gamma, st2, ctx.count)
                else:  # running statistics: BN is a fixed per-channel affine
                    dx = K.scale_mul(dz, colscale=rstd * gamma)
                dx = dx.view(B, H, W, cin).permute(0, 3, 1, 2)
        return dx, dw, db, dgamma, dbeta, None, None, None, None


# The stem / downsample layers run natively: 3x3 stride-2 convs as gather + MFMA GEMM with their
# BatchNorms (+ GELU) folded into the gather (ConvS2Fn), the stem's last BN on BNRowsFn. There is no
# vendor-convolution path.


def _run_downsample_native(seq, x, dt):
    """The reference's downsample nn.Sequential (stem: Conv, BN, GELU, Conv, BN; stage: BN, Conv)
    on ConvS2Fn / BNRowsFn. Returns the NCHW-logical view of channels-last rows."""
    mods = list(seq)
    i, pend_bn, pend_gelu = 0, None, False
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            if i == len(mods) - 1:  # trailing BN of the stem: applied to the conv output rows
                x = BNRowsFn.apply(x, m.weight, m.bias, m, isinstance(m, nn.SyncBatchNorm))
            else:
                pend_bn = m
        elif isinstance(m, nn.GELU):
            assert pend_bn is not None
            pend_gelu = True
        else:
            assert isinstance(m, nn.Conv2d) and m.kernel_size == (3, 3) and m.stride == (2, 2) and m.padding == (1, 1)
            B, _, H, W = x.shape
            bn = pend_bn
            y = ConvS2Fn.apply(x, m.weight, m.bias, bn.weight if bn is not None else None,
                               bn.bias if bn is not None else None, bn, isinstance(bn, nn.SyncBatchNorm), pend_gelu,
                               dt)
            Ho, Wo = (H + 1) // 2, (W + 1) // 2
            x = y.view(B, Ho, Wo, m.out_channels).permute(0, 3, 1, 2)
            pend_bn, pend_gelu = None, False
        i += 1
    return x


class DFormer(nn.Module):
    """DFormer backbone (DFormer.py:184-305). forward(x, x_e) -> (outs[4] NCHW views, None) like the
    reference; outs are channels-last buffers in the compute dtype."""

    def __init__(self, in_channels=4, depths=(2, 2, 8, 2), dims=(32, 64, 128, 256), out_indices=(0, 1, 2, 3),
                 windows=(7, 7, 7, 7), norm_cfg=None, mlp_ratios=(8, 8, 4, 4), num_heads=(2, 4, 10, 16),
                 last_block=(50, 50, 50, 50), drop_path_rate=0.1, init_cfg=None):
        super().__init__()
        syncbn = bool(norm_cfg) and norm_cfg.get("type") == "SyncBN" and collectives_on()
        self.depths = depths
        self.dims = dims
        self.mlp_ratios = mlp_ratios
        self.out_indices = out_indices
        self.compute_dtype = torch.float32
        self.downsample_layers = nn.ModuleList()
        self.downsample_layers.append(nn.Sequential(
            nn.Conv2d(3, dims[0] // 2, 3, 2, 1), nn.BatchNorm2d(dims[0] // 2), nn.GELU(),
            nn.Conv2d(dims[0] // 2, dims[0], 3, 2, 1), nn.BatchNorm2d(dims[0])))
        # unused by the reference forward (DFormer.py:202-203, 287-291); kept for state_dict parity
        self.stem_e_fc1 = nn.Linear(360, 640)
        self.stem_e_fc2 = nn.Linear(1, 480)
        self.downsample_layers_e = nn.ModuleList()
        self.downsample_layers_e.append(nn.Sequential(
            nn.Conv2d(1, dims[0] // 4, 3, 2, 1), nn.BatchNorm2d(dims[0] // 4), nn.GELU(),
            nn.Conv2d(dims[0] // 4, dims[0] // 2, 3, 2, 1), nn.BatchNorm2d(dims[0] // 2)))
        for i in range(len(dims) - 1):
            self.downsample_layers.append(nn.Sequential(_bn(dims[i], syncbn),
                                                        nn.Conv2d(dims[i], dims[i + 1], 3, 2, 1)))
            self.downsample_layers_e.append(nn.Sequential(_bn(dims[i] // 2, syncbn),
                                                          nn.Conv2d(dims[i] // 2, dims[i + 1] // 2, 3, 2, 1)))
        self.stages = nn.ModuleList()
        dp_rates = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        cur = 0
        for i in range(len(dims)):
            self.stages.append(nn.Sequential(*[
                Block(index=cur + j, dim=dims[i], window=windows[i],
                      dropout_layer=dict(type="DropPath", drop_prob=dp_rates[cur + j]), num_head=num_heads[i],
                      norm_cfg=norm_cfg, block_index=depths[i] - j, last_block_index=last_block[i],
                      mlp_ratio=mlp_ratios[i], drop_depth=((i == 3) & (j == depths[i] - 1)))
                for j in range(depths[i])]))
            for blk in self.stages[-1]:
                blk.stage = f"s{i}"
            cur += depths[i]
        for p in (self.stem_e_fc1.weight, self.stem_e_fc1.bias, self.stem_e_fc2.weight, self.stem_e_fc2.bias):
            p.requires_grad_(False)  # never used: excluded from gradients (and DDP buckets)

    def load_state_dict(self, *a, **k):
        r = super().load_state_dict(*a, **k)
        invalidate_weights()
        return r

    def _draw_drop_path(self, B, dev):
        """mmcv DropPath scales floor(keep + U[0,1)) / keep for all four DropPath calls of every
        Block, drawn by one RNG launch for the whole backbone instead of four per Block."""
        blocks = [b for st in self.stages for b in st]
        if not self.training or all(b.drop_prob == 0.0 for b in blocks):
            return
        keep = getattr(self, "_keep", None)
        if keep is None or keep.device != dev:
            keep = self._keep = torch.tensor([1.0 - b.drop_prob for b in blocks], device=dev).view(-1, 1, 1)
        rs = (keep + torch.rand(len(blocks), 4, B, device=dev)).floor_().div_(keep)
        for b, r in zip(blocks, rs.unbind(0)):
            b._row_scales = r if b.drop_prob > 0 else None

    def _downsample(self, i, x, e):
        if not x.is_cuda:
            raise RuntimeError("dformer_amd runs on the HIP library only (tensors must be on the GPU)")
        dt = self.compute_dtype
        seq_e = self.downsample_layers_e[i]
        if any(isinstance(m, nn.SyncBatchNorm) for m in seq_e):
            return (_run_downsample_native(self.downsample_layers[i], x, dt),
                    _run_downsample_native(seq_e, e, dt))
        # the two branches' stems / downsamples are independent: the depth one runs on the side
        # stream (its backward too) next to the RGB one on the step's stream (same box, alternated:
        # 506.2 / 509.8 vs 503.3 / 500.2 images/s; SyncBN keeps both on the step's stream)
        side, main = _side_stream(x.device), torch.cuda.current_stream(x.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            e2 = _run_downsample_native(seq_e, e, dt)
        e.record_stream(side)
        x2 = _run_downsample_native(self.downsample_layers[i], x, dt)
        main.wait_stream(side)
        e2.record_stream(main)
        return x2, e2

    def forward(self, x, x_e):
        if x_e is None:
            x_e = x
        if x.dim() == 3:
            x = x.unsqueeze(0)
        if x_e.dim() == 3:
            x_e = x_e.unsqueeze(2)
        x_e = x_e[:, 0:1]
        dt = self.compute_dtype
        self._draw_drop_path(x.shape[0], x.device)
        outs = []
        for i in range(4):
            K.TAG = f"s{i}.down"
            x, x_e = self._downsample(i, x, x_e)
            xh = x.permute(0, 2, 3, 1).to(dt).contiguous()
            eh = x_e.permute(0, 2, 3, 1).to(dt).contiguous()
            for blk in self.stages[i]:
                xh, eh = blk(xh, eh)
            x = xh.permute(0, 3, 1, 2)  # NCHW view of the channels-last buffer
            x_e = eh.permute(0, 3, 1, 2)
            outs.append(x)
        return outs, None


def DFormer_Tiny(pretrained=False, **kwargs):
    return DFormer(dims=[32, 64, 128, 256], mlp_ratios=[8, 8, 4, 4], depths=[3, 3, 5, 2], num_heads=[1, 2, 4, 8],
                   windows=[0, 7, 7, 7], **kwargs)


def DFormer_Small(pretrained=False, **kwargs):
    return DFormer(dims=[64, 128, 256, 512], mlp_ratios=[8, 8, 4, 4], depths=[2, 2, 4, 2], num_heads=[1, 2, 4, 8],
                   windows=[0, 7, 7, 7], **kwargs)


def DFormer_Base(pretrained=False, drop_path_rate=0.1, **kwargs):
    return DFormer(dims=[64, 128, 256, 512], mlp_ratios=[8, 8, 4, 4], depths=[3, 3, 12, 2], num_heads=[1, 2, 4, 8],
                   windows=[0, 7, 7, 7], drop_path_rate=drop_path_rate, **kwargs)


def DFormer_Large(pretrained=False, drop_path_rate=0.1, **kwargs):
    return DFormer(dims=[96, 192, 288, 576], mlp_ratios=[8, 8, 4, 4], depths=[3, 3, 12, 2], num_heads=[1, 2, 4, 8],
                   windows=[0, 7, 7, 7], drop_path_rate=drop_path_rate, **kwargs)
