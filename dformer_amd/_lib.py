"""ctypes binding of libdformer_hip.so (the C ABI declared in include/dformer_hip.h).

This is the only place Python touches the native library. Every wrapper takes torch tensors
that already live on the GPU, passes raw pointers + sizes + the current HIP stream, and
raises RuntimeError with the library's message on a non-zero status. There is no CPU
fallback: if the library is missing the import fails loudly.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DFM_LIB_PATH: load another build of the library (profiling A/B of compile-time variants only)
LIB_PATH = os.environ.get("DFM_LIB_PATH") or os.path.join(_HERE, "libdformer_hip.so")

F32, BF16, F16 = 0, 1, 2

c_int, c_long, c_float, c_double, c_void_p, c_size_t = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                                         ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t)
P = c_void_p


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
                ("a_kcontig", c_int), ("b_kcontig", c_int),
                ("lda", c_long), ("ldb", c_long), ("ldc", c_long),
                ("stride_a", c_long), ("stride_b", c_long), ("stride_c", c_long),
                ("alpha", c_float), ("beta", c_float), ("c_f32", c_int),
                ("bias", P), ("act", c_int), ("preact", P), ("ldpre", c_long),
                ("mul", P), ("ldmul", c_long), ("res", P), ("ldres", c_long),
                ("colscale", P), ("rowscale", P), ("rows_per_scale", c_long), ("split_k", c_int),
                ("act_col0", c_int), ("colsum", P), ("colsum_accumulate", c_int), ("mul_gelu_grad", c_int),
                ("workspace_bytes", ctypes.c_long),
                ("mul2", P), ("ldmul2", c_long), ("out2", P), ("ldout2", c_long)]


class PartialSum(ctypes.Structure):
    """DfmPartialSum: a deferred reduction second stage (dfm_partial_sum_group)."""
    _fields_ = [("part", P), ("out0", P), ("out1", P), ("n", c_long), ("n0", c_long), ("nblk", c_int),
                ("layout", c_int), ("accumulate", c_int)]


class ConvFFNDesc(ctypes.Structure):
    """DfmConvFFNDesc: shape of one fused ConvFFN call."""
    _fields_ = [("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("hidden", c_int), ("ln_eps", c_float)]


class BlockDesc(ctypes.Structure):
    """DfmBlockDesc: one encoder Block (dfm_block_fwd / dfm_block_bwd)."""
    _fields_ = [("B", c_int), ("H", c_int), ("W", c_int), ("C", c_int), ("heads", c_int), ("window", c_int),
                ("hidden", c_int), ("drop_depth", c_int), ("fused_ffn", c_int), ("ln_eps", c_float)]


# the DFM_BP_* indices of dfm_block_fwd's parameter array: the reference Block's state_dict keys
# (DFormer.py:70-181) in the header's enum order
BLOCK_PARAM_NAMES = (
    "attn.norm.weight", "attn.norm.bias", "attn.norm_e.weight", "attn.norm_e.bias",
    "attn.q.weight", "attn.q.bias", "attn.q_cut.weight", "attn.q_cut.bias", "attn.l.weight", "attn.l.bias",
    "attn.conv.weight", "attn.conv.bias", "attn.a.weight", "attn.a.bias", "attn.e_fore.weight", "attn.e_fore.bias",
    "attn.e_conv.weight", "attn.e_conv.bias", "attn.e_back.weight", "attn.e_back.bias", "attn.kv.weight",
    "attn.kv.bias", "attn.short_cut_linear.weight", "attn.short_cut_linear.bias", "attn.proj.weight",
    "attn.proj.bias", "attn.proj_e.weight", "attn.proj_e.bias",
    "layer_scale_1", "layer_scale_1_e", "layer_scale_2", "layer_scale_2_e",
    "mlp.norm.weight", "mlp.norm.bias", "mlp.fc1.weight", "mlp.fc1.bias", "mlp.pos.weight", "mlp.pos.bias",
    "mlp.fc2.weight", "mlp.fc2.bias",
    "mlp_e2.norm.weight", "mlp_e2.norm.bias", "mlp_e2.fc1.weight", "mlp_e2.fc1.bias", "mlp_e2.pos.weight",
    "mlp_e2.pos.bias", "mlp_e2.fc2.weight", "mlp_e2.fc2.bias")
# entries passed in the activation dtype (nn.Linear weights); every other entry is float32
BLOCK_GEMM_WEIGHTS = frozenset(n for n in BLOCK_PARAM_NAMES if n.endswith(".weight") and any(
    k in n for k in (".q.", ".q_cut.", ".l.", ".a.", ".e_fore.", ".e_back.", ".kv.", ".short_cut_linear.", ".proj.",
                     ".proj_e.", ".fc1.", ".fc2.")))


# name -> (restype, argtypes)
_SIGS = {
    "dfm_last_error": (ctypes.c_char_p, []),
    "dfm_abi_version": (c_int, []),
    "dfm_build_tag": (ctypes.c_char_p, []),
    "dfm_gemm_workspace_size": (c_size_t, [ctypes.POINTER(GemmDesc)]),
    "dfm_gemm": (c_int, [c_int, ctypes.POINTER(GemmDesc), P, P, P, P, P]),
    "dfm_gemm_group_workspace_size": (c_size_t, [c_int, ctypes.POINTER(GemmDesc)]),
    "dfm_gemm_group": (c_int, [c_int, c_int, ctypes.POINTER(GemmDesc), P, P, P, P, P]),
    "dfm_layernorm_fwd": (c_int, [c_int, c_long, c_int, P, c_long, P, P, c_float, P, c_long, P, P, P]),
    "dfm_layernorm_bwd_workspace": (c_size_t, [c_long, c_int]),
    "dfm_layernorm_bwd": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, P, P, P, c_long, P, c_long, c_int,
                                  P, P, P, P, P]),
    "dfm_residual_bwd_workspace": (c_size_t, [c_long, c_int]),
    "dfm_residual_bwd": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, P, c_long, P, c_long, P, P, P, P]),
    "dfm_dwconv_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, P, c_int, P, c_long, P, c_long,
                               P]),
    "dfm_dwconv_bwd_data": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_int, P, c_long,
                                    c_int, P]),
    "dfm_dwconv_bwd_weight_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "dfm_dwconv_bwd_weight": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, P,
                                      P]),
    "dfm_dwconv_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_int, P, c_long,
                               c_int, P, P, P, P, P]),
    "dfm_partial_sum_group": (c_int, [c_int, P, P]),
    "dfm_convffn_supported": (c_int, [c_int, ctypes.POINTER(ConvFFNDesc)]),
    "dfm_convffn_fwd": (c_int, [c_int, ctypes.POINTER(ConvFFNDesc)] + [P] * 20),
    "dfm_convffn_bwd_workspace_size": (c_size_t, [c_int, ctypes.POINTER(ConvFFNDesc)]),
    "dfm_convffn_bwd": (c_int, [c_int, ctypes.POINTER(ConvFFNDesc)] + [P] * 26 + [c_size_t, P]),
    "dfm_block_saved_size": (c_size_t, [c_int, ctypes.POINTER(BlockDesc)]),
    "dfm_block_workspace_size": (c_size_t, [c_int, ctypes.POINTER(BlockDesc)]),
    "dfm_block_fwd": (c_int, [c_int, ctypes.POINTER(BlockDesc), P, P, P, P, P, P, P, c_size_t, P, c_size_t, P]),
    "dfm_block_bwd": (c_int, [c_int, ctypes.POINTER(BlockDesc), P, P, P, P, P, c_size_t, P, P, P, P, P, P, c_size_t,
                              P]),
    "dfm_group_scale": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, c_long, P]),
    "dfm_nmf_update_mm": (c_int, [c_int, c_long, c_int, P, P, P, c_float, P, P, P, c_int, P]),
    "dfm_nmf_update_bwd_mm": (c_int, [c_int, c_long, c_int, P, P, P, P, P, P, P, c_float, P, P, c_int, P, P, P,
                                      c_int, P]),
    "dfm_nmf_saved_size": (c_size_t, [c_int, c_int, c_long, c_long, c_int, c_int]),
    "dfm_nmf_fwd_workspace_size": (c_size_t, [c_int, c_int, c_long, c_long, c_int, c_int]),
    "dfm_nmf_bwd_workspace_size": (c_size_t, [c_int, c_int, c_long, c_long, c_int, c_int]),
    "dfm_nmf_fwd": (c_int, [c_int, c_int, c_long, c_long, c_int, c_int, c_float, P, P, P, P, c_long, P, c_long, P]),
    "dfm_nmf_bwd": (c_int, [c_int, c_int, c_long, c_long, c_int, c_int, c_float, P, P, P, c_long, P, P, P, c_long,
                            P]),
    "dfm_colsum_workspace": (c_size_t, [c_long, c_int]),
    "dfm_colsum": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, c_long, P, c_int, P, P]),
    "dfm_cast": (c_int, [c_int, c_int, c_long, P, P, P]),
    "dfm_pack_slices": (c_int, [c_int, c_int, P, P, c_long, c_int, P, P]),
    "dfm_gelu_bwd": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, c_long, c_int, P]),
    "dfm_scale_mul": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, P, c_long, c_float, P, c_long, c_int,
                              P]),
    "dfm_dual_mul": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, c_long, P, c_long, P, c_long, P]),
    "dfm_adaptive_pool7_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P]),
    "dfm_adaptive_pool7_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, c_int, P]),
    "dfm_bilinear_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, c_int, P]),
    "dfm_bilinear_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, c_int, P]),
    "dfm_pooled_attn_workspace": (c_size_t, [c_int, c_int, c_int, c_int]),
    "dfm_pooled_attn_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, P, c_long, c_float, P, c_long,
                                    P, P, P]),
    "dfm_pooled_attn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, P, c_long, c_float, P, c_long,
                                    P, c_long, P, P, P, P, c_long, P, P]),
    "dfm_bn_workspace": (c_size_t, [c_long, c_int]),
    "dfm_bn_stats": (c_int, [c_int, c_long, c_int, P, c_long, P, P, P]),
    "dfm_bn_finalize": (c_int, [c_int, P, c_double, c_float, c_float, P, P, P, P, P]),
    "dfm_bn_merge": (c_int, [c_int, c_int, P, P, P, P]),
    "dfm_bn_apply": (c_int, [c_int, c_long, c_int, P, c_long, P, P, P, P, P, c_long, c_int, P, c_long, P]),
    "dfm_bn_bwd_stats": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, P, P, P, P]),
    "dfm_bn_bwd_apply": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, P, P, P, c_double, P, c_long, c_int,
                                 P]),
    "dfm_relu_bwd": (c_int, [c_int, c_long, c_int, P, c_long, P, c_long, P, c_long, P]),
    "dfm_conv3s2_im2col": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_long, c_long, c_long, P, P, P,
                                   P, P, c_int, c_int, P, P]),
    "dfm_conv3s2_col2im": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, P, P, P, c_int, P,
                                   c_long, c_int, P]),
    "dfm_conv3s2_col2im_nchw": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, c_long, P, c_long, c_long,
                                        c_long, c_long, P]),
    "dfm_conv3_weight_pack": (c_int, [c_int, c_int, c_int, c_int, P, P, P]),
    "dfm_conv3_weight_unpack": (c_int, [c_int, c_int, c_int, P, P, c_int, P]),
    "dfm_resize_nchw": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_long, c_long, c_long, c_long, P, c_int,
                                c_int, c_int, c_int, P, P]),
    "dfm_msf_accumulate": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, c_int, c_int, c_int, c_int, c_int,
                                   P, P]),
    "dfm_seg_confusion": (c_int, [c_long, c_int, P, P, c_int, P, P]),
    "dfm_nmf_update": (c_int, [c_long, P, P, P, c_float, P, P, c_int, P]),
    "dfm_nmf_update_bwd": (c_int, [c_long, P, P, P, P, P, c_float, P, c_int, P, P, P, c_int, P]),
    "dfm_grad_nonfinite": (c_int, [c_long, P, P, P]),
    "dfm_softmax_rows": (c_int, [c_long, c_int, P, P, P]),
    "dfm_softmax_rows_bwd": (c_int, [c_long, c_int, P, P, P, c_int, P]),
    "dfm_seg_loss_workspace": (c_size_t, [c_int, c_int, c_int]),
    "dfm_seg_loss_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, c_int, P, P, P, P]),
    "dfm_seg_loss_bwd_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "dfm_seg_loss_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, c_int, P, P, P, P, P, P]),
    "dfm_seg_loss_grad_partials_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "dfm_seg_loss_fwd_grad": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, c_int, P, P, P]),
    "dfm_seg_loss_bwd_gather": (c_int, [c_int, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "dfm_adamw": (c_int, [c_long, P, P, P, P, c_float, c_float, c_float, c_float, c_float, c_int, c_float, P, c_int,
                          P]),
    "dfm_adamw_dev": (c_int, [c_long, P, P, P, P, P, c_float, c_float, c_float, c_float, c_float, P, c_int, P]),
    "dfm_adamw_amp": (c_int, [c_long, P, P, P, P, P, P, P, c_float, c_float, c_float, c_float, c_float, P, c_int, P]),
    "dfm_loss_scale_update": (c_int, [P, P, c_float, c_float, c_int, P]),
    "dfm_trace_set": (c_int, [c_int, ctypes.c_char_p]),
    "dfm_trace_take": (c_int, [ctypes.POINTER(c_void_p), c_int]),
    "dfm_trace_read": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_float), c_int]),
    "dfm_kernel_name": (ctypes.c_char_p, [c_void_p]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"dformer_amd: native library missing at {LIB_PATH}; run "
                          f"`python -c 'import __graft_entry__ as g; g.build()'` (make -C dformer_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()
SYMBOLS = tuple(_SIGS)
BUILD_TAG = lib.dfm_build_tag().decode()


def check(status, what):
    if status != 0:
        raise RuntimeError(f"{what} failed ({status}): {lib.dfm_last_error().decode()}")


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float16:
        return F16
    raise TypeError(f"dformer_amd: unsupported dtype {t.dtype}")


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream
