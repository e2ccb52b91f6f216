/* dformer_hip.h — C ABI of libdformer_hip.so, the MI355X (gfx950) kernels behind DFormer's
 * encoder Block and segmentation decoders.
 *
 * Contract:
 *   - plain pointers (device memory) + sizes/strides in ELEMENTS; no torch types;
 *   - the caller owns every buffer, including workspaces (query the *_workspace functions);
 *     the library never allocates, never synchronises the host, and only enqueues on `stream`
 *     (a hipStream_t passed as void*; NULL = default stream);
 *   - return 0 on success, negative on bad arguments / unsupported dtype / launch failure;
 *     dfm_last_error() returns a thread-local message for the last failure;
 *   - dtype selects the storage type of activations: DFM_F32, DFM_BF16 or DFM_F16 (IEEE half,
 *     the reference's torch.autocast(float16) path, utils/train.py:289). Statistics,
 *     accumulators, LayerNorm / BatchNorm affine params, biases, depthwise weights and
 *     gradients of parameters are always float32.
 *   - layouts are NHWC ("channels-last"): pixel p of image b at row (b*H + h)*W + w,
 *     channel c at column c; `ld*` is the row (pixel) stride so column slices of a wider
 *     buffer can be read and written in place.
 *
 * Each entry point names the reference operation it replaces (file:line in
 * Originofamonia/DFormer).
 */
#ifndef DFORMER_HIP_H
#define DFORMER_HIP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFM_OK 0
#define DFM_ERR_ARG (-1)
#define DFM_ERR_DTYPE (-2)
#define DFM_ERR_LAUNCH (-3)

#define DFM_F32 0
#define DFM_BF16 1
#define DFM_F16 2

typedef void* dfm_stream_t;

const char* dfm_last_error(void);
int dfm_abi_version(void); /* 13: DfmGemmDesc.mul2 / out2 (second epilogue output); 12: dfm_build_tag; 11: dfm_block_fwd / dfm_block_bwd (+ dfm_block_saved_size /
                              dfm_block_workspace_size); 10: dfm_convffn_fwd / dfm_convffn_bwd (fused ConvFFN); 9: dfm_nmf_fwd / dfm_nmf_bwd (+ dfm_nmf_saved_size); 8: deferred reduction
                              second stages (dfm_partial_sum_group); 7: DfmGemmDesc.workspace_bytes + stride /
                              leading-dimension validation */
/* The build this process loaded: "default" (or a variant build's DFM_BUILD_TAG) and its compile-time
 * reduction geometry, e.g. "default red=512x256" (at most 512 column-reduction blocks of >= 256 rows). */
const char* dfm_build_tag(void);

/* ---------------------------------------------------------------- launch tracer (measurement)
 * Off by default (one branch per launch). DFM_TRACE_RECORD: every kernel the library enqueues is
 * recorded (dfm_trace_take returns and clears them: the kernels one entry point launched);
 * DFM_TRACE_TIME: launches of the kernel(s) whose demangled name is `probe_name` (several names separated
 * by '\n'; NULL or "" = every
 * kernel) are bracketed by HIP events on their own stream; dfm_trace_read synchronises on the last
 * event and returns per-launch milliseconds. dfm_kernel_name: the demangled name rocprofv3 prints.
 * Used by bench.py (per-kernel FLOP/byte accounting and the dominant kernel's live roofline). */
#define DFM_TRACE_RECORD 1
#define DFM_TRACE_TIME 2
int dfm_trace_set(int flags, const char* probe_name);
int dfm_trace_take(const void** funcs, int max);
int dfm_trace_read(const void** funcs, float* ms, int max);
const char* dfm_kernel_name(const void* func);

/* ---------------------------------------------------------------- GEMM (MFMA)
 * C[b][m][n] = epilogue( alpha * sum_k A(b,m,k) * B(b,k,n) )
 *   A(m,k) = A[m*lda + k] if a_kcontig else A[k*lda + m]
 *   B(k,n) = B[n*ldb + k] if b_kcontig else B[k*ldb + n]
 * Replaces every nn.Linear / 1x1 conv / torch.bmm on the hot path:
 *   DFormer.py:76-95 (q, q_cut, a, l, kv, e_fore, e_back, proj, proj_e, short_cut_linear),
 *   DFormer.py:53-55 (fc1, fc2), ham_head.py:46-145 (NMF bmm), ham_head.py:156-220 (1x1
 *   ConvModules), decode_head.py:104 (conv_seg), MLPDecoder.py:14-57 (linear_c*, fuse, pred),
 *   and their backward (dX = dY W: a_kcontig=1,b_kcontig=0; dW = dY^T X: both 0, split_k).
 * Epilogue, in order (each optional):
 *   v += beta * C_old ; v += bias[n] ; [n >= act_col0: preact[m,n-act_col0] = v ; v = act(v)
 *   (1 gelu, 2 relu, 3 gelu with preact[m,n-act_col0] = gelu'(v) instead of v: the GELU
 *   backward becomes a plain product)] ;
 *   v *= mul[m,n] ; v = res[m,n] + colscale[n] * rowscale[m / rows_per_scale] * v ;
 *   C[m,n] = v (stored as dtype, or float32 when c_f32).
 * Operands A, B, mul, res, preact are `dtype`; C is dtype or float32 (c_f32).
 */
typedef struct DfmGemmDesc {
  int M, N, K;
  int batch;
  int a_kcontig, b_kcontig;
  long lda, ldb, ldc;
  long stride_a, stride_b, stride_c; /* batch strides, elements */
  float alpha, beta;
  int c_f32;
  const float* bias;
  int act;
  void* preact;
  long ldpre;
  const void* mul;
  long ldmul;
  const void* res;
  long ldres;
  const float* colscale;
  const float* rowscale;
  long rows_per_scale;
  int split_k;  /* 0 = auto, 1 = off, >1 = forced */
  int act_col0; /* act / preact apply to columns n >= act_col0; preact[m, n - act_col0] */
  float* colsum; /* optional float32 [M]: (+)= alpha * sum_k A(m,k) — the bias gradient of a wgrad
                    GEMM, computed as a virtual all-ones column of B (batch must be 1) */
  int colsum_accumulate;
  int mul_gelu_grad; /* 1: the multiplier is gelu'(mul[m,n]) (GELU backward fused into a dgrad GEMM) */
  long workspace_bytes; /* size of the workspace passed with the call; it must be at least
                           dfm_gemm_workspace_size(d) (for dfm_gemm_group: d[0] carries the size of
                           the one shared workspace, >= dfm_gemm_group_workspace_size) */
  /* optional second output (ABI 13): out2[m, n] = v * mul2[m, n], v the epilogue value before `mul` /
   * `res` (after beta, bias, act) — the two products of an elementwise x * y backward
   * (dy*y -> dx, dy*x -> dy') written by the GEMM that produces dy (batch 1, output dtype, no res) */
  const void* mul2;
  long ldmul2;
  void* out2;
  long ldout2;
} DfmGemmDesc;

size_t dfm_gemm_workspace_size(const DfmGemmDesc* d);
int dfm_gemm(int dtype, const DfmGemmDesc* d, const void* A, const void* B, void* C, void* workspace,
             dfm_stream_t stream);
/* n (1..8) independent GEMMs of one operand layout in ONE launch (+ one split-K combine launch):
 * the weight gradients of a Block's backward (DFormer.py:76-95 / 53-55 nn.Linear backward), which
 * share the chip instead of each splitting K across all of it. Same semantics per problem as
 * dfm_gemm (epilogue, colsum bias gradient); workspace from dfm_gemm_group_workspace_size. */
size_t dfm_gemm_group_workspace_size(int n, const DfmGemmDesc* d);
int dfm_gemm_group(int dtype, int n, const DfmGemmDesc* d, const void* const* A, const void* const* B,
                   void* const* C, void* workspace, dfm_stream_t stream);

/* ---------------------------------------------------------------- deferred reduction second stages
 * The parameter-gradient reductions below (LayerNorm dgamma / dbeta, layer-scale dscale, depthwise
 * dw / db) run in two stages: per-block partials in the caller's workspace, then a fixed-order sum
 * over the blocks. With `defer` NULL an entry point launches both. With `defer` non-NULL it launches
 * only the first stage and describes the second in *defer; dfm_partial_sum_group then runs up to 16
 * such sums in ONE launch (a Block's backward issues them together at its end, with its grouped
 * weight gradients). Until that launch the workspace must stay untouched and the outputs unread.
 * Results are bit-identical to the undeferred call (same partials, same summation order).
 *   layout 0: out0[e] = sum_b part[b*n + e]                      (e < n)
 *   layout 1: e < n0 ? out0[e] : out1[e - n0]
 *   layout 2: depthwise [C][n0] with n0 = k*k + 1: out0[c*(n0-1) + i] for i < n0-1, out1[c] (bias)
 *   accumulate: out += sum instead of out = sum. */
typedef struct DfmPartialSum {
  const float* part;
  float* out0;
  float* out1;
  long n;
  long n0;
  int nblk;
  int layout;
  int accumulate;
} DfmPartialSum;
int dfm_partial_sum_group(int n, const DfmPartialSum* sums, dfm_stream_t stream);

/* ---------------------------------------------------------------- LayerNorm, channels_last
 * DFormer.py:21-45 (F.layer_norm over the last dim, eps 1e-6). mean/rstd: float32 [rows].
 * bwd: dx (+= when accumulate), dgamma/dbeta float32 [C] (overwritten); workspace from
 * dfm_layernorm_bwd_workspace; defer: see dfm_partial_sum_group. */
int dfm_layernorm_fwd(int dtype, long rows, int C, const void* x, long ldx, const float* gamma,
                      const float* beta, float eps, void* y, long ldy, float* mean, float* rstd,
                      dfm_stream_t stream);
size_t dfm_layernorm_bwd_workspace(long rows, int C);
/* dx = LN-backward(dy) [+ dres] [+ dx when accumulate]  (dres: the residual branch's gradient) */
int dfm_layernorm_bwd(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                      const float* gamma, const float* mean, const float* rstd, const void* dres, long lddres,
                      void* dx, long lddx, int accumulate, float* dgamma, float* dbeta, void* workspace,
                      DfmPartialSum* defer, dfm_stream_t stream);

/* ---------------------------------------------------------------- residual / layer-scale backward
 * Block.forward's x + DropPath(ls * f) (DFormer.py:173-179), backward in one pass over dout and f:
 *   df[r,c] = dout[r,c] * colscale[c] * rowscale[r/rps];   dscale[c] = sum_r dout * f * rowscale[r/rps]
 * (rowscale NULL = 1; dscale overwritten; workspace from dfm_residual_bwd_workspace; defer: see
 * dfm_partial_sum_group). */
size_t dfm_residual_bwd_workspace(long rows, int C);
int dfm_residual_bwd(int dtype, long rows, int C, const void* dout, long lddout, const void* f, long ldf,
                     const float* colscale, const float* rowscale, long rows_per_scale, void* df, long lddf,
                     float* dscale, void* workspace, DfmPartialSum* defer, dfm_stream_t stream);

/* ---------------------------------------------------------------- depthwise conv k x k, NHWC
 * DFormer.py:80-81 (7x7 conv/e_conv, pad 3) and DFormer.py:54,62 (3x3 pos + identity).
 * w: float32 [C][k][k], bias float32 [C] or NULL. add_identity (flags): bit 0: y += x; bit 1 (with
 * gelu_out): y receives gelu'(y) instead of y. gelu_out (optional): GELU(y) as well (the ConvFFN
 * activation, DFormer.py:64).
 * bwd_data: dx (+= when accumulate) = conv(dy, flipped w) (+ dy when add_identity).
 * bwd_weight: dw [C][k][k], db [C] (overwritten), workspace from dfm_dwconv_bwd_weight_workspace;
 * defer: see dfm_partial_sum_group. */
int dfm_dwconv_fwd(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx, const float* w,
                   const float* bias, int add_identity, void* y, long ldy, void* gelu_out, long ldg,
                   dfm_stream_t stream);
int dfm_dwconv_bwd_data(int dtype, int B, int H, int W, int C, int k, const void* dy, long lddy,
                        const float* w, int add_identity, void* dx, long lddx, int accumulate,
                        dfm_stream_t stream);
size_t dfm_dwconv_bwd_weight_workspace(int B, int H, int W, int C, int k);
int dfm_dwconv_bwd_weight(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx,
                          const void* dy, long lddy, float* dw, float* db, void* workspace,
                          DfmPartialSum* defer, dfm_stream_t stream);
/* bwd_data and bwd_weight in one pass over dy and x: dx (+= when accumulate), dw, db as above; workspace
 * from dfm_dwconv_bwd_weight_workspace. k = 3 (the ConvFFN's pos conv, add_identity allowed) or k = 7 (the
 * attention's conv / e_conv, add_identity 0; dw and db bit-identical to dfm_dwconv_bwd_weight's). */
int dfm_dwconv_bwd(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx, const void* dy,
                   long lddy, const float* w, int add_identity, void* dx, long lddx, int accumulate, float* dw,
                   float* db, void* workspace, DfmPartialSum* defer, dfm_stream_t stream);

/* ---------------------------------------------------------------- fused ConvFFN (K4)
 * DFormer.py:48-67 (MLP: LN -> fc1 -> DW3x3 + identity -> GELU -> fc2) inside Block's residual
 * (DFormer.py:176-179):  out = x + rowscale[p / (H*W)] * ls * f,
 *   f = fc2(GELU(DW3x3(h) + bpos + h)) + b2,  h = fc1(LN(x)) + b1.
 * x, out, f, xn, dx, dout: [B*H*W][C] contiguous NHWC rows (dtype); h: [B*H*W][hidden] (dtype), written
 * by the forward for the backward (the only hidden-sized tensor the forward writes); xn = LN(x) (the
 * fc1 weight gradient's operand; the forward writes it when xn is non-NULL, the backward requires it);
 * gelu_out / gelu_grad ([B*H*W][hidden] dtype, both or neither): GELU(hpre) and GELU'(hpre) as well, the
 * operands the op-level backward (fc2 weight gradient, GELU backward) reads;
 * w1 [hidden][C], w2 [C][hidden] (dtype); ln_w, ln_b, b1, bpos, b2, ls: float32; wpos [hidden][9]
 * float32; rowscale float32 [B] (DropPath keep mask / keep probability) or NULL; mean / rstd float32
 * [B*H*W] (the LayerNorm statistics, written by the forward). dtype bf16 or f16 (float32 runs the
 * unfused entry points); dfm_convffn_supported says whether (C, hidden) has fused kernels.
 * The backward writes dx (LayerNorm backward + the residual's dout) and every parameter gradient
 * (float32, overwritten: dw1 [hidden][C], dw2 [C][hidden], dwpos [hidden][9], dls = layer-scale),
 * reducing them in a fixed order (bit-reproducible); workspace from dfm_convffn_bwd_workspace_size. */
typedef struct DfmConvFFNDesc {
  int B, H, W, C, hidden;
  float ln_eps;
} DfmConvFFNDesc;
int dfm_convffn_supported(int dtype, const DfmConvFFNDesc* d);
int dfm_convffn_fwd(int dtype, const DfmConvFFNDesc* d, const void* x, const float* ln_w, const float* ln_b,
                    const void* w1, const float* b1, const float* wpos, const float* bpos, const void* w2,
                    const float* b2, const float* ls, const float* rowscale, void* out, void* f, void* h,
                    void* xn, float* mean, float* rstd, void* gelu_out, void* gelu_grad, dfm_stream_t stream);
size_t dfm_convffn_bwd_workspace_size(int dtype, const DfmConvFFNDesc* d);
int dfm_convffn_bwd(int dtype, const DfmConvFFNDesc* d, const void* dout, const void* x, const void* h,
                    const void* xn, const void* f, const float* mean, const float* rstd, const float* ln_w,
                    const float* ln_b,
                    const void* w1, const float* wpos, const float* bpos, const void* w2, const float* ls,
                    const float* rowscale, void* dx, float* dln_w, float* dln_b, float* dw1, float* db1,
                    float* dwpos, float* dbpos, float* dw2, float* db2, float* dls, void* workspace,
                    size_t workspace_bytes, dfm_stream_t stream);

/* ---------------------------------------------------------------- encoder Block
 * DFormer.py:147-181 Block.forward (x, x_e) -> (x + DropPath(ls1 * attn(x, x_e)) + DropPath(ls2 * mlp(.)),
 * x_e likewise with ls1_e / mlp_e2 / ls2_e), forward and backward, every kernel enqueued on `stream`.
 * x, y, dx, dy: [B*H*W][C]; xe, ye, dxe, dye: [B*H*W][C/2] (NHWC rows, dtype).
 * params: DFM_BLOCK_NPARAM pointers indexed by the DFM_BP_* enum (the reference state_dict entries of
 *   one Block, DFormer.py:70-181): the nn.Linear weights (the 11 names marked "dtype" below) are dtype
 *   copies ([out][in] row-major), every other entry (LayerNorm affine, biases, depthwise [C][k][k]
 *   weights, layer scales) float32. Entries the Block does not have are ignored (kv / short_cut_linear
 *   without a window; proj_e, layer_scale_1_e / _2_e and mlp_e2 with drop_depth).
 *   Contiguous q | q_cut | l (weights and biases, in that order) run as one GEMM, as the training step does.
 * grads: the same indexing, float32 [same shape] (overwritten; NULL entries are rejected for
 *   parameters the Block has).
 * rowscale: NULL, or 4 float32 [B] pointers (each may be NULL = 1): the per-sample DropPath scales
 *   (keep mask / keep prob) of, in mmcv's call order, attn x, mlp x, attn x_e, mlp x_e.
 * The forward writes `saved` (dfm_block_saved_size bytes) for the backward, which also reads x and
 * xe again; both use `workspace` (dfm_block_workspace_size bytes) as scratch. With drop_depth the x_e
 * output is the attention's e_back result (no proj_e / residual / mlp_e2; DFormer.py:133, 177-181): ye
 * receives it when non-NULL, and dye, when non-NULL, flows back through e_back (the encoder discards
 * the last Block's x_e, so both may be NULL). NULL params / grads entries the Block has: DFM_ERR_ARG.
 * fused_ffn: ConvFFNs with fused kernels (dfm_convffn_supported) run dfm_convffn_fwd / _bwd. */
typedef struct DfmBlockDesc {
  int B, H, W, C;
  int heads;      /* num_head */
  int window;     /* 7: pooled-query attention (DFormer.py:90-96, 119-131); 0: none */
  int hidden;     /* mlp hidden width = mlp_ratio * C (mlp_e2: hidden / 2) */
  int drop_depth; /* last Block of the last stage: no proj_e / layer_scale_*_e / mlp_e2 */
  int fused_ffn;
  float ln_eps;   /* 1e-6 */
} DfmBlockDesc;
enum {
  DFM_BP_NORM_W, DFM_BP_NORM_B, DFM_BP_NORM_E_W, DFM_BP_NORM_E_B, /* attn.norm, attn.norm_e */
  DFM_BP_Q_W, DFM_BP_Q_B,               /* attn.q [C][C] (dtype) */
  DFM_BP_QCUT_W, DFM_BP_QCUT_B,         /* attn.q_cut [C/2][C] (dtype) */
  DFM_BP_L_W, DFM_BP_L_B,               /* attn.l [C][C] (dtype) */
  DFM_BP_CONV_W, DFM_BP_CONV_B,         /* attn.conv [C][7][7] */
  DFM_BP_A_W, DFM_BP_A_B,               /* attn.a [C][C] (dtype) */
  DFM_BP_EFORE_W, DFM_BP_EFORE_B,       /* attn.e_fore [C/2][C/2] (dtype) */
  DFM_BP_ECONV_W, DFM_BP_ECONV_B,       /* attn.e_conv [C/2][7][7] */
  DFM_BP_EBACK_W, DFM_BP_EBACK_B,       /* attn.e_back [C/2][C/2] (dtype) */
  DFM_BP_KV_W, DFM_BP_KV_B,             /* attn.kv [C][C] (dtype; window only) */
  DFM_BP_SC_W, DFM_BP_SC_B,             /* attn.short_cut_linear [C/2][3C/2] (dtype; window only) */
  DFM_BP_PROJ_W, DFM_BP_PROJ_B,         /* attn.proj [C][fw] (dtype), fw = 2C with a window, 3C/2 without */
  DFM_BP_PROJE_W, DFM_BP_PROJE_B,       /* attn.proj_e [C/2][fw] (dtype) */
  DFM_BP_LS1, DFM_BP_LS1E, DFM_BP_LS2, DFM_BP_LS2E, /* layer_scale_1, _1_e, _2, _2_e */
  DFM_BP_MLP_NORM_W, DFM_BP_MLP_NORM_B, /* mlp.norm */
  DFM_BP_MLP_FC1_W, DFM_BP_MLP_FC1_B,   /* mlp.fc1 [hidden][C] (dtype) */
  DFM_BP_MLP_POS_W, DFM_BP_MLP_POS_B,   /* mlp.pos [hidden][3][3] */
  DFM_BP_MLP_FC2_W, DFM_BP_MLP_FC2_B,   /* mlp.fc2 [C][hidden] (dtype) */
  DFM_BP_MLPE_NORM_W, DFM_BP_MLPE_NORM_B, /* mlp_e2.*, C/2 and hidden/2 */
  DFM_BP_MLPE_FC1_W, DFM_BP_MLPE_FC1_B,
  DFM_BP_MLPE_POS_W, DFM_BP_MLPE_POS_B,
  DFM_BP_MLPE_FC2_W, DFM_BP_MLPE_FC2_B,
  DFM_BLOCK_NPARAM
};
size_t dfm_block_saved_size(int dtype, const DfmBlockDesc* d);
size_t dfm_block_workspace_size(int dtype, const DfmBlockDesc* d);
int dfm_block_fwd(int dtype, const DfmBlockDesc* d, const void* const* params, const float* const* rowscale,
                  const void* x, const void* xe, void* y, void* ye, void* saved, size_t saved_bytes, void* workspace,
                  size_t workspace_bytes, dfm_stream_t stream);
int dfm_block_bwd(int dtype, const DfmBlockDesc* d, const void* const* params, const float* const* rowscale,
                  const void* x, const void* xe, const void* saved, size_t saved_bytes, const void* dy,
                  const void* dye, void* dx, void* dxe, float* const* grads, void* workspace, size_t workspace_bytes,
                  dfm_stream_t stream);

/* ---------------------------------------------------------------- reductions / elementwise */
/* out[c] (+= when accumulate) = sum_rows x[r,c] * (mul ? mul[r,c] : 1) * (rowscale ? rowscale[r/rps] : 1)
 * (bias grads: nn.Linear backward; layer_scale grads: DFormer.py:173-179). */
size_t dfm_colsum_workspace(long rows, int C);
int dfm_colsum(int dtype, long rows, int C, const void* x, long ldx, const void* mul, long ldmul,
               const float* rowscale, long rows_per_scale, float* out, int accumulate, void* workspace,
               dfm_stream_t stream);
/* y = op(x): 0 copy/cast, used for float32 <-> bf16 conversion (dtype_in, dtype_out). */
int dfm_cast(int dtype_in, int dtype_out, long n, const void* x, void* y, dfm_stream_t stream);
/* n (<= 32) row-major [rows, cols] sources of dtypes src_dtypes[i] packed side by side (converted) into
 * dst [rows, n * cols] of dtype_out, one launch (the NMF backward's rank-R factors, ham_head.py:120-145) */
int dfm_pack_slices(int dtype_out, int n, const void* const* srcs, const int* src_dtypes, long rows, int cols,
                    void* dst, dfm_stream_t stream);
/* dx (+= when accumulate) = dy * gelu'(pre)   (nn.GELU backward, DFormer.py:56,97,113) */
int dfm_gelu_bwd(int dtype, long rows, int C, const void* dy, long lddy, const void* pre, long ldpre,
                 void* dx, long lddx, int accumulate, dfm_stream_t stream);
/* dst (+= when accumulate) = alpha * src * (mul ? mul : 1) * (colscale ? colscale[c] : 1)
 *   * (rowscale ? rowscale[r/rps] : 1)   — the residual / layer-scale / DropPath chain rule
 *   (DFormer.py:173-179) and q*a, cx*xe products (DFormer.py:134-135). */
int dfm_scale_mul(int dtype, long rows, int C, const void* src, long ldsrc, const void* mul, long ldmul,
                  const float* colscale, const float* rowscale, long rows_per_scale, float alpha,
                  void* dst, long lddst, int accumulate, dfm_stream_t stream);

/* y[r, c] = x[r, c] * scale[(r / rows_per_group) * C + c]: a per-group channel scale in one launch
 * (Dropout2d's per-image channel mask / keep ahead of the classifier, decode_head.py:226-231, and its
 * backward; y may alias x). */
int dfm_group_scale(int dtype, long rows, int C, const void* x, long ldx, const float* scale,
                    long rows_per_group, void* y, long ldy, dfm_stream_t stream);
/* o1 = src * m1, o2 = src * m2 in one pass over src: the gradients of an elementwise product
 * d(q*a) -> (d*a, d*q), d(cx*xe') -> (d*xe', d*cx) (DFormer.py:134-135 backward). */
int dfm_dual_mul(int dtype, long rows, int C, const void* src, long ldsrc, const void* m1, long ld1, const void* m2,
                 long ld2, void* o1, long ldo1, void* o2, long ldo2, dfm_stream_t stream);

/* ---------------------------------------------------------------- pooled-query attention
 * AdaptiveAvgPool2d(7) over NHWC (DFormer.py:92,124): y[b][i*7+j][c] = bin mean. */
int dfm_adaptive_pool7_fwd(int dtype, int B, int H, int W, int C, const void* x, long ldx, void* y,
                           long ldy, dfm_stream_t stream);
int dfm_adaptive_pool7_bwd(int dtype, int B, int H, int W, int C, const void* dy, long lddy, void* dx,
                           long lddx, int accumulate, dfm_stream_t stream);
/* F.interpolate(bilinear, align_corners=False) NHWC [B,Hi,Wi,C] -> [B,Ho,Wo,C]
 * (DFormer.py:131, ham_head.py:226-231, MLPDecoder.py:67-73, builder.py:203). */
int dfm_bilinear_fwd(int dtype, int B, int Hi, int Wi, int Ho, int Wo, int C, const void* x, long ldx,
                     void* y, long ldy, int accumulate, dfm_stream_t stream);
int dfm_bilinear_bwd(int dtype, int B, int Hi, int Wi, int Ho, int Wo, int C, const void* dy, long lddy,
                     void* dx, long lddx, int accumulate, dfm_stream_t stream);
/* softmax(q*scale k^T) v for 49 pooled queries over N keys, per (b, head) (DFormer.py:119-130).
 * q: [B][49][ldq] head h at cols h*dh; k, v: [B][N][ldkv] head h at cols h*dh; o like q.
 * lse: float32 [B][heads][49] saved for backward. */
size_t dfm_pooled_attn_workspace(int B, int heads, int N, int dh);
int dfm_pooled_attn_fwd(int dtype, int B, int heads, int N, int dh, const void* q, long ldq, const void* k,
                        const void* v, long ldkv, float scale, void* o, long ldo, float* lse,
                        void* workspace, dfm_stream_t stream);
int dfm_pooled_attn_bwd(int dtype, int B, int heads, int N, int dh, const void* q, long ldq, const void* k,
                        const void* v, long ldkv, float scale, const void* o, long ldo, const void* dout,
                        long lddo, const float* lse, void* dq, void* dk, void* dv, long lddkv,
                        void* workspace, dfm_stream_t stream);

/* ---------------------------------------------------------------- BatchNorm (+ SyncBN stats)
 * mmcv ConvModule norm / nn.BatchNorm2d / SyncBatchNorm over NHWC rows (ham_head.py:204-220,
 * MLPDecoder.py:53). stats: float32 [3][C] = (sum (x-K), sum (x-K)^2, K) with the shift K = x[row 0]
 * (no E[x^2]-E[x]^2 cancellation when |mean| >> std); finalize: mean = K + S1/n,
 * var = S2/n - (S1/n)^2. For SyncBN (torch SyncBatchNorm's all_gather of per-rank statistics,
 * torch/nn/modules/_functions.py) the all-gathered per-rank triples [shards][3][C] are merged on the
 * device by dfm_bn_merge (counts: float32 [shards] rows per rank) into one triple shifted by rank 0's K
 * (fp64, fixed rank order; exact identity for one shard), which dfm_bn_finalize takes with the total
 * count. apply: y = act((x - mean) * rstd * gamma + beta) [+ res] ; mean/rstd float32 [C]. */
size_t dfm_bn_workspace(long rows, int C);
int dfm_bn_stats(int dtype, long rows, int C, const void* x, long ldx, float* stats, void* workspace,
                 dfm_stream_t stream);
int dfm_bn_finalize(int C, const float* stats, double count, float eps, float momentum, float* mean,
                    float* rstd, float* running_mean, float* running_var, dfm_stream_t stream);
int dfm_bn_merge(int shards, int C, const float* parts, const float* counts, float* stats, dfm_stream_t stream);
int dfm_bn_apply(int dtype, long rows, int C, const void* x, long ldx, const float* mean, const float* rstd,
                 const float* gamma, const float* beta, const void* res, long ldres, int act, void* y,
                 long ldy, dfm_stream_t stream);
/* bwd: given dy (already multiplied by the activation mask by the caller) compute
 * stats2 float32 [2][C] = (sum dy, sum dy*xhat) ; then dx = gamma*rstd*(dy - s0/n - xhat*s1/n). */
int dfm_bn_bwd_stats(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                     const float* mean, const float* rstd, float* stats2, void* workspace, dfm_stream_t stream);
int dfm_bn_bwd_apply(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                     const float* mean, const float* rstd, const float* gamma, const float* stats2,
                     double count, void* dx, long lddx, int accumulate, dfm_stream_t stream);
/* act backward helper: dst = dy * (y > 0) (ReLU backward given the ReLU output) */
int dfm_relu_bwd(int dtype, long rows, int C, const void* dy, long lddy, const void* y, long ldy, void* dx,
                 long lddx, dfm_stream_t stream);

/* ---------------------------------------------------------------- dense 3x3 stride-2 conv
 * Stems / stage downsampling (DFormer.py:194-228, 295-303: nn.Conv2d(cin, cout, 3, 2, 1) after
 * BN/SyncBN, or after BN + GELU inside the stem) as gather + dfm_gemm over NHWC rows.
 * im2col: cols[m][(kh*3+kw)*Cin + c] = act(bn(x[b][c][2*oh-1+kh][2*ow-1+kw])), zero outside the
 *   image and for columns >= 9*Cin up to Kp (Kp % 8 == 0); m = (b*Ho + oh)*Wo + ow,
 *   Ho = (H+1)/2, Wo = (W+1)/2. x is NCHW-logical with element strides (sb, sc, sh, sw), so the
 *   raw float32 image, a channel view and NHWC rows (sc = 1) are all read in place.
 *   bn (mean/rstd/gamma/beta, nullable together): (v - mean)*rstd*gamma + beta; gelu: exact GELU.
 * col2im (backward data): dx[p][c] (+)= act'(.) * sum over the taps of p of dcols (fixed order,
 *   deterministic); x / bn / gelu recompute the GELU derivative at the folded BN output. dx is
 *   the gradient w.r.t. the BN output (the BN backward runs on dfm_bn_bwd_*). Cin % 8 == 0.
 * weight_pack: w float32 [Cout][Cin][3][3] -> wp [Cout][Kp] in (kh, kw, c) column order;
 * weight_unpack: the weight gradient of the packed layout back to [Cout][Cin][3][3]. */
int dfm_conv3s2_im2col(int dtype_in, int dtype_out, int B, int H, int W, int Cin, long sb, long sc, long sh,
                       long sw, const void* x, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, int gelu, int Kp, void* cols, dfm_stream_t stream);
int dfm_conv3s2_col2im(int dtype, int B, int H, int W, int Cin, const void* dcols, long ldc, const void* x,
                       long ldx, const float* mean, const float* rstd, const float* gamma, const float* beta,
                       int gelu, void* dx, long lddx, int accumulate, dfm_stream_t stream);
/* col2im_nchw: the same gather without BN / GELU for any Cin, into dx (dtype_out) with element
 * strides (sb, sc, sh, sw) — the input gradient of the stem's first conv. */
int dfm_conv3s2_col2im_nchw(int dtype, int dtype_out, int B, int H, int W, int Cin, const void* dcols, long ldc,
                            void* dx, long sb, long sc, long sh, long sw, dfm_stream_t stream);
int dfm_conv3_weight_pack(int dtype_out, int Cout, int Cin, int Kp, const float* w, void* wp,
                          dfm_stream_t stream);
int dfm_conv3_weight_unpack(int Cout, int Cin, int Kp, const float* dwp, float* dw, int accumulate,
                            dfm_stream_t stream);

/* ---------------------------------------------------------------- multi-scale + flip evaluation
 * utils/val_mm.py:325-472 evaluate_msf, utils/metrics_new.py:16-20 Metrics.update.
 * resize_nchw: y [B][C][Ho][Wo] (contiguous) = F.interpolate(x, (Ho, Wo), 'bilinear',
 *   align_corners), then torch.flip(dims=(3,)) when flip; x NCHW-logical with element strides.
 * msf_accumulate: acc [B*H*W][ncls] float32 (NHWC rows) += softmax over classes of the decoder's
 *   low-res logits low [B*h*w][ldl] upsampled to (Hs, Ws) with align_corners=False (the model's
 *   output at scale s, builder.py:203), flipped back along W when flip, then resized to (H, W)
 *   with align_corners=True. ncls <= 64.
 * seg_confusion: hist [ncls*ncls] uint64 += bincount(label * ncls + argmax(acc)) over pixels
 *   whose label != ignore (and within [0, ncls)). */
int dfm_resize_nchw(int dtype_in, int dtype_out, int B, int C, int Hi, int Wi, long sb, long sc, long sh, long sw,
                    const void* x, int Ho, int Wo, int align_corners, int flip, void* y, dfm_stream_t stream);
int dfm_msf_accumulate(int dtype, int B, int h, int w, int ncls, const void* low, long ldl, int Hs, int Ws, int H,
                       int W, int flip, float* acc, dfm_stream_t stream);
int dfm_seg_confusion(long npix, int ncls, const float* acc, const long long* label, int ignore,
                      unsigned long long* hist, dfm_stream_t stream);

/* ---------------------------------------------------------------- NMF2D multiplicative update
 * ham_head.py:120-145:  out = a * num / (den + eps)  (float32), and its backward:
 *   ga (+= when accumulate_ga) = g * num / (den+eps);  gnum = g * a / (den+eps);
 *   gden = -g * out / (den+eps).
 * out16 / gnum16 (nullable): 16-bit copies (copy_dtype DFM_BF16 or DFM_F16) of out / gnum, the
 * operands of the 16-bit NMF GEMMs (the reference's autocast runs ham_head.py's bmm in the
 * autocast dtype). */
int dfm_nmf_update(long n, const float* a, const float* num, const float* den, float eps, float* out,
                   void* out16, int copy_dtype, dfm_stream_t stream);
int dfm_nmf_update_bwd(long n, const float* g, const float* a, const float* num, const float* den,
                       const float* out, float eps, float* ga, int accumulate_ga, float* gnum, float* gden,
                       void* gnum16, int copy_dtype, dfm_stream_t stream);
/* The same updates with their rank-R denominator products fused in (R = 64), per batch b and row n
 * of [batch][rows][R] float32 operands and [batch][R][R] Gram matrices:
 *   dfm_nmf_update_mm:     den = a M (ham_head.py:120-141's  C (B^T B)  /  B (C^T C)), written;
 *                          out = a * num / (den + eps) (+ out16).
 *   dfm_nmf_update_bwd_mm: g' = g [+ A2 (S + S^T)]  (the symmetric Gram gradient of the NEXT update
 *                          in time, e.g. gC += Cn (gQ + gQ^T), folded into this pass);
 *                          ga (+=) = g' num / (den+eps) [+ gden Mg]; gnum = g' a / (den+eps) (+ gnum16);
 *                          gden = -g' out / (den+eps)   (Mg: the Gram matrix of this update's den).
 * Each replaces one or three row-by-R x R GEMM launches and their [rows, R] round trips. */
int dfm_nmf_update_mm(int batch, long rows, int R, const float* a, const float* num, const float* M, float eps,
                      float* den, float* out, void* out16, int copy_dtype, dfm_stream_t stream);
int dfm_nmf_update_bwd_mm(int batch, long rows, int R, const float* g, const float* A2, const float* S,
                          const float* a, const float* num, const float* den, const float* out, float eps,
                          const float* Mg, float* ga, int accumulate_ga, float* gnum, float* gden, void* gnum16,
                          int copy_dtype, dfm_stream_t stream);
/* The NMF2D forward and backward (ham_head.py:60-145: coef = softmax(x B0), `steps` updates of C and B,
 * the final C update, y = C B^T; rank R = 64) as two calls: x [batch][N][D] (dtype), bases
 * [batch][D][R] float32 (a constant: not modified, no gradient), y / gy / gx [batch][N][D] (dtype).
 * dfm_nmf_fwd keeps every step's factors in `saved` (dfm_nmf_saved_size bytes) for dfm_nmf_bwd, or
 * nothing when saved is NULL (inference); the backward returns gx = dL/dx through every update.
 * Workspaces: dfm_nmf_fwd_workspace_size (sized for saved == NULL, which needs the most) and
 * dfm_nmf_bwd_workspace_size bytes; sizes 0 = unsupported dtype / shape / rank. */
size_t dfm_nmf_saved_size(int dtype, int batch, long N, long D, int R, int steps);
size_t dfm_nmf_fwd_workspace_size(int dtype, int batch, long N, long D, int R, int steps);
size_t dfm_nmf_bwd_workspace_size(int dtype, int batch, long N, long D, int R, int steps);
int dfm_nmf_fwd(int dtype, int batch, long N, long D, int R, int steps, float eps, const void* x,
                const float* bases, void* y, void* saved, long saved_bytes, void* workspace, long workspace_bytes,
                dfm_stream_t stream);
int dfm_nmf_bwd(int dtype, int batch, long N, long D, int R, int steps, float eps, const void* x,
                const float* bases, const void* saved, long saved_bytes, const void* gy, void* gx, void* workspace,
                long workspace_bytes, dfm_stream_t stream);
/* row softmax over R (NMF coef init, ham_head.py:48-49) and its backward */
int dfm_softmax_rows(long rows, int R, const float* x, float* y, dfm_stream_t stream);
int dfm_softmax_rows_bwd(long rows, int R, const float* y, const float* dy, float* dx, int accumulate,
                         dfm_stream_t stream);

/* ---------------------------------------------------------------- segmentation loss
 * builder.py:203,230: logits [B,h,w,ncls] (NHWC, low res) bilinearly upsampled to [B,H,W]
 * + cross-entropy(ignore_index) + mean over valid pixels. Fused: the full-resolution logits are
 * never materialised. loss_out: float32 [2] = (sum of CE, valid count). dlogits float32 low-res; gscale: device float32 scalar (upstream grad) or NULL = 1. */
size_t dfm_seg_loss_workspace(int B, int H, int W);
int dfm_seg_loss_fwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                     const long* label, int ignore, float* lse, float* loss_out, void* workspace,
                     dfm_stream_t stream);
/* bwd workspace: dfm_seg_loss_bwd_workspace bytes (required). Every upsampling factor is
 * deterministic (fixed-order sums, no atomics): an integer factor (H = S h, W = S w, S in {2, 4, 8})
 * takes per-tile corner partials + a 4-way gather, any other factor (h <= H, w <= W, W / w up to
 * ~120) a separable x-pass into rx [B][H][w][ncls] float32 and a y-pass. */
size_t dfm_seg_loss_bwd_workspace(int B, int h, int w, int ncls, int H, int W);
int dfm_seg_loss_bwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                     const long* label, int ignore, const float* lse, const float* loss_out,
                     const float* gscale, float* dlogits, void* workspace, dfm_stream_t stream);

/* Training: the loss AND its gradient's per-tile partials in one pass (integer factor S in {4, 8}: the
 * ham head's x8, the MLP decoder's x4 at 480x640): each S x S pixel tile's 2 x 2 low-res logit rows
 * are read once, loss_out = (sum, count) as dfm_seg_loss_fwd; grad_partials (dfm_seg_loss_grad_partials_size
 * bytes, 0 = factor unsupported) must survive until dfm_seg_loss_bwd_gather, which writes dlogits
 * (dtype_out) = gscale / max(count, 1) * the fixed-order sum of the corner partials of each cell. */
size_t dfm_seg_loss_grad_partials_size(int B, int h, int w, int ncls, int H, int W);
int dfm_seg_loss_fwd_grad(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                          const long* label, int ignore, float* loss_out, float* grad_partials, dfm_stream_t stream);
int dfm_seg_loss_bwd_gather(int dtype_out, int B, int h, int w, int ncls, const float* grad_partials,
                            const float* loss_out, const float* gscale, void* dlogits, dfm_stream_t stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.AdamW step (train.py:210-216) over a flat float32 parameter buffer; optional
 * 16-bit shadow copy (copy_dtype DFM_BF16 / DFM_F16) for the next step's GEMM operands.
 * grad_scale multiplies g (1/world, and 1/loss-scale on the fp16 path). */
int dfm_adamw(long n, float* p, const float* g, float* m, float* v, float lr, float beta1, float beta2,
              float eps, float weight_decay, int step, float grad_scale, void* copy, int copy_dtype,
              dfm_stream_t stream);
/* The same step with lr and step (as float) read from device memory hyper[2] = {lr, step}: what a
 * captured HIP graph of the whole training step calls, the host refreshing hyper before a replay. */
int dfm_adamw_dev(long n, float* p, const float* g, float* m, float* v, const float* hyper, float beta1,
                  float beta2, float eps, float weight_decay, float grad_scale, void* copy, int copy_dtype,
                  dfm_stream_t stream);
/* fp16 loss scaling (utils/train.py:289, 323-345 torch.cuda.amp.GradScaler): flag[0] = 1 when any
 * gradient element is inf / nan (flag is not cleared: the caller zeroes it per step). */
int dfm_grad_nonfinite(long n, const float* g, int* flag, dfm_stream_t stream);
/* The loss scaler decided on the device, so the fp16 step replays from a captured graph: amp[4] =
 * {scale, growth_tracker, applied_steps, skipped} float32. dfm_adamw_amp is dfm_adamw_dev that
 * skips the update when flag[0] is set, unscales by 1/amp[0] and uses step amp[2] + 1;
 * dfm_loss_scale_update (launched after every group's AdamW) applies GradScaler.update — backoff
 * on overflow, growth after `interval` clean steps — counts the step and clears flag. */
int dfm_adamw_amp(long n, float* p, const float* g, float* m, float* v, const float* hyper, const float* amp,
                  const int* flag, float beta1, float beta2, float eps, float weight_decay, float grad_scale,
                  void* copy, int copy_dtype, dfm_stream_t stream);
int dfm_loss_scale_update(float* amp, int* flag, float growth, float backoff, int interval, dfm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DFORMER_HIP_H */
