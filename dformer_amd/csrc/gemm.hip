// C entry points of the MFMA GEMM (include/dformer_hip.h): descriptor validation, split-K /
// workspace sizing, and dispatch to the per-dtype instantiations (gemm_bf16.hip, gemm_f16.hip,
// gemm_f32.hip). Kernels and tile selection: gemm_impl.h.
#include "gemm_impl.h"

extern "C" size_t dfm_gemm_workspace_size(const DfmGemmDesc* d) {
  const int s = std::max(choose_splits(d, 2), choose_splits(d, 4));
  if (s <= 1) return 0;
  const long ldw = (d->N + (d->colsum ? 1 : 0) + 7) & ~7L;
  return (size_t)s * (d->batch > 0 ? d->batch : 1) * d->M * ldw * sizeof(float);
}

// Shape / stride validation shared by dfm_gemm and dfm_gemm_group (problem q): every operand row
// fits its leading dimension, consecutive batch matrices do not overlap (a zero A / B batch stride
// broadcasts one matrix; C must not), and the epilogue operands are at least N columns wide.
static int validate_desc(const DfmGemmDesc* d, const char* who, int q) {
  DFM_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 0, "%s: negative size (problem %d)", who, q);
  if (d->M == 0 || d->N == 0) return DFM_OK;
  const long ra = d->a_kcontig ? d->M : d->K, ca = d->a_kcontig ? d->K : d->M;  // rows x cols in memory
  const long rb = d->b_kcontig ? d->N : d->K, cb = d->b_kcontig ? d->K : d->N;
  DFM_CHECK_ARG(d->lda >= ca, "%s: lda %ld < %ld (problem %d)", who, d->lda, ca, q);
  DFM_CHECK_ARG(d->ldb >= cb, "%s: ldb %ld < %ld (problem %d)", who, d->ldb, cb, q);
  DFM_CHECK_ARG(d->ldc >= d->N, "%s: ldc %ld < N %d (problem %d)", who, d->ldc, d->N, q);
  if (d->batch > 1) {
    const long ea = ra > 0 ? (ra - 1) * d->lda + ca : 0, eb = rb > 0 ? (rb - 1) * d->ldb + cb : 0;
    const long ec = (long)(d->M - 1) * d->ldc + d->N;
    DFM_CHECK_ARG(d->stride_a == 0 || d->stride_a >= ea, "%s: stride_a %ld < %ld, batch matrices overlap (problem %d)",
                  who, d->stride_a, ea, q);
    DFM_CHECK_ARG(d->stride_b == 0 || d->stride_b >= eb, "%s: stride_b %ld < %ld, batch matrices overlap (problem %d)",
                  who, d->stride_b, eb, q);
    DFM_CHECK_ARG(d->stride_c >= ec, "%s: stride_c %ld < %ld, batch outputs overlap (problem %d)", who, d->stride_c,
                  ec, q);
    DFM_CHECK_ARG(d->stride_a >= 0 && d->stride_b >= 0, "%s: negative batch stride (problem %d)", who, q);
  }
  const long npre = d->N - d->act_col0;
  DFM_CHECK_ARG(d->act_col0 >= 0 && d->act_col0 <= d->N, "%s: act_col0 out of range (problem %d)", who, q);
  DFM_CHECK_ARG(d->preact == nullptr || d->ldpre >= npre, "%s: ldpre too small (problem %d)", who, q);
  DFM_CHECK_ARG(d->mul == nullptr || d->ldmul >= d->N, "%s: ldmul too small (problem %d)", who, q);
  DFM_CHECK_ARG(d->res == nullptr || d->ldres >= d->N, "%s: ldres too small (problem %d)", who, q);
  DFM_CHECK_ARG(d->rowscale == nullptr || d->rows_per_scale > 0, "%s: rows_per_scale must be > 0 (problem %d)", who,
                q);
  DFM_CHECK_ARG(d->colsum == nullptr || d->batch <= 1, "%s: colsum needs batch 1 (problem %d)", who, q);
  DFM_CHECK_ARG(d->workspace_bytes >= 0, "%s: negative workspace size (problem %d)", who, q);
  DFM_CHECK_ARG(!d->out2 == !d->mul2, "%s: out2 and mul2 go together (problem %d)", who, q);
  DFM_CHECK_ARG(d->out2 == nullptr || (d->ldout2 >= d->N && d->ldmul2 >= d->N && d->batch <= 1 && !d->res &&
                                       !d->c_f32 && !d->colsum),
                "%s: out2 needs ldout2 / ldmul2 >= N, batch 1, no res / colsum, output in the operand dtype (problem %d)",
                who, q);
  return DFM_OK;
}

extern "C" int dfm_gemm(int dtype, const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws,
                        dfm_stream_t stream) {
  DFM_CHECK_ARG(d && A && B && C, "dfm_gemm: null argument");
  if (int st = validate_desc(d, "dfm_gemm", 0)) return st;
  if (d->M == 0 || d->N == 0) return DFM_OK;
  const size_t need = dfm_gemm_workspace_size(d);
  DFM_CHECK_ARG(need == 0 || (ws != nullptr && (size_t)d->workspace_bytes >= need),
                "dfm_gemm: workspace of %ld bytes, %zu needed", d->workspace_bytes, need);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return dfm_gemm_bf16(d, A, B, C, ws, s);
  if (dtype == DFM_F16) return dfm_gemm_f16(d, A, B, C, ws, s);
  if (dtype == DFM_F32) return dfm_gemm_f32(d, A, B, C, ws, s);
  dfm_set_error("dfm_gemm: unsupported dtype %d", dtype);
  return DFM_ERR_DTYPE;
}

extern "C" size_t dfm_gemm_group_workspace_size(int n, const DfmGemmDesc* d) {
  if (n < 1 || n > GMAX || d == nullptr) return 0;
  if (d[0].a_kcontig) {  // forward / input-gradient groups: ring members run unsplit, the rest one by one
    size_t one = 0;
    for (int q = 0; q < n; ++q) one = std::max(one, dfm_gemm_workspace_size(&d[q]));
    return one;
  }
  int splits[GMAX];
  group_splits(n, d, splits);
  size_t total = 0, one = 0;
  for (int q = 0; q < n; ++q) {
    total += group_ws_bytes(&d[q], splits[q]);
    one = std::max(one, dfm_gemm_workspace_size(&d[q]));  // k-contiguous-A groups may run problems singly
  }
  return std::max(total, one);
}

extern "C" int dfm_gemm_group(int dtype, int n, const DfmGemmDesc* d, const void* const* A, const void* const* B,
                              void* const* C, void* ws, dfm_stream_t stream) {
  DFM_CHECK_ARG(d && A && B && C && n >= 1 && n <= GMAX, "dfm_gemm_group: 1 <= n <= %d problems", GMAX);
  for (int q = 0; q < n; ++q) {
    DFM_CHECK_ARG(A[q] && B[q] && C[q], "dfm_gemm_group: null operand (problem %d)", q);
    DFM_CHECK_ARG(d[q].M > 0 && d[q].N > 0 && d[q].K >= 0, "dfm_gemm_group: bad size (problem %d)", q);
    DFM_CHECK_ARG(d[q].a_kcontig == d[0].a_kcontig && d[q].b_kcontig == d[0].b_kcontig,
                  "dfm_gemm_group: problems must share one operand layout");
    if (int st = validate_desc(&d[q], "dfm_gemm_group", q)) return st;
  }
  const size_t need = dfm_gemm_group_workspace_size(n, d);
  DFM_CHECK_ARG(need == 0 || (ws != nullptr && (size_t)d[0].workspace_bytes >= need),
                "dfm_gemm_group: workspace of %ld bytes, %zu needed", d[0].workspace_bytes, need);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return dfm_gemm_group_bf16(n, d, A, B, C, ws, s);
  if (dtype == DFM_F16) return dfm_gemm_group_f16(n, d, A, B, C, ws, s);
  if (dtype == DFM_F32) return dfm_gemm_group_f32(n, d, A, B, C, ws, s);
  dfm_set_error("dfm_gemm_group: unsupported dtype %d", dtype);
  return DFM_ERR_DTYPE;
}
