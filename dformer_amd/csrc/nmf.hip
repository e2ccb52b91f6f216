// NMF2D forward in one entry point (ham_head.py:60-145, MD_R = 64): the whole multiplicative-update
// loop of the Hamburger's matrix decomposition issued from the library, for hosts that bind the C
// ABI without the Python orchestration (decoders.NMF2DFn issues the same launches one by one and
// keeps every step's factors for its backward). Host code only: it enqueues dfm_gemm /
// dfm_softmax_rows / dfm_cast / dfm_nmf_update_mm on the caller's stream, in exactly NMF2DFn's
// order and with its descriptors, so the two paths give identical bits.
//
// Shapes per image (batch b), NHWC orientation (the reference's x^T):
//   x [N, D] (dtype), bases B0 [D, R] fp32, coef C [N, R] fp32, y = C B^T [N, D] (dtype)
//   coef = softmax_rows(x B0)                                         (ham_head.py:48-49, 116-117)
//   repeat steps:  C <- C * (x B) / (C (B^T B) + eps)                 (ham_head.py:120-128)
//                  B <- B * (x^T C) / (B (C^T C) + eps)               (ham_head.py:130-138)
//   C <- C * (x B) / (C (B^T B) + eps)                                (compute_coef, :140-141)
// For 16-bit x the x-streaming products take 16-bit copies of B / C (written by the update kernels)
// with fp32 accumulation; the factors, Gram matrices and updates stay fp32.
#include "common.h"

#include <algorithm>

namespace {

constexpr int NMF_RANK = 64;

struct NmfPlan {
  int dtype, batch, R;
  long N, D;
  bool lp;
  // workspace carve-up (byte offsets)
  size_t num_c, c0, c1, den_c, num_b, b0, b1, den_b, gram, c16, b16, gemm_ws, total;
  size_t gemm_bytes;
  DfmGemmDesc xb, xtc, btb, ctc, out;
};

DfmGemmDesc bmm_desc(int M, int N, int K, int batch, bool a_t, bool b_t, long lda, long ldb, long ldc, long sa,
                     long sb, long sc, int c_f32) {
  DfmGemmDesc d{};
  d.M = M; d.N = N; d.K = K; d.batch = batch;
  d.a_kcontig = !a_t; d.b_kcontig = b_t;
  d.lda = lda; d.ldb = ldb; d.ldc = ldc;
  d.stride_a = sa; d.stride_b = sb; d.stride_c = sc;
  d.alpha = 1.f; d.beta = 0.f; d.c_f32 = c_f32;
  d.rows_per_scale = 1;
  return d;
}

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

NmfPlan nmf_plan(int dtype, int batch, long N, long D, int R) {
  NmfPlan p{};
  p.dtype = dtype; p.batch = batch; p.N = N; p.D = D; p.R = R;
  p.lp = dtype != DFM_F32;
  const int c32 = p.lp ? 1 : 0;
  // the descriptors K.bmm builds for NMF2DFn's products (a [b][rows][cols] row-major per image)
  p.xb = bmm_desc((int)N, R, (int)D, batch, false, false, D, R, R, N * D, D * R, N * R, c32);   // x B
  p.xtc = bmm_desc((int)D, R, (int)N, batch, true, false, D, R, R, N * D, N * R, D * R, c32);   // x^T C
  p.btb = bmm_desc(R, R, (int)D, batch, true, false, R, R, R, D * R, D * R, R * R, 0);          // B^T B
  p.ctc = bmm_desc(R, R, (int)N, batch, true, false, R, R, R, N * R, N * R, R * R, 0);          // C^T C
  p.out = bmm_desc((int)N, (int)D, R, batch, false, true, R, R, D, N * R, D * R, N * D, 0);     // C B^T
  p.gemm_bytes = std::max({dfm_gemm_workspace_size(&p.xb), dfm_gemm_workspace_size(&p.xtc),
                           dfm_gemm_workspace_size(&p.btb), dfm_gemm_workspace_size(&p.ctc),
                           dfm_gemm_workspace_size(&p.out)});
  const size_t fc = (size_t)batch * N * R * sizeof(float), fb = (size_t)batch * D * R * sizeof(float);
  const size_t es = p.lp ? 2 : 4;
  size_t o = 0;
  auto take = [&](size_t bytes) { const size_t at = o; o += al256(bytes); return at; };
  p.num_c = take(fc); p.c0 = take(fc); p.c1 = take(fc); p.den_c = take(fc);
  p.num_b = take(fb); p.b0 = take(fb); p.b1 = take(fb); p.den_b = take(fb);
  p.gram = take((size_t)batch * R * R * sizeof(float));
  p.c16 = p.lp ? take((size_t)batch * N * R * es) : 0;
  p.b16 = p.lp ? take((size_t)batch * D * R * es) : 0;
  p.gemm_ws = take(std::max(p.gemm_bytes, (size_t)1));
  p.total = o;
  return p;
}

}  // namespace

extern "C" size_t dfm_nmf_fwd_workspace_size(int dtype, int batch, long N, long D, int R) {
  if (batch <= 0 || N <= 0 || D <= 0 || R != NMF_RANK) return 0;
  return nmf_plan(dtype, batch, N, D, R).total;
}

extern "C" int dfm_nmf_fwd(int dtype, int batch, long N, long D, int R, int steps, float eps, const void* x,
                           const float* bases, void* y, void* workspace, long workspace_bytes, dfm_stream_t stream) {
  DFM_CHECK_ARG(x && bases && y && workspace, "dfm_nmf_fwd: null argument");
  DFM_CHECK_ARG(dtype == DFM_F32 || dtype == DFM_BF16 || dtype == DFM_F16, "dfm_nmf_fwd: bad dtype");
  DFM_CHECK_ARG(batch > 0 && N > 0 && D > 0 && steps >= 0, "dfm_nmf_fwd: bad shape");
  DFM_CHECK_ARG(R == NMF_RANK, "dfm_nmf_fwd: R=%d unsupported (the fused updates are rank 64)", R);
  NmfPlan p = nmf_plan(dtype, batch, N, D, R);
  DFM_CHECK_ARG(workspace_bytes >= (long)p.total, "dfm_nmf_fwd: workspace %ld < %zu bytes", workspace_bytes,
                p.total);
  char* ws = (char*)workspace;
  float* num_c = (float*)(ws + p.num_c);
  float* cbuf[2] = {(float*)(ws + p.c0), (float*)(ws + p.c1)};
  float* den_c = (float*)(ws + p.den_c);
  float* num_b = (float*)(ws + p.num_b);
  float* bbuf[2] = {(float*)(ws + p.b0), (float*)(ws + p.b1)};
  float* den_b = (float*)(ws + p.den_b);
  float* gram = (float*)(ws + p.gram);
  void* gws = ws + p.gemm_ws;
  void* c16 = p.lp ? (void*)(ws + p.c16) : nullptr;
  void* b16 = p.lp ? (void*)(ws + p.b16) : nullptr;
  const int copy = p.lp ? dtype : 0;
  for (DfmGemmDesc* d : {&p.xb, &p.xtc, &p.btb, &p.ctc, &p.out}) d->workspace_bytes = (long)p.gemm_bytes;
  int rc;
#define NMF_DO(call)          \
  do {                        \
    rc = (call);              \
    if (rc != DFM_OK) return rc; \
  } while (0)
  // coef = softmax(x B0); the 16-bit operand copy of B0 for the x products
  const float* Bt = bases;
  const void* Bop = bases;
  if (p.lp) {
    NMF_DO(dfm_cast(DFM_F32, dtype, (long)batch * D * R, bases, b16, stream));
    Bop = b16;
  }
  NMF_DO(dfm_gemm(dtype, &p.xb, x, Bop, num_c, gws, stream));
  NMF_DO(dfm_softmax_rows((long)batch * N, R, num_c, cbuf[0], stream));
  const float* Ct = cbuf[0];
  int ci = 1, bi = 0;
  for (int it = 0; it < steps; ++it) {
    // C <- C * (x B) / (C (B^T B) + eps)
    NMF_DO(dfm_gemm(dtype, &p.xb, x, Bop, num_c, gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &p.btb, Bt, Bt, gram, gws, stream));
    float* Cn = cbuf[ci];
    NMF_DO(dfm_nmf_update_mm(batch, N, R, Ct, num_c, gram, eps, den_c, Cn, c16, copy, stream));
    const void* Cop = p.lp ? (const void*)c16 : (const void*)Cn;
    // B <- B * (x^T C) / (B (C^T C) + eps)
    NMF_DO(dfm_gemm(dtype, &p.xtc, x, Cop, num_b, gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &p.ctc, Cn, Cn, gram, gws, stream));
    float* Bn = bbuf[bi];
    NMF_DO(dfm_nmf_update_mm(batch, D, R, Bt, num_b, gram, eps, den_b, Bn, b16, copy, stream));
    Bop = p.lp ? (const void*)b16 : (const void*)Bn;
    Ct = Cn;
    Bt = Bn;
    ci ^= 1;
    bi ^= 1;
  }
  // compute_coef, then y = C B^T
  NMF_DO(dfm_gemm(dtype, &p.xb, x, Bop, num_c, gws, stream));
  NMF_DO(dfm_gemm(DFM_F32, &p.btb, Bt, Bt, gram, gws, stream));
  float* Cf = cbuf[ci];
  NMF_DO(dfm_nmf_update_mm(batch, N, R, Ct, num_c, gram, eps, den_c, Cf, c16, copy, stream));
  const void* Cfop = p.lp ? (const void*)c16 : (const void*)Cf;
  NMF_DO(dfm_gemm(dtype, &p.out, Cfop, Bop, y, gws, stream));
#undef NMF_DO
  return DFM_OK;
}
