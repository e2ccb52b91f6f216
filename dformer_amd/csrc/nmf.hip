// NMF2D forward and backward as library entry points (ham_head.py:60-145, MD_R = 64): the whole
// multiplicative-update loop of the Hamburger's matrix decomposition, and its gradient through every
// update, issued from the library. Host code only: it enqueues dfm_gemm / dfm_softmax_rows(_bwd) /
// dfm_cast / dfm_nmf_update_mm / dfm_nmf_update_bwd_mm / dfm_pack_slices on the caller's stream.
//
// Shapes per image (batch b), NHWC orientation (the reference's x^T):
//   x [N, D] (dtype), bases B0 [D, R] fp32, coef C [N, R] fp32, y = C B^T [N, D] (dtype)
//   coef = softmax_rows(x B0)                                         (ham_head.py:48-49, 116-117)
//   repeat steps:  C <- C * (x B) / (C (B^T B) + eps)                 (ham_head.py:120-128)
//                  B <- B * (x^T C) / (B (C^T C) + eps)               (ham_head.py:130-138)
//   C <- C * (x B) / (C (B^T B) + eps)                                (compute_coef, :140-141)
// For 16-bit x the x-streaming products take 16-bit copies of B / C (written by the update kernels)
// with fp32 accumulation; the factors, Gram matrices and updates stay fp32.
//
// Backward (the gradient of y w.r.t. x; the bases are a random constant): every update's gradient in
// reverse order (dfm_nmf_update_bwd_mm, with each den product's gradient and the symmetric Gram
// gradient of the next update folded in), the coef softmax's backward, and every rank-R contribution
// P Q^T to gx packed side by side and applied by ONE GEMM over K = (2 steps + 2) R.
#include "common.h"

#include <algorithm>
#include <vector>

namespace {

constexpr int NMF_RANK = 64;

DfmGemmDesc bmm_desc(int M, int N, int K, int batch, bool a_t, bool b_t, long lda, long ldb, long ldc, long sa,
                     long sb, long sc, int c_f32, float beta = 0.f) {
  DfmGemmDesc d{};
  d.M = M; d.N = N; d.K = K; d.batch = batch;
  d.a_kcontig = !a_t; d.b_kcontig = b_t;
  d.lda = lda; d.ldb = ldb; d.ldc = ldc;
  d.stride_a = sa; d.stride_b = sb; d.stride_c = sc;
  d.alpha = 1.f; d.beta = beta; d.c_f32 = c_f32;
  d.rows_per_scale = 1;
  return d;
}

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

struct Carve {  // sequential 256-byte aligned sub-buffers of one caller-owned buffer
  size_t off = 0;
  size_t take(size_t bytes) {
    const size_t at = off;
    off += al256(bytes);
    return at;
  }
};

// The descriptors decoders.NMF2DFn's K.bmm calls build (a [b][rows][cols] row-major per image).
struct NmfDescs {
  DfmGemmDesc xb, xtc, btb, ctc, out, xb_acc, xtc_acc, gx;
  size_t ws;
  NmfDescs(int batch, long N, long D, int R, int steps, bool lp) {
    const int c32 = lp ? 1 : 0;
    xb = bmm_desc((int)N, R, (int)D, batch, false, false, D, R, R, N * D, D * R, N * R, c32);   // x B
    xtc = bmm_desc((int)D, R, (int)N, batch, true, false, D, R, R, N * D, N * R, D * R, c32);   // x^T C
    btb = bmm_desc(R, R, (int)D, batch, true, false, R, R, R, D * R, D * R, R * R, 0);          // B^T B
    ctc = bmm_desc(R, R, (int)N, batch, true, false, R, R, R, N * R, N * R, R * R, 0);          // C^T C
    out = bmm_desc((int)N, (int)D, R, batch, false, true, R, R, D, N * R, D * R, N * D, 0);     // C B^T
    xb_acc = xb;                                                                                 // gC += x g
    xb_acc.beta = 1.f;
    xtc_acc = xtc;                                                                               // gB += x^T g
    xtc_acc.beta = 1.f;
    const long KT = (long)(2 * steps + 2) * R;                                                   // sum P_i Q_i^T
    gx = bmm_desc((int)N, (int)D, (int)KT, batch, false, true, KT, KT, D, N * KT, D * KT, N * D, 0);
    ws = 1;
    for (const DfmGemmDesc* d : {&xb, &xtc, &btb, &ctc, &out, &xb_acc, &xtc_acc, &gx})
      ws = std::max(ws, dfm_gemm_workspace_size(d));
    for (DfmGemmDesc* d : {&xb, &xtc, &btb, &ctc, &out, &xb_acc, &xtc_acc, &gx}) d->workspace_bytes = (long)ws;
  }
};

// Where the forward's factors live: in `saved` (training: every step kept for the backward) or in
// a ping-pong set inside the workspace (inference).
struct FwdSlots {
  long fc, fb, fr;  // bytes of one [b][N][R] / [b][D][R] / [b][R][R] fp32 buffer
  bool keep;
  int steps;
  size_t c, b, num1, den1, m1, num2, den2, q, c16, b16, total;
  FwdSlots(int batch, long N, long D, int R, int steps_, bool lp, bool keep_) : steps(steps_) {
    keep = keep_;
    fc = (long)batch * N * R * 4;
    fb = (long)batch * D * R * 4;
    fr = (long)batch * R * R * 4;
    const int T = steps;
    Carve cv;
    const size_t afc = al256(fc), afb = al256(fb), afr = al256(fr);
    c = cv.take(afc * (keep ? T + 2 : 2));     // C_0 = coef, C_1 .. C_{T+1}
    b = cv.take(afb * (keep ? T + 1 : 2));     // B_1 .. B_T (B_0 is the caller's bases)
    num1 = cv.take(afc * (keep ? T + 1 : 1));  // x B_s           (s = 0 .. T)
    den1 = cv.take(afc * (keep ? T + 1 : 1));  // C_s (B_s^T B_s)
    m1 = cv.take(afr * (keep ? T + 1 : 1));    // B_s^T B_s
    num2 = cv.take(afb * (keep ? T + 1 : 1));  // x^T C_{s+1}     (s = 0 .. T-1)
    den2 = cv.take(afb * (keep ? T + 1 : 1));  // B_s (C^T C)
    q = cv.take(afr * (keep ? T + 1 : 1));     // C_{s+1}^T C_{s+1}
    c16 = lp ? cv.take((size_t)batch * N * R * 2) : 0;  // 16-bit copy of the latest C (final: C_{T+1})
    b16 = lp ? cv.take((size_t)batch * D * R * 2) : 0;  // 16-bit copy of the latest B (final: B_T)
    total = cv.off;
  }
  // C_s / B_s (s >= 1) / per-step buffers; inference reuses two (C, B) or one buffer
  size_t C(int s) const { return c + al256(fc) * (keep ? s : s & 1); }
  size_t Bk(int s) const { return b + al256(fb) * (keep ? s - 1 : s & 1); }
  size_t NUM1(int s) const { return num1 + al256(fc) * (keep ? s : 0); }
  size_t DEN1(int s) const { return den1 + al256(fc) * (keep ? s : 0); }
  size_t M1(int s) const { return m1 + al256(fr) * (keep ? s : 0); }
  size_t NUM2(int s) const { return num2 + al256(fb) * (keep ? s : 0); }
  size_t DEN2(int s) const { return den2 + al256(fb) * (keep ? s : 0); }
  size_t Q(int s) const { return q + al256(fr) * (keep ? s : 0); }
};

bool nmf_shape_ok(int dtype, int batch, long N, long D, int R, int steps) {
  return (dtype == DFM_F32 || dtype == DFM_BF16 || dtype == DFM_F16) && batch > 0 && N > 0 && D > 0 && steps >= 0 &&
         R == NMF_RANK;
}

#define NMF_DO(call)             \
  do {                           \
    const int rc_ = (call);      \
    if (rc_ != DFM_OK) return rc_; \
  } while (0)

}  // namespace

extern "C" size_t dfm_nmf_saved_size(int dtype, int batch, long N, long D, int R, int steps) {
  if (!nmf_shape_ok(dtype, batch, N, D, R, steps)) return 0;
  return FwdSlots(batch, N, D, R, steps, dtype != DFM_F32, true).total;
}

extern "C" size_t dfm_nmf_fwd_workspace_size(int dtype, int batch, long N, long D, int R, int steps) {
  if (!nmf_shape_ok(dtype, batch, N, D, R, steps)) return 0;
  const NmfDescs g(batch, N, D, R, steps, dtype != DFM_F32);
  return FwdSlots(batch, N, D, R, steps, dtype != DFM_F32, false).total + al256(g.ws);
}

extern "C" int dfm_nmf_fwd(int dtype, int batch, long N, long D, int R, int steps, float eps, const void* x,
                           const float* bases, void* y, void* saved, long saved_bytes, void* workspace,
                           long workspace_bytes, dfm_stream_t stream) {
  DFM_CHECK_ARG(x && bases && y && workspace, "dfm_nmf_fwd: null argument");
  DFM_CHECK_ARG(nmf_shape_ok(dtype, batch, N, D, R, steps),
                "dfm_nmf_fwd: unsupported dtype / shape (R=%d; the fused updates are rank 64)", R);
  const bool lp = dtype != DFM_F32, keep = saved != nullptr;
  const NmfDescs g(batch, N, D, R, steps, lp);
  const FwdSlots sl(batch, N, D, R, steps, lp, keep);
  DFM_CHECK_ARG(!keep || saved_bytes >= (long)sl.total, "dfm_nmf_fwd: saved %ld < %zu bytes", saved_bytes, sl.total);
  const size_t need = keep ? al256(g.ws) : sl.total + al256(g.ws);
  DFM_CHECK_ARG(workspace_bytes >= (long)need, "dfm_nmf_fwd: workspace %ld < %zu bytes", workspace_bytes, need);
  char* fs = keep ? (char*)saved : (char*)workspace;  // factor storage
  void* gws = (char*)workspace + (keep ? 0 : sl.total);
  auto F = [&](size_t off) { return (float*)(fs + off); };
  void* c16 = lp ? (void*)(fs + sl.c16) : nullptr;
  void* b16 = lp ? (void*)(fs + sl.b16) : nullptr;
  const int copy = lp ? dtype : 0;
  // coef = softmax(x B0); the 16-bit operand copy of B0 for the x products
  const float* Bt = bases;
  const void* Bop = bases;
  if (lp) {
    NMF_DO(dfm_cast(DFM_F32, dtype, (long)batch * D * R, bases, b16, stream));
    Bop = b16;
  }
  NMF_DO(dfm_gemm(dtype, &g.xb, x, Bop, F(sl.NUM1(0)), gws, stream));
  NMF_DO(dfm_softmax_rows((long)batch * N, R, F(sl.NUM1(0)), F(sl.C(0)), stream));
  for (int s = 0; s < steps; ++s) {
    // C_{s+1} = C_s * (x B_s) / (C_s (B_s^T B_s) + eps)
    const float* Cs = F(sl.C(s));
    // (step 0: NUM1(0) still holds x B_0, the softmax's input)
    if (s > 0) NMF_DO(dfm_gemm(dtype, &g.xb, x, Bop, F(sl.NUM1(s)), gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &g.btb, Bt, Bt, F(sl.M1(s)), gws, stream));
    float* Cn = F(sl.C(s + 1));
    NMF_DO(dfm_nmf_update_mm(batch, N, R, Cs, F(sl.NUM1(s)), F(sl.M1(s)), eps, F(sl.DEN1(s)), Cn, c16, copy, stream));
    // B_{s+1} = B_s * (x^T C_{s+1}) / (B_s (C^T C) + eps)
    NMF_DO(dfm_gemm(dtype, &g.xtc, x, lp ? (const void*)c16 : (const void*)Cn, F(sl.NUM2(s)), gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &g.ctc, Cn, Cn, F(sl.Q(s)), gws, stream));
    float* Bn = F(sl.Bk(s + 1));
    NMF_DO(dfm_nmf_update_mm(batch, D, R, Bt, F(sl.NUM2(s)), F(sl.Q(s)), eps, F(sl.DEN2(s)), Bn, b16, copy, stream));
    Bop = lp ? (const void*)b16 : (const void*)Bn;
    Bt = Bn;
  }
  // compute_coef, then y = C B^T
  const int T = steps;
  NMF_DO(dfm_gemm(dtype, &g.xb, x, Bop, F(sl.NUM1(T)), gws, stream));
  NMF_DO(dfm_gemm(DFM_F32, &g.btb, Bt, Bt, F(sl.M1(T)), gws, stream));
  float* Cf = F(sl.C(T + 1));
  NMF_DO(dfm_nmf_update_mm(batch, N, R, F(sl.C(T)), F(sl.NUM1(T)), F(sl.M1(T)), eps, F(sl.DEN1(T)), Cf, c16, copy,
                           stream));
  NMF_DO(dfm_gemm(dtype, &g.out, lp ? (const void*)c16 : (const void*)Cf, Bop, y, gws, stream));
  return DFM_OK;
}

namespace {
struct BwdSlots {
  size_t gnum_c, gnum_b, gc, gb, gden_c, gden_b, g16, sm, gq, pc, qc, gws, total;
  BwdSlots(int batch, long N, long D, int R, int steps, size_t es, size_t gemm_ws) {
    const size_t fc = al256((size_t)batch * N * R * 4), fb = al256((size_t)batch * D * R * 4);
    const size_t fr = al256((size_t)batch * R * R * 4);
    const long KT = (long)(2 * steps + 2) * R;
    Carve cv;
    gnum_c = cv.take(fc * (steps + 2));  // the P operands computed here: gnum (final), gnum1_s, gS
    gnum_b = cv.take(fb * (steps + 1));  // the Q operands computed here: gnum2_s
    gc = cv.take(fc * 2);
    gb = cv.take(fb * 2);
    gden_c = cv.take(fc);
    gden_b = cv.take(fb);
    g16 = cv.take((size_t)batch * std::max(N, D) * R * es);
    sm = cv.take(fr);
    gq = cv.take(fr);
    pc = cv.take((size_t)batch * N * KT * es);
    qc = cv.take((size_t)batch * D * KT * es);
    gws = cv.take(gemm_ws);
    total = cv.off;
  }
};
}  // namespace

extern "C" size_t dfm_nmf_bwd_workspace_size(int dtype, int batch, long N, long D, int R, int steps) {
  if (!nmf_shape_ok(dtype, batch, N, D, R, steps)) return 0;
  const NmfDescs g(batch, N, D, R, steps, dtype != DFM_F32);
  return BwdSlots(batch, N, D, R, steps, dtype == DFM_F32 ? 4 : 2, g.ws).total;
}

extern "C" int dfm_nmf_bwd(int dtype, int batch, long N, long D, int R, int steps, float eps, const void* x,
                           const float* bases, const void* saved, long saved_bytes, const void* gy, void* gx,
                           void* workspace, long workspace_bytes, dfm_stream_t stream) {
  DFM_CHECK_ARG(x && bases && saved && gy && gx && workspace, "dfm_nmf_bwd: null argument");
  DFM_CHECK_ARG(nmf_shape_ok(dtype, batch, N, D, R, steps),
                "dfm_nmf_bwd: unsupported dtype / shape (R=%d; the fused updates are rank 64)", R);
  const bool lp = dtype != DFM_F32;
  const NmfDescs g(batch, N, D, R, steps, lp);
  const FwdSlots sl(batch, N, D, R, steps, lp, true);
  const BwdSlots w(batch, N, D, R, steps, lp ? 2 : 4, g.ws);
  DFM_CHECK_ARG(saved_bytes >= (long)sl.total, "dfm_nmf_bwd: saved %ld < %zu bytes", saved_bytes, sl.total);
  DFM_CHECK_ARG(workspace_bytes >= (long)w.total, "dfm_nmf_bwd: workspace %ld < %zu bytes", workspace_bytes, w.total);
  const char* fs = (const char*)saved;
  char* ws = (char*)workspace;
  auto S = [&](size_t off) { return (const float*)(fs + off); };
  auto W = [&](size_t off) { return (float*)(ws + off); };
  const size_t fc = al256((size_t)batch * N * R * 4), fb = al256((size_t)batch * D * R * 4);
  auto Bs = [&](int s) { return s == 0 ? bases : S(sl.Bk(s)); };
  const int T = steps, copy = lp ? dtype : 0;
  void* gws = ws + w.gws;
  void* g16 = lp ? (void*)(ws + w.g16) : nullptr;
  float* gden_c = W(w.gden_c);
  float* gden_b = W(w.gden_b);
  float* sm = W(w.sm);
  float* gq = W(w.gq);
  std::vector<const void*> P, Q;  // gx = sum_i P_i Q_i^T
  int gci = 0, gbi = 0;
  auto gC_buf = [&](int i) { return W(w.gc + fc * i); };
  auto gB_buf = [&](int i) { return W(w.gb + fb * i); };
  int pn = 0;
  auto gnum_c = [&]() { return W(w.gnum_c + fc * (pn++)); };
  int qn = 0;
  auto gnum_b = [&]() { return W(w.gnum_b + fb * (qn++)); };
  const void* Bt16 = lp ? (const void*)(fs + sl.b16) : (const void*)Bs(T);
  const void* Cf16 = lp ? (const void*)(fs + sl.c16) : (const void*)S(sl.C(T + 1));
  // gC = gy B_T, gB = gy^T C_{T+1}
  float* gC = gC_buf(gci);
  float* gB = gB_buf(gbi);
  NMF_DO(dfm_gemm(dtype, &g.xb, gy, Bt16, gC, gws, stream));
  NMF_DO(dfm_gemm(dtype, &g.xtc, gy, Cf16, gB, gws, stream));
  // final coef update C_{T+1} = C_T * num / (C_T M + eps): ga = gC_T (+ gden M), gnum, gden
  {
    float* gCt = gC_buf(gci ^= 1);
    float* gnum = gnum_c();
    NMF_DO(dfm_nmf_update_bwd_mm(batch, N, R, gC, nullptr, nullptr, S(sl.C(T)), S(sl.NUM1(T)), S(sl.DEN1(T)),
                                 S(sl.C(T + 1)), eps, S(sl.M1(T)), gCt, 0, gnum, gden_c, g16, copy, stream));
    P.push_back(gnum);  // gx += gnum B_T^T
    Q.push_back(Bs(T));
    NMF_DO(dfm_gemm(dtype, &g.xtc_acc, x, lp ? (const void*)g16 : (const void*)gnum, gB, gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &g.ctc, S(sl.C(T)), gden_c, sm, gws, stream));  // pending: B_T (gM + gM^T)
    gC = gCt;
  }
  const float* pendA = Bs(T);
  for (int s = T - 1; s >= 0; --s) {
    // B-update B_{s+1} = B_s * num2 / (B_s Q + eps), with gB += B_{s+1} (S + S^T) folded in
    float* gBp = gB_buf(gbi ^= 1);
    float* gnum2 = gnum_b();
    NMF_DO(dfm_nmf_update_bwd_mm(batch, D, R, gB, pendA, sm, Bs(s), S(sl.NUM2(s)), S(sl.DEN2(s)), Bs(s + 1), eps,
                                 S(sl.Q(s)), gBp, 0, gnum2, gden_b, g16, copy, stream));
    P.push_back(S(sl.C(s + 1)));  // gx += C_{s+1} gnum2^T
    Q.push_back(gnum2);
    NMF_DO(dfm_gemm(dtype, &g.xb_acc, x, lp ? (const void*)g16 : (const void*)gnum2, gC, gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &g.btb, Bs(s), gden_b, gq, gws, stream));  // gQ = B_s^T gden2
    // C-update C_{s+1} = C_s * num1 / (C_s M1 + eps), with gC += C_{s+1} (gQ + gQ^T) folded in
    float* gCp = gC_buf(gci ^= 1);
    float* gnum1 = gnum_c();
    NMF_DO(dfm_nmf_update_bwd_mm(batch, N, R, gC, S(sl.C(s + 1)), gq, S(sl.C(s)), S(sl.NUM1(s)), S(sl.DEN1(s)),
                                 S(sl.C(s + 1)), eps, S(sl.M1(s)), gCp, 0, gnum1, gden_c, g16, copy, stream));
    P.push_back(gnum1);  // gx += gnum1 B_s^T
    Q.push_back(Bs(s));
    NMF_DO(dfm_gemm(dtype, &g.xtc_acc, x, lp ? (const void*)g16 : (const void*)gnum1, gBp, gws, stream));
    NMF_DO(dfm_gemm(DFM_F32, &g.ctc, S(sl.C(s)), gden_c, sm, gws, stream));  // pending: B_s (gM1 + gM1^T)
    pendA = Bs(s);
    gB = gBp;
    gC = gCp;
  }
  // (the pending Gram term belongs to the random bases B0: no gradient); coef = softmax(x B0)
  float* gS = gnum_c();
  NMF_DO(dfm_softmax_rows_bwd((long)batch * N, R, S(sl.C(0)), gC, gS, 0, stream));
  P.push_back(gS);  // gx += gS B0^T
  Q.push_back(bases);
  const int n = (int)P.size();
  DFM_CHECK_ARG(n == 2 * T + 2, "dfm_nmf_bwd: internal term count %d", n);
  std::vector<int> f32(n, DFM_F32);
  NMF_DO(dfm_pack_slices(dtype, n, P.data(), f32.data(), (long)batch * N, R, ws + w.pc, stream));
  NMF_DO(dfm_pack_slices(dtype, n, Q.data(), f32.data(), (long)batch * D, R, ws + w.qc, stream));
  NMF_DO(dfm_gemm(dtype, &g.gx, ws + w.pc, ws + w.qc, gx, gws, stream));
  return DFM_OK;
}
