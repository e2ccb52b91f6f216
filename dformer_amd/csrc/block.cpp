// Host-side composition of DFormer's encoder Block (DFormer.py:147-181) out of the library's kernels:
// dfm_block_fwd / dfm_block_bwd (include/dformer_hip.h), the same launch sequence as the Python
// autograd Functions of dformer_amd/functional.py (AttentionFn, ConvFFNFn) on one stream, with the
// ConvFFNs on the fused dfm_convffn_* kernels where they exist and the op-level chain elsewhere.
//
// Every entry point runs its sequence twice: a planning pass that only sizes the three arenas
// (saved activations that live from the forward to the backward, temporaries of the call, and the
// per-launch scratch the kernels' own workspaces need, reused launch after launch on the one stream),
// then the launching pass over the caller's buffers. The same code decides both, so the sizes the
// *_size functions report are exactly what the launches use.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <math.h>
#include <string.h>

#include "../../include/dformer_hip.h"

void dfm_set_error(const char* fmt, ...);

namespace {

constexpr size_t kAlign = 256;
size_t up(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

// a bump allocator over one caller buffer; in the planning pass base is null and only sizes count
struct Arena {
  char* base = nullptr;
  size_t off = 0, peak = 0;
  void* take(size_t bytes) {
    void* p = base ? base + off : nullptr;
    off += up(bytes);
    if (off > peak) peak = off;
    return p;
  }
};

// a [rows][cols] view with row stride ld (elements); col(c) = the view starting at column c
struct V {
  void* p = nullptr;
  long ld = 0;
  size_t es = 2;
  V col(long c) const { return V{p ? static_cast<char*>(p) + c * es : nullptr, ld, es}; }
};

struct Run {
  int dt;
  size_t es;
  hipStream_t s;
  bool plan;
  Arena saved, tmp;
  size_t scratch_need = 0;
  char* scratch = nullptr;
  size_t scratch_cap = 0;
  int err = DFM_OK;

  Run(int dtype, bool planning, hipStream_t st) : dt(dtype), es(dtype == DFM_F32 ? 4 : 2), s(st), plan(planning) {}
  V act(long rows, long cols, Arena& a) { return V{a.take((size_t)rows * cols * es), cols, es}; }
  V keep(long rows, long cols) { return act(rows, cols, saved); }
  V temp(long rows, long cols) { return act(rows, cols, tmp); }
  float* keepf(long n) { return static_cast<float*>(saved.take((size_t)n * 4)); }
  void* scr(size_t bytes) {
    if (bytes > scratch_need) scratch_need = bytes;
    return bytes ? scratch : nullptr;
  }
  bool ok(int rc) {
    if (rc != DFM_OK && err == DFM_OK) err = rc;
    return err == DFM_OK;
  }
  bool live() const { return !plan && err == DFM_OK; }
};

// ---------------------------------------------------------------- GEMM helpers (nn.Linear and its backward)
DfmGemmDesc gdesc() {
  DfmGemmDesc d;
  memset(&d, 0, sizeof(d));
  d.batch = 1;
  d.alpha = 1.f;
  d.rows_per_scale = 1;
  return d;
}

// GEMMs issued while a Group is open are collected and launched together (dfm_gemm_group: the
// independent forward / input-gradient GEMMs of one Block phase, as functional.AttentionFn does)
struct GemmBatch {
  int n = 0;
  DfmGemmDesc d[8];
  const void* A[8];
  const void* B[8];
  void* C[8];
};
thread_local GemmBatch* t_batch = nullptr;

void gemm(Run& r, DfmGemmDesc d, const void* A, const void* B, void* C) {
  if (t_batch && t_batch->n < 8) {
    const int i = t_batch->n++;
    t_batch->d[i] = d, t_batch->A[i] = A, t_batch->B[i] = B, t_batch->C[i] = C;
    return;
  }
  const size_t need = dfm_gemm_workspace_size(&d);
  void* ws = r.scr(need);
  d.workspace_bytes = (long)r.scratch_cap;
  if (r.live()) r.ok(dfm_gemm(r.dt, &d, A, B, C, ws, r.s));
}

struct Group {
  Run& r;
  GemmBatch b;
  explicit Group(Run& run) : r(run) { t_batch = &b; }
  ~Group() {
    t_batch = nullptr;
    if (b.n == 1) {
      gemm(r, b.d[0], b.A[0], b.B[0], b.C[0]);
      return;
    }
    if (b.n == 0) return;
    void* ws = r.scr(dfm_gemm_group_workspace_size(b.n, b.d));
    b.d[0].workspace_bytes = (long)r.scratch_cap;
    if (r.live()) r.ok(dfm_gemm_group(r.dt, b.n, b.d, b.A, b.B, b.C, ws, r.s));
  }
};

struct Epi {  // optional epilogue operands of a forward Linear (see DfmGemmDesc)
  int act = 0;
  int act_col0 = 0;
  V preact, mul, res;
  const float* colscale = nullptr;
  const float* rowscale = nullptr;
  long rps = 1;
};

// y[M][N] = epi(x[M][K] W[N][K]^T + b)
void linear(Run& r, V x, long M, long K, const void* w, long N, const float* b, V y, const Epi& e = Epi()) {
  DfmGemmDesc d = gdesc();
  d.M = (int)M, d.N = (int)N, d.K = (int)K;
  d.a_kcontig = 1, d.b_kcontig = 1;
  d.lda = x.ld, d.ldb = K, d.ldc = y.ld;
  d.bias = b;
  d.act = e.act, d.act_col0 = e.act_col0;
  d.preact = e.preact.p, d.ldpre = e.preact.ld;
  d.mul = e.mul.p, d.ldmul = e.mul.ld;
  d.res = e.res.p, d.ldres = e.res.ld;
  d.colscale = e.colscale, d.rowscale = e.rowscale, d.rows_per_scale = e.rps;
  gemm(r, d, x.p, w, y.p);
}

// dx[M][K] (+)= (dy[M][N] W[N][K]) (* mul)
void dgrad(Run& r, V dy, long M, long N, const void* w, long K, V dx, bool accumulate = false, V mul = V()) {
  DfmGemmDesc d = gdesc();
  d.M = (int)M, d.N = (int)K, d.K = (int)N;
  d.a_kcontig = 1, d.b_kcontig = 0;
  d.lda = dy.ld, d.ldb = K, d.ldc = dx.ld;
  d.beta = accumulate ? 1.f : 0.f;
  d.mul = mul.p, d.ldmul = mul.ld;
  gemm(r, d, dy.p, w, dx.p);
}

// dx[M][Kc] = (dy[M][N] W[N][k0 : k0 + Kc]) (* mul), dx2 = (dy W[N][k0 : k0 + Kc]) * mul2 (second epilogue
// output, when dx2 is given): column block k0 of an input gradient, W rows ldw elements apart
void dgrad_cols(Run& r, V dy, long M, long N, const void* w, long ldw, long k0, long Kc, V dx, V mul = V(),
                V mul2 = V(), V dx2 = V()) {
  DfmGemmDesc d = gdesc();
  d.M = (int)M, d.N = (int)Kc, d.K = (int)N;
  d.a_kcontig = 1, d.b_kcontig = 0;
  d.lda = dy.ld, d.ldb = ldw, d.ldc = dx.ld;
  d.mul = mul.p, d.ldmul = mul.ld;
  d.mul2 = mul2.p, d.ldmul2 = mul2.ld, d.out2 = dx2.p, d.ldout2 = dx2.ld;
  gemm(r, d, dy.p, w ? static_cast<const char*>(w) + k0 * r.es : nullptr, dx.p);
}

// dW[N][K] = dy[M][N]^T x[M][K] (float32), db[N] = sum_M dy
void wgrad(Run& r, V dy, long M, long N, V x, long K, float* dw, float* db) {
  DfmGemmDesc d = gdesc();
  d.M = (int)N, d.N = (int)K, d.K = (int)M;
  d.a_kcontig = 0, d.b_kcontig = 0;
  d.lda = dy.ld, d.ldb = x.ld, d.ldc = K;
  d.c_f32 = r.dt != DFM_F32;
  // every Linear of the Block has a bias: the planning pass (null gradient pointers) sizes the
  // workspace for the fused bias-gradient column all the same
  d.colsum = r.plan ? reinterpret_cast<float*>(16) : db;
  gemm(r, d, dy.p, x.p, dw);
}

// the kernels' own scratch (reduction partials) is taken from the shared per-launch scratch
void layernorm(Run& r, long rows, int C, V x, const float* g, const float* b, float eps, V y, float* mu, float* rs) {
  if (r.live()) r.ok(dfm_layernorm_fwd(r.dt, rows, C, x.p, x.ld, g, b, eps, y.p, y.ld, mu, rs, r.s));
}
void layernorm_bwd(Run& r, long rows, int C, V x, V dy, const float* g, const float* mu, const float* rs, V dres, V dx,
                   float* dg, float* db) {
  void* ws = r.scr(dfm_layernorm_bwd_workspace(rows, C));
  if (r.live())
    r.ok(dfm_layernorm_bwd(r.dt, rows, C, x.p, x.ld, dy.p, dy.ld, g, mu, rs, dres.p, dres.ld, dx.p, dx.ld, 0, dg, db, ws,
                           nullptr, r.s));
}
void residual_bwd(Run& r, long rows, int C, V dout, V f, const float* ls, const float* rowscale, long rps, V df,
                  float* dls) {
  void* ws = r.scr(dfm_residual_bwd_workspace(rows, C));
  if (r.live())
    r.ok(dfm_residual_bwd(r.dt, rows, C, dout.p, dout.ld, f.p, f.ld, ls, rowscale, rps, df.p, df.ld, dls, ws, nullptr,
                          r.s));
}

struct FfnSaved {  // what a ConvFFN's forward keeps for its backward
  V xn, h, f, gp, g;  // gp = GELU'(hpre), g = GELU(hpre): the op-level chain only
  float* mean = nullptr;
  float* rstd = nullptr;
};
struct FfnGrads {
  float *dln_w, *dln_b, *dw1, *db1, *dwpos, *dbpos, *dw2, *db2, *dls;
};

struct Shape {
  int B, H, W;
  long P() const { return (long)B * H * W; }
};

// ---------------------------------------------------------------- ConvFFN, op-level chain
// functional.ConvFFNFn (DFormer.py:48-67 inside the Block residual, 176-179): LN, fc1, DW3x3 + identity
// writing GELU'(hpre) and GELU(hpre) from one erf, fc2 with the residual / layer-scale / DropPath epilogue.
void ffn_chain_fwd(Run& r, Shape sh, int C, int R, float eps, V x, const float* ln_w, const float* ln_b, const void* w1,
                   const float* b1, const float* wpos, const float* bpos, const void* w2, const float* b2,
                   const float* ls, const float* rowscale, V out, const FfnSaved& sv) {
  const long P = sh.P();
  layernorm(r, P, C, x, ln_w, ln_b, eps, sv.xn, sv.mean, sv.rstd);
  linear(r, sv.xn, P, C, w1, R, b1, sv.h);
  if (r.live())
    r.ok(dfm_dwconv_fwd(r.dt, sh.B, sh.H, sh.W, R, 3, sv.h.p, sv.h.ld, wpos, bpos, 3, sv.gp.p, sv.gp.ld, sv.g.p,
                        sv.g.ld, r.s));
  Epi e;
  e.preact = sv.f, e.res = x, e.colscale = ls, e.rowscale = rowscale, e.rps = (long)sh.H * sh.W;
  linear(r, sv.g, P, R, w2, C, b2, out, e);
}

void ffn_chain_bwd(Run& r, Shape sh, int C, int R, V dout, V x, const FfnSaved& sv, const float* ln_w, const void* w1,
                   const float* wpos, const void* w2, const float* ls, const float* rowscale, V dx, const FfnGrads& gr) {
  const long P = sh.P();
  V df = r.temp(P, C);
  residual_bwd(r, P, C, dout, sv.f, ls, rowscale, (long)sh.H * sh.W, df, gr.dls);
  wgrad(r, df, P, C, sv.g, R, gr.dw2, gr.db2);
  V dhpre = r.temp(P, R);
  dgrad(r, df, P, C, w2, R, dhpre, false, sv.gp);  // GELU backward: times the stored GELU'(hpre)
  V dh = r.temp(P, R);
  void* ws = r.scr(dfm_dwconv_bwd_weight_workspace(sh.B, sh.H, sh.W, R, 3));
  if (r.live())
    r.ok(dfm_dwconv_bwd(r.dt, sh.B, sh.H, sh.W, R, 3, sv.h.p, sv.h.ld, dhpre.p, dhpre.ld, wpos, 1, dh.p, dh.ld, 0,
                        gr.dwpos, gr.dbpos, ws, nullptr, r.s));
  wgrad(r, dh, P, R, sv.xn, C, gr.dw1, gr.db1);
  V dxn = r.temp(P, C);
  dgrad(r, dh, P, R, w1, C, dxn);
  layernorm_bwd(r, P, C, x, dxn, ln_w, sv.mean, sv.rstd, dout, dx, gr.dln_w, gr.dln_b);
}

// ---------------------------------------------------------------- the Block
bool adjacent(const void* a, size_t bytes, const void* b) {
  return a && b && static_cast<const char*>(a) + bytes == static_cast<const char*>(b);
}

struct BlockIO {
  const void* const* p;  // params
  const float* rs[4];
  V x, xe;
};

struct AttnSaved {
  V xn, xen, qcl, lpre, apre, a, e1, e2, xep, f, p1, p1e, kv, pooled, m, o;
  float *mu1, *rs1, *mu2, *rs2, *lse;
  V x1, xe1;  // the attention outputs = the ConvFFN inputs
  FfnSaved ffn, ffne;
};

const float* F(const void* const* p, int i) { return static_cast<const float*>(p[i]); }

struct Dims {
  Shape sh;
  long P;
  int C, Ch, fw, R, heads, window, dhd;
  bool drop_depth, fused_ffn, fused_e;
  float eps;
};

Dims dims_of(int dtype, const DfmBlockDesc* d) {
  Dims m;
  m.sh = Shape{d->B, d->H, d->W};
  m.P = m.sh.P();
  m.C = d->C, m.Ch = d->C / 2;
  m.window = d->window;
  m.fw = d->window ? 2 * m.C : m.C + m.Ch;
  m.R = d->hidden;
  m.heads = d->heads;
  m.dhd = d->heads > 0 ? m.C / d->heads / 2 : 0;
  m.drop_depth = d->drop_depth != 0;
  m.eps = d->ln_eps;
  DfmConvFFNDesc fd{d->B, d->H, d->W, m.C, m.R, d->ln_eps};
  DfmConvFFNDesc fe{d->B, d->H, d->W, m.Ch, m.R / 2, d->ln_eps};
  m.fused_ffn = d->fused_ffn && dfm_convffn_supported(dtype, &fd);
  m.fused_e = d->fused_ffn && dfm_convffn_supported(dtype, &fe);
  return m;
}

FfnSaved ffn_saved(Run& r, long P, int C, int R, bool fused) {
  FfnSaved s;
  s.xn = r.keep(P, C);
  s.h = r.keep(P, R);
  s.f = r.keep(P, C);
  s.mean = r.keepf(P);
  s.rstd = r.keepf(P);
  if (!fused) {  // the op-level chain also keeps GELU'(hpre) and GELU(hpre)
    s.gp = r.keep(P, R);
    s.g = r.keep(P, R);
  }
  return s;
}

AttnSaved carve_saved(Run& r, const Dims& m) {
  AttnSaved s;
  const long P = m.P;
  const int C = m.C, Ch = m.Ch;
  s.xn = r.keep(P, C);
  s.xen = r.keep(P, Ch);
  s.mu1 = r.keepf(P), s.rs1 = r.keepf(P), s.mu2 = r.keepf(P), s.rs2 = r.keepf(P);
  s.qcl = r.keep(P, 2 * C + Ch);
  s.lpre = r.keep(P, C);
  s.apre = r.keep(P, C);
  s.a = r.keep(P, C);
  s.e1 = r.keep(P, Ch);
  s.e2 = r.keep(P, Ch);
  s.xep = r.keep(P, Ch);
  s.f = r.keep(P, m.fw);
  s.p1 = r.keep(P, C);
  s.x1 = r.keep(P, C);
  if (!m.drop_depth) {
    s.p1e = r.keep(P, Ch);
    s.xe1 = r.keep(P, Ch);
  }
  s.lse = nullptr;
  if (m.window) {
    s.kv = r.keep(P, C);
    s.pooled = r.keep((long)m.sh.B * 49, C + Ch);
    s.m = r.keep((long)m.sh.B * 49, Ch);
    s.o = r.keep((long)m.sh.B * 49, Ch);
    s.lse = r.keepf((long)m.sh.B * m.heads * 49);
  }
  s.ffn = ffn_saved(r, P, C, m.R, m.fused_ffn);
  if (!m.drop_depth) s.ffne = ffn_saved(r, P, Ch, m.R / 2, m.fused_e);
  return s;
}

void ffn_fwd(Run& r, const Dims& m, bool fused, int C, int R, V x, const void* const* p, int base, const float* ls,
             const float* rowscale, V out, const FfnSaved& sv) {
  const float *ln_w = F(p, base), *ln_b = F(p, base + 1), *b1 = F(p, base + 3), *wpos = F(p, base + 4),
              *bpos = F(p, base + 5), *b2 = F(p, base + 7);
  const void *w1 = p[base + 2], *w2 = p[base + 6];
  if (fused) {
    DfmConvFFNDesc fd{m.sh.B, m.sh.H, m.sh.W, C, R, m.eps};
    if (r.live())
      r.ok(dfm_convffn_fwd(r.dt, &fd, x.p, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls, rowscale, out.p, sv.f.p, sv.h.p,
                           sv.xn.p, sv.mean, sv.rstd, nullptr, nullptr, r.s));
    return;
  }
  ffn_chain_fwd(r, m.sh, C, R, m.eps, x, ln_w, ln_b, w1, b1, wpos, bpos, w2, b2, ls, rowscale, out, sv);
}

void ffn_bwd(Run& r, const Dims& m, bool fused, int C, int R, V dout, V x, const void* const* p, int base,
             const float* ls, const float* rowscale, V dx, float* const* g, int lsi, const FfnSaved& sv) {
  FfnGrads gr{g[base], g[base + 1], g[base + 2], g[base + 3], g[base + 4], g[base + 5], g[base + 6], g[base + 7], g[lsi]};
  if (fused) {
    DfmConvFFNDesc fd{m.sh.B, m.sh.H, m.sh.W, C, R, m.eps};
    const size_t need = dfm_convffn_bwd_workspace_size(r.dt, &fd);
    void* ws = r.scr(need);
    if (r.live())
      r.ok(dfm_convffn_bwd(r.dt, &fd, dout.p, x.p, sv.h.p, sv.xn.p, sv.f.p, sv.mean, sv.rstd, F(p, base), F(p, base + 1),
                           p[base + 2], F(p, base + 4), F(p, base + 5), p[base + 6], ls, rowscale, dx.p, gr.dln_w,
                           gr.dln_b, gr.dw1, gr.db1, gr.dwpos, gr.dbpos, gr.dw2, gr.db2, gr.dls, ws, r.scratch_cap,
                           r.s));
    return;
  }
  ffn_chain_bwd(r, m.sh, C, R, dout, x, sv, F(p, base), p[base + 2], F(p, base + 4), p[base + 6], ls, rowscale, dx,
                gr);
}

// AttentionFn.forward (functional.py) = DFormer.py:70-140 + the Block's first residuals (DFormer.py:173-175)
void block_fwd(Run& r, const Dims& m, const BlockIO& io, V y, V ye) {
  const void* const* p = io.p;
  AttnSaved s = carve_saved(r, m);
  const long P = m.P, rps = (long)m.sh.H * m.sh.W;
  const int C = m.C, Ch = m.Ch, fw = m.fw;
  layernorm(r, P, Ch, io.xe, F(p, DFM_BP_NORM_E_W), F(p, DFM_BP_NORM_E_B), m.eps, s.xen, s.mu2, s.rs2);
  layernorm(r, P, C, io.x, F(p, DFM_BP_NORM_W), F(p, DFM_BP_NORM_B), m.eps, s.xn, s.mu1, s.rs1);
  // q | q_cut | l: GELU on the l columns, GELU'(l pre-activation) kept in lpre
  const size_t es = r.es;
  const bool one = adjacent(p[DFM_BP_Q_W], (size_t)C * C * es, p[DFM_BP_QCUT_W]) &&
                   adjacent(p[DFM_BP_QCUT_W], (size_t)Ch * C * es, p[DFM_BP_L_W]) &&
                   adjacent(p[DFM_BP_Q_B], (size_t)C * 4, p[DFM_BP_QCUT_B]) &&
                   adjacent(p[DFM_BP_QCUT_B], (size_t)Ch * 4, p[DFM_BP_L_B]);
  Epi el;
  el.act = 3, el.preact = s.lpre;
  {
    Group grp(r);  // q | q_cut | l with e_fore
    if (one) {
      el.act_col0 = C + Ch;
      linear(r, s.xn, P, C, p[DFM_BP_Q_W], 2 * C + Ch, F(p, DFM_BP_Q_B), s.qcl, el);
    } else {
      linear(r, s.xn, P, C, p[DFM_BP_Q_W], C, F(p, DFM_BP_Q_B), s.qcl);
      linear(r, s.xn, P, C, p[DFM_BP_QCUT_W], Ch, F(p, DFM_BP_QCUT_B), s.qcl.col(C));
      linear(r, s.xn, P, C, p[DFM_BP_L_W], C, F(p, DFM_BP_L_B), s.qcl.col(C + Ch), el);
    }
    linear(r, s.xen, P, Ch, p[DFM_BP_EFORE_W], Ch, F(p, DFM_BP_EFORE_B), s.e1);
  }
  V q = s.qcl, cx = s.qcl.col(C), g = s.qcl.col(C + Ch);
  if (r.live())
    r.ok(dfm_dwconv_fwd(r.dt, m.sh.B, m.sh.H, m.sh.W, C, 7, g.p, g.ld, F(p, DFM_BP_CONV_W), F(p, DFM_BP_CONV_B), 0,
                        s.apre.p, s.apre.ld, nullptr, 0, r.s));
  if (r.live())
    r.ok(dfm_dwconv_fwd(r.dt, m.sh.B, m.sh.H, m.sh.W, Ch, 7, s.e1.p, s.e1.ld, F(p, DFM_BP_ECONV_W),
                        F(p, DFM_BP_ECONV_B), 0, s.e2.p, s.e2.ld, nullptr, 0, r.s));
  {
    Group grp(r);  // a with e_back and kv
    Epi ea;        // f[:, :C] = q * a(DW7(l)), a kept
    ea.mul = q, ea.preact = s.a;
    linear(r, s.apre, P, C, p[DFM_BP_A_W], C, F(p, DFM_BP_A_B), s.f, ea);
    Epi ee;  // f[:, fw - Ch:] = cx * e_back(DW7(e_fore(LN_e xe))), e_back's output kept
    ee.mul = cx, ee.preact = s.xep;
    linear(r, s.e2, P, Ch, p[DFM_BP_EBACK_W], Ch, F(p, DFM_BP_EBACK_B), s.f.col(fw - Ch), ee);
    if (m.window) linear(r, g, P, C, p[DFM_BP_KV_W], C, F(p, DFM_BP_KV_B), s.kv);
  }
  if (m.window) {  // softmax(q_pool k^T) v over the 7 x 7 pooled queries, upsampled into f[:, C:C+Ch]
    const int B = m.sh.B;
    if (r.live())
      r.ok(dfm_adaptive_pool7_fwd(r.dt, B, m.sh.H, m.sh.W, C, s.xn.p, s.xn.ld, s.pooled.p, s.pooled.ld, r.s));
    if (r.live())
      r.ok(dfm_adaptive_pool7_fwd(r.dt, B, m.sh.H, m.sh.W, Ch, s.xen.p, s.xen.ld, s.pooled.col(C).p, s.pooled.ld, r.s));
    linear(r, s.pooled, (long)B * 49, C + Ch, p[DFM_BP_SC_W], Ch, F(p, DFM_BP_SC_B), s.m);
    void* ws = r.scr(dfm_pooled_attn_workspace(B, m.heads, (int)(P / B), m.dhd));
    if (r.live())
      r.ok(dfm_pooled_attn_fwd(r.dt, B, m.heads, (int)(P / B), m.dhd, s.m.p, s.m.ld, s.kv.p, s.kv.col(Ch).p, s.kv.ld,
                               1.0f / sqrtf((float)m.dhd), s.o.p, s.o.ld, s.lse, ws, r.s));
    if (r.live())
      r.ok(dfm_bilinear_fwd(r.dt, B, 7, 7, m.sh.H, m.sh.W, Ch, s.o.p, s.o.ld, s.f.col(C).p, s.f.ld, 0, r.s));
  }
  {
    Group grp(r);  // proj with proj_e
    Epi ep;
    ep.preact = s.p1, ep.res = io.x, ep.colscale = F(p, DFM_BP_LS1), ep.rowscale = io.rs[0], ep.rps = rps;
    linear(r, s.f, P, fw, p[DFM_BP_PROJ_W], C, F(p, DFM_BP_PROJ_B), s.x1, ep);
    if (!m.drop_depth) {
      Epi epe;
      epe.preact = s.p1e, epe.res = io.xe, epe.colscale = F(p, DFM_BP_LS1E), epe.rowscale = io.rs[2], epe.rps = rps;
      linear(r, s.f, P, fw, p[DFM_BP_PROJE_W], Ch, F(p, DFM_BP_PROJE_B), s.xe1, epe);
    }
  }
  // the ConvFFNs with the Block's second residuals (DFormer.py:176-181)
  ffn_fwd(r, m, m.fused_ffn, C, m.R, s.x1, p, DFM_BP_MLP_NORM_W, F(p, DFM_BP_LS2), io.rs[1], y, s.ffn);
  if (!m.drop_depth)
    ffn_fwd(r, m, m.fused_e, Ch, m.R / 2, s.xe1, p, DFM_BP_MLPE_NORM_W, F(p, DFM_BP_LS2E), io.rs[3], ye, s.ffne);
  else if (ye.p && r.live())  // DFormer.py:133, 177-181: x_e leaves a drop_depth Block as e_back's output
    r.ok(dfm_scale_mul(r.dt, P, Ch, s.xep.p, s.xep.ld, nullptr, 0, nullptr, nullptr, 1, 1.f, ye.p, ye.ld, 0, r.s));
}

// AttentionFn._backward (functional.py), after both ConvFFN backwards
void block_bwd(Run& r, const Dims& m, const BlockIO& io, V dy, V dye, V dx, V dxe, float* const* gr) {
  const void* const* p = io.p;
  AttnSaved s = carve_saved(r, m);
  const long P = m.P, rps = (long)m.sh.H * m.sh.W;
  const int C = m.C, Ch = m.Ch, fw = m.fw, B = m.sh.B;
  const size_t es = r.es;
  V dx1 = r.temp(P, C);
  ffn_bwd(r, m, m.fused_ffn, C, m.R, dy, s.x1, p, DFM_BP_MLP_NORM_W, F(p, DFM_BP_LS2), io.rs[1], dx1, gr,
          DFM_BP_LS2, s.ffn);
  V dxe1;
  if (!m.drop_depth) {
    dxe1 = r.temp(P, Ch);
    ffn_bwd(r, m, m.fused_e, Ch, m.R / 2, dye, s.xe1, p, DFM_BP_MLPE_NORM_W, F(p, DFM_BP_LS2E), io.rs[3], dxe1, gr,
            DFM_BP_LS2E, s.ffne);
  }  // with drop_depth the x_e output is e_back's output (no identity path): dye joins dxe' below
  // proj / proj_e: one weight-gradient GEMM each, one input-gradient GEMM over [dp1 | dp1e] when the
  // two weights are stacked in memory
  V dpc = r.temp(P, C + Ch);
  residual_bwd(r, P, C, dx1, s.p1, F(p, DFM_BP_LS1), io.rs[0], rps, dpc, gr[DFM_BP_LS1]);
  wgrad(r, dpc, P, C, s.f, fw, gr[DFM_BP_PROJ_W], gr[DFM_BP_PROJ_B]);
  // the projections' input gradient df = dpc [Wp; Wpe] (one GEMM when the two weights are stacked in
  // memory, or Wp alone with drop_depth) by its column blocks f = cat(q * a, attn, cx * xe'), the two
  // products' backward in the epilogues (second output): dq = df_q a, da = df_q q; dcx = df_e xe',
  // dxe' = df_e cx; df is only materialised for the attention block (or, with separate weights, whole)
  const bool stacked = m.drop_depth || adjacent(p[DFM_BP_PROJ_W], (size_t)C * fw * es, p[DFM_BP_PROJE_W]);
  const long Kp = m.drop_depth ? C : C + Ch;
  if (!m.drop_depth) {
    residual_bwd(r, P, Ch, dxe1, s.p1e, F(p, DFM_BP_LS1E), io.rs[2], rps, dpc.col(C), gr[DFM_BP_LS1E]);
    wgrad(r, dpc.col(C), P, Ch, s.f, fw, gr[DFM_BP_PROJE_W], gr[DFM_BP_PROJE_B]);
  }
  V q = s.qcl, cx = s.qcl.col(C), g = s.qcl.col(C + Ch);
  V dqcl = r.temp(P, 2 * C + Ch);
  V dq = dqcl, dcx = dqcl.col(C), dl = dqcl.col(C + Ch);
  V da = r.temp(P, C), dxep = r.temp(P, Ch);
  V dfa;  // df's attention block (window only)
  if (stacked) {
    if (m.window) dfa = r.temp(P, Ch);
    Group grp(r);
    dgrad_cols(r, dpc, P, Kp, p[DFM_BP_PROJ_W], fw, 0, C, dq, s.a, q, da);
    dgrad_cols(r, dpc, P, Kp, p[DFM_BP_PROJ_W], fw, fw - Ch, Ch, dcx, s.xep, cx, dxep);
    if (m.window) dgrad_cols(r, dpc, P, Kp, p[DFM_BP_PROJ_W], fw, C, Ch, dfa);
  } else {
    V df = r.temp(P, fw);
    dgrad(r, dpc, P, C, p[DFM_BP_PROJ_W], fw, df);
    dgrad(r, dpc.col(C), P, Ch, p[DFM_BP_PROJE_W], fw, df, true);
    if (r.live())
      r.ok(dfm_dual_mul(r.dt, P, C, df.p, df.ld, s.a.p, s.a.ld, q.p, q.ld, dq.p, dq.ld, da.p, da.ld, r.s));
    if (r.live())
      r.ok(dfm_dual_mul(r.dt, P, Ch, df.col(fw - Ch).p, df.ld, s.xep.p, s.xep.ld, cx.p, cx.ld, dcx.p, dcx.ld, dxep.p,
                        dxep.ld, r.s));
    dfa = df.col(C);
  }
  // depth branch: cx * e_back(DW7(e_fore(LN_e xe)))
  if (m.drop_depth && dye.p && r.live())
    r.ok(dfm_scale_mul(r.dt, P, Ch, dye.p, dye.ld, nullptr, 0, nullptr, nullptr, 1, 1.f, dxep.p, dxep.ld, 1, r.s));
  wgrad(r, dxep, P, Ch, s.e2, Ch, gr[DFM_BP_EBACK_W], gr[DFM_BP_EBACK_B]);
  V de2 = r.temp(P, Ch);
  dgrad(r, dxep, P, Ch, p[DFM_BP_EBACK_W], Ch, de2);
  {
    void* ws = r.scr(dfm_dwconv_bwd_weight_workspace(B, m.sh.H, m.sh.W, Ch, 7));
    if (r.live())
      r.ok(dfm_dwconv_bwd_weight(r.dt, B, m.sh.H, m.sh.W, Ch, 7, s.e1.p, s.e1.ld, de2.p, de2.ld, gr[DFM_BP_ECONV_W],
                                 gr[DFM_BP_ECONV_B], ws, nullptr, r.s));
  }
  V de1 = r.temp(P, Ch);
  if (r.live())
    r.ok(dfm_dwconv_bwd_data(r.dt, B, m.sh.H, m.sh.W, Ch, 7, de2.p, de2.ld, F(p, DFM_BP_ECONV_W), 0, de1.p, de1.ld, 0,
                             r.s));
  wgrad(r, de1, P, Ch, s.xen, Ch, gr[DFM_BP_EFORE_W], gr[DFM_BP_EFORE_B]);
  V dxen = r.temp(P, Ch);
  dgrad(r, de1, P, Ch, p[DFM_BP_EFORE_W], Ch, dxen);
  // pooled-query attention
  V dg = r.temp(P, C), dxn = r.temp(P, C), dpooled, dkv;
  if (m.window) {
    const long B49 = (long)B * 49;
    V dout_o = r.temp(B49, Ch);
    if (r.live())
      r.ok(dfm_bilinear_bwd(r.dt, B, 7, 7, m.sh.H, m.sh.W, Ch, dfa.p, dfa.ld, dout_o.p, dout_o.ld, 0, r.s));
    V dm = r.temp(B49, Ch);
    dkv = r.temp(P, C);
    void* ws = r.scr(dfm_pooled_attn_workspace(B, m.heads, (int)(P / B), m.dhd));
    if (r.live())
      r.ok(dfm_pooled_attn_bwd(r.dt, B, m.heads, (int)(P / B), m.dhd, s.m.p, s.m.ld, s.kv.p, s.kv.col(Ch).p, s.kv.ld,
                               1.0f / sqrtf((float)m.dhd), s.o.p, s.o.ld, dout_o.p, dout_o.ld, s.lse, dm.p,
                               dkv.p, dkv.col(Ch).p, dkv.ld, ws, r.s));
    wgrad(r, dm, B49, Ch, s.pooled, C + Ch, gr[DFM_BP_SC_W], gr[DFM_BP_SC_B]);
    dpooled = r.temp(B49, C + Ch);
    dgrad(r, dm, B49, Ch, p[DFM_BP_SC_W], C + Ch, dpooled);
    if (r.live())
      r.ok(dfm_adaptive_pool7_bwd(r.dt, B, m.sh.H, m.sh.W, C, dpooled.p, dpooled.ld, dxn.p, dxn.ld, 0, r.s));
    wgrad(r, dkv, P, C, g, C, gr[DFM_BP_KV_W], gr[DFM_BP_KV_B]);
  }
  // q * a(DW7(l)) (dq, da from the projection's input-gradient epilogue)
  wgrad(r, da, P, C, s.apre, C, gr[DFM_BP_A_W], gr[DFM_BP_A_B]);
  V dapre = r.temp(P, C);
  {
    Group grp(r);  // the a and kv input gradients
    dgrad(r, da, P, C, p[DFM_BP_A_W], C, dapre);
    if (m.window) dgrad(r, dkv, P, C, p[DFM_BP_KV_W], C, dg);
  }
  {
    void* ws = r.scr(dfm_dwconv_bwd_weight_workspace(B, m.sh.H, m.sh.W, C, 7));
    if (r.live())
      r.ok(dfm_dwconv_bwd_weight(r.dt, B, m.sh.H, m.sh.W, C, 7, g.p, g.ld, dapre.p, dapre.ld, gr[DFM_BP_CONV_W],
                                 gr[DFM_BP_CONV_B], ws, nullptr, r.s));
  }
  if (r.live())
    r.ok(dfm_dwconv_bwd_data(r.dt, B, m.sh.H, m.sh.W, C, 7, dapre.p, dapre.ld, F(p, DFM_BP_CONV_W), 0, dg.p, dg.ld,
                             m.window ? 1 : 0, r.s));
  if (r.live())  // lpre holds GELU'(l pre-activation)
    r.ok(dfm_scale_mul(r.dt, P, C, dg.p, dg.ld, s.lpre.p, s.lpre.ld, nullptr, nullptr, 1, 1.f, dl.p, dl.ld, 0, r.s));
  if (m.window && r.live())
    r.ok(dfm_adaptive_pool7_bwd(r.dt, B, m.sh.H, m.sh.W, Ch, dpooled.col(C).p, dpooled.ld, dxen.p, dxen.ld, 1, r.s));
  // q | q_cut | l
  const bool one_w = adjacent(p[DFM_BP_Q_W], (size_t)C * C * es, p[DFM_BP_QCUT_W]) &&
                     adjacent(p[DFM_BP_QCUT_W], (size_t)Ch * C * es, p[DFM_BP_L_W]);
  wgrad(r, dq, P, C, s.xn, C, gr[DFM_BP_Q_W], gr[DFM_BP_Q_B]);
  wgrad(r, dcx, P, Ch, s.xn, C, gr[DFM_BP_QCUT_W], gr[DFM_BP_QCUT_B]);
  wgrad(r, dl, P, C, s.xn, C, gr[DFM_BP_L_W], gr[DFM_BP_L_B]);
  if (one_w) {
    dgrad(r, dqcl, P, 2 * C + Ch, p[DFM_BP_Q_W], C, dxn, m.window != 0);
  } else {
    dgrad(r, dq, P, C, p[DFM_BP_Q_W], C, dxn, m.window != 0);
    dgrad(r, dcx, P, Ch, p[DFM_BP_QCUT_W], C, dxn, true);
    dgrad(r, dl, P, C, p[DFM_BP_L_W], C, dxn, true);
  }
  layernorm_bwd(r, P, C, io.x, dxn, F(p, DFM_BP_NORM_W), s.mu1, s.rs1, dx1, dx, gr[DFM_BP_NORM_W], gr[DFM_BP_NORM_B]);
  layernorm_bwd(r, P, Ch, io.xe, dxen, F(p, DFM_BP_NORM_E_W), s.mu2, s.rs2, dxe1, dxe, gr[DFM_BP_NORM_E_W],
                gr[DFM_BP_NORM_E_B]);
}

// whether the Block described by m has parameter DFM_BP_i (kv / short_cut_linear need the window; proj_e,
// the _e layer scales and mlp_e2 are absent with drop_depth)
bool block_has_param(const Dims& m, int i) {
  if (!m.window && (i == DFM_BP_KV_W || i == DFM_BP_KV_B || i == DFM_BP_SC_W || i == DFM_BP_SC_B)) return false;
  if (m.drop_depth && (i == DFM_BP_PROJE_W || i == DFM_BP_PROJE_B || i == DFM_BP_LS1E || i == DFM_BP_LS2E ||
                       (i >= DFM_BP_MLPE_NORM_W && i <= DFM_BP_MLPE_FC2_B)))
    return false;
  return true;
}

bool desc_ok(int dtype, const DfmBlockDesc* d) {
  return d && (dtype == DFM_F32 || dtype == DFM_BF16 || dtype == DFM_F16) && d->B > 0 && d->H > 0 && d->W > 0 &&
         d->C > 0 && d->C % 16 == 0 && d->hidden > 0 && d->hidden % 16 == 0 &&
         (d->window == 0 || (d->window == 7 && d->heads > 0 && d->C % (2 * d->heads) == 0));
}

// sizes of (saved, workspace) for one Block
// Both parameter layouts are planned (separate q / q_cut / l and proj / proj_e weights, and the stacked ones
// the training step passes, which run as one GEMM): the planning pass only compares pointers, so the stacked
// layout is described by placeholder addresses that are never dereferenced.
void block_sizes(int dtype, const DfmBlockDesc* d, size_t* saved, size_t* ws) {
  const Dims m = dims_of(dtype, d);
  static float* const gnone[DFM_BLOCK_NPARAM] = {};
  const void* none[DFM_BLOCK_NPARAM] = {};
  const void* stacked[DFM_BLOCK_NPARAM] = {};
  const size_t es = dtype == DFM_F32 ? 4 : 2;
  char* const w0 = reinterpret_cast<char*>(size_t(1) << 40);
  char* const b0 = reinterpret_cast<char*>(size_t(1) << 41);
  char* const p0 = reinterpret_cast<char*>(size_t(1) << 42);
  stacked[DFM_BP_Q_W] = w0;
  stacked[DFM_BP_QCUT_W] = w0 + (size_t)m.C * m.C * es;
  stacked[DFM_BP_L_W] = w0 + (size_t)(m.C + m.Ch) * m.C * es;
  stacked[DFM_BP_Q_B] = b0;
  stacked[DFM_BP_QCUT_B] = b0 + (size_t)m.C * 4;
  stacked[DFM_BP_L_B] = b0 + (size_t)(m.C + m.Ch) * 4;
  stacked[DFM_BP_PROJ_W] = p0;
  stacked[DFM_BP_PROJE_W] = p0 + (size_t)m.C * m.fw * es;
  size_t sv = 0, tmp = 0, scr = 0;
  for (const void* const* params : {(const void* const*)none, (const void* const*)stacked}) {
    BlockIO io{params, {nullptr, nullptr, nullptr, nullptr}, V{nullptr, m.C, es}, V{nullptr, m.Ch, es}};
    Run f(dtype, true, nullptr), b(dtype, true, nullptr);
    block_fwd(f, m, io, V{nullptr, m.C, es}, V{nullptr, m.Ch, es});
    block_bwd(b, m, io, V{nullptr, m.C, es}, V{nullptr, m.Ch, es}, V{nullptr, m.C, es}, V{nullptr, m.Ch, es}, gnone);
    sv = std::max(sv, f.saved.peak);
    tmp = std::max({tmp, f.tmp.peak, b.tmp.peak});
    scr = std::max({scr, f.scratch_need, b.scratch_need});
  }
  *saved = sv;
  *ws = tmp + up(scr);
}

}  // namespace

// ---------------------------------------------------------------- Block entry points
extern "C" size_t dfm_block_saved_size(int dtype, const DfmBlockDesc* d) {
  if (!desc_ok(dtype, d)) return 0;
  size_t sv, ws;
  block_sizes(dtype, d, &sv, &ws);
  return sv;
}

extern "C" size_t dfm_block_workspace_size(int dtype, const DfmBlockDesc* d) {
  if (!desc_ok(dtype, d)) return 0;
  size_t sv, ws;
  block_sizes(dtype, d, &sv, &ws);
  return ws;
}

namespace {
int block_call(bool fwd, int dtype, const DfmBlockDesc* d, const void* const* params, const float* const* rowscale,
               const void* x, const void* xe, const void* saved, size_t saved_bytes, void* y, void* ye, const void* dy,
               const void* dye, void* dx, void* dxe, float* const* grads, void* workspace, size_t workspace_bytes,
               hipStream_t s) {
  const char* who = fwd ? "dfm_block_fwd" : "dfm_block_bwd";
  if (!desc_ok(dtype, d) || !params || !x || !xe) {
    dfm_set_error("%s: bad descriptor / dtype %d or null argument", who, dtype);
    return DFM_ERR_ARG;
  }
  const Dims m = dims_of(dtype, d);
  if (fwd ? (!y || (!m.drop_depth && !ye)) : (!dy || !dx || !dxe || !grads || (!m.drop_depth && !dye))) {
    dfm_set_error("%s: null output / gradient argument", who);
    return DFM_ERR_ARG;
  }
  size_t need_sv, need_ws;
  block_sizes(dtype, d, &need_sv, &need_ws);
  if (!saved || saved_bytes < need_sv || workspace_bytes < need_ws || !workspace) {
    dfm_set_error("%s: saved %zu / workspace %zu bytes, %zu / %zu needed", who, saved_bytes, workspace_bytes, need_sv,
                  need_ws);
    return DFM_ERR_ARG;
  }
  // every parameter (and, backward, every gradient slot) the Block has must be given: a NULL bias or
  // bias-gradient pointer would otherwise read as "no bias" / "skip" inside the GEMM epilogue
  for (int i = 0; i < DFM_BLOCK_NPARAM; ++i) {
    if (!block_has_param(m, i)) continue;
    if (!params[i] || (!fwd && !grads[i])) {
      dfm_set_error("%s: %s entry %d is NULL (the Block has this parameter)", who, params[i] ? "grads" : "params", i);
      return DFM_ERR_ARG;
    }
  }
  // the temporaries' peak of THIS direction decides where the scratch starts
  Run p(dtype, true, nullptr);
  const size_t es = p.es;
  BlockIO io{params, {nullptr, nullptr, nullptr, nullptr}, V{const_cast<void*>(x), m.C, es},
             V{const_cast<void*>(xe), m.Ch, es}};
  if (rowscale)
    for (int i = 0; i < 4; ++i) io.rs[i] = rowscale[i];
  static float* const gnone[DFM_BLOCK_NPARAM] = {};
  const V vy{y, m.C, es}, vye{ye, m.Ch, es}, vdy{const_cast<void*>(dy), m.C, es}, vdye{const_cast<void*>(dye), m.Ch, es},
      vdx{dx, m.C, es}, vdxe{dxe, m.Ch, es};
  if (fwd) block_fwd(p, m, io, vy, vye);
  else block_bwd(p, m, io, vdy, vdye, vdx, vdxe, gnone);
  Run r(dtype, false, s);
  r.saved.base = static_cast<char*>(const_cast<void*>(saved));
  r.tmp.base = static_cast<char*>(workspace);
  r.scratch = static_cast<char*>(workspace) + p.tmp.peak;
  r.scratch_cap = workspace_bytes - p.tmp.peak;
  if (fwd) block_fwd(r, m, io, vy, vye);
  else block_bwd(r, m, io, vdy, vdye, vdx, vdxe, grads);
  return r.err;
}
}  // namespace

extern "C" int dfm_block_fwd(int dtype, const DfmBlockDesc* d, const void* const* params, const float* const* rowscale,
                             const void* x, const void* xe, void* y, void* ye, void* saved, size_t saved_bytes,
                             void* workspace, size_t workspace_bytes, dfm_stream_t stream) {
  return block_call(true, dtype, d, params, rowscale, x, xe, saved, saved_bytes, y, ye, nullptr, nullptr, nullptr,
                    nullptr, nullptr, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dfm_block_bwd(int dtype, const DfmBlockDesc* d, const void* const* params, const float* const* rowscale,
                             const void* x, const void* xe, const void* saved, size_t saved_bytes, const void* dy,
                             const void* dye, void* dx, void* dxe, float* const* grads, void* workspace,
                             size_t workspace_bytes, dfm_stream_t stream) {
  return block_call(false, dtype, d, params, rowscale, x, xe, saved, saved_bytes, nullptr, nullptr, dy, dye, dx, dxe,
                    grads, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}
