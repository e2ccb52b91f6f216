#pragma once
// MFMA GEMM for gfx950 with fused epilogues (DFormer linears / 1x1 convs / NMF bmm) — kernels and
// host-side tile selection (included by gemm.hip, the C entry points, and the per-dtype units).
//
// One templated kernel covers the three layouts of a linear layer's forward and backward:
//   forward  Y  = X W^T   : A k-contiguous, B k-contiguous
//   dgrad    dX = dY W    : A k-contiguous, B row-contiguous   (ds_read_b64_tr_b16 for B)
//   wgrad    dW = dY^T X  : A row-contiguous, B row-contiguous (split-K over pixels); the bias
//                           gradient sum_p dY[p, :] rides along as a virtual all-ones column of X
// bf16 operands use v_mfma_f32_16x16x32_bf16 (fp32 accumulate); float32 operands use the
// exact-f32 v_mfma_f32_16x16x4_f32. Both operands are staged through a double-buffered LDS
// tile filled by 16-byte register-staged loads; row-contiguous bf16 tiles are consumed with
// the hardware transposing LDS read so no operand is ever transposed in memory.
// The epilogue stages the fp32 accumulator tile through LDS (two row halves) and applies bias /
// activation / multiplier / residual on 8-column vectors, so every global read and write of the
// output side is a coalesced 16-byte access (these GEMMs are mostly HBM-bound: K <= 2048).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  float* ws;
  int M, N, K, batch, splits, Nw, ldw;  // ldw: split-K workspace row stride (Nw rounded up to 8)
  long lda, ldb, ldc, sa, sb, sc;
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
  long rps;
  int act_col0;
  float* colsum;   // optional: colsum[m] (+)= alpha * sum_k A(m,k)  (virtual ones column of B)
  int colsum_acc;
  int ala, alb;    // operand rows 16-byte aligned (vector loads)
  int vec_ok;      // output-side rows 16-byte aligned (vector epilogue)
  int mul_gelu_grad;
  int tiles_n;     // output column tiles (grid.x enumerates tiles_m * tiles_n)
  int tiles_m;     // output row tiles (glds kernel)
  int n_fast;      // glds kernel: consecutive (XCD-local) blocks walk column tiles of one row tile
  int xcd_map;     // gemm_kernel: XCD-aware block renumbering (always on)
  const void* mul2;  // optional second output C2[m, n] = (value before mul / res) * mul2[m, n]
  long ldmul2;
  void* C2;
  long ldc2;
};


template <typename T> struct Mf;
template <> struct Mf<bf16_t> {
  static constexpr int VEC = 8;    // elements per 16-byte vector
  static constexpr int KSTEP = 32; // k per MFMA
  static constexpr int PADK = 16;  // k-contiguous row pad: rows 160 B apart, conflict-free ds_read_b128 fragments
  static constexpr int PADR = 0;   // row-contiguous rows: no pad, 16-byte chunks XOR-swizzled (tr_swz)
};
template <> struct Mf<f16_t> : Mf<bf16_t> {};
template <> struct Mf<float> {
  static constexpr int VEC = 4;
  static constexpr int KSTEP = 4;
  static constexpr int PADK = 1;
  static constexpr int PADR = 16;
};

// Load one 16-byte vector (VEC elements) of operand tile element (r, k..k+VEC) or (k, r..r+VEC)
// with zero fill outside [0, rows) x [0, K).
template <typename T, bool KC>
DFM_INLINE uint4 load_vec(const T* __restrict__ p, long ld, int r, int k, int rows, int K, bool aligned,
                          int ones_r) {
  constexpr int VEC = Mf<T>::VEC;
  uint4 out = make_uint4(0, 0, 0, 0);
  if (KC) {
    if (r == ones_r) {  // virtual all-ones row (bias-gradient column of a wgrad GEMM)
      T tmp[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) tmp[e] = Num<T>::from_f(k + e < K ? 1.0f : 0.0f);
      return *reinterpret_cast<uint4*>(tmp);
    }
    if (r >= rows) return out;
    const T* src = p + (long)r * ld + k;
    if (aligned && k + VEC <= K) return *reinterpret_cast<const uint4*>(src);
    T tmp[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) tmp[e] = (k + e < K) ? src[e] : Num<T>::from_f(0.f);
    return *reinterpret_cast<uint4*>(tmp);
  } else {
    if (k >= K) return out;
    const T* src = p + (long)k * ld + r;
    if (aligned && r + VEC <= rows) return *reinterpret_cast<const uint4*>(src);
    T tmp[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) tmp[e] = (r + e < rows) ? src[e] : Num<T>::from_f(r + e == ones_r ? 1.0f : 0.0f);
    return *reinterpret_cast<uint4*>(tmp);
  }
}

template <typename T, int R, int BK, bool KC, int NT>
struct TileGeom {
  static constexpr int VEC = Mf<T>::VEC;
  // k-contiguous: [R][BK+PADK]; row-contiguous: [BK][R+PADR]
  static constexpr int LD = KC ? (BK + Mf<T>::PADK) : (R + Mf<T>::PADR);
  static constexpr int ELEMS = KC ? R * LD : BK * LD;
  static constexpr int TOTAL = R * BK / VEC;        // 16-byte vectors per tile
  static constexpr int NVEC = (TOTAL + NT - 1) / NT;  // vectors per thread (last one partial)
};

// Guarded tile load: zero fill outside [0, rows) x [0, K), scalar fallback for unaligned rows.
template <typename T, int R, int BK, bool KC, int NT>
DFM_INLINE void stage_load(uint4* regs, const T* __restrict__ base, long ld, int r0, int k0, int rows, int K,
                           bool aligned, int ones_r = -1) {
  using G = TileGeom<T, R, BK, KC, NT>;
  constexpr int VEC = G::VEC;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    const int v = threadIdx.x + i * NT;
    if (G::TOTAL % NT != 0 && v >= G::TOTAL) break;
    if (KC) {
      const int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
      regs[i] = load_vec<T, true>(base, ld, r0 + r, k0 + kc, rows, K, aligned, ones_r);
    } else {
      const int k = v / (R / VEC), rc = (v % (R / VEC)) * VEC;
      regs[i] = load_vec<T, false>(base, ld, r0 + rc, k0 + k, rows, K, aligned, ones_r);
    }
  }
}

// Branch-free tile loads for a k-range fully inside [0, K) with 16-byte aligned rows. Each
// thread's byte offsets inside the tile are computed once per block (rows past the edge point
// at a clamped in-bounds row instead of being zero-filled: they only feed output rows / columns
// that are never stored); per k-slice only the wave-uniform tile base moves, so every load is
// one unconditional `global_load_dwordx4 v, v_off, s_base`.
template <typename T, int R, int BK, bool KC, int NT>
DFM_INLINE void fast_offsets(unsigned* off, long ld, int r0, int rows) {
  using G = TileGeom<T, R, BK, KC, NT>;
  constexpr int VEC = G::VEC;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    int v = threadIdx.x + i * NT;
    if (G::TOTAL % NT != 0 && v >= G::TOTAL) v = 0;
    if (KC) {
      const int r = r0 + v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
      const int rr = r < rows ? r : rows - 1;
      off[i] = (unsigned)(((long)rr * ld + kc) * sizeof(T));
    } else {
      const int k = v / (R / VEC), rc = r0 + (v % (R / VEC)) * VEC;
      const int rr = rc < rows ? rc : 0;
      off[i] = (unsigned)(((long)k * ld + rr) * sizeof(T));
    }
  }
}

template <typename T, int R, int BK, bool KC, int NT>
DFM_INLINE void stage_load_fast(uint4* regs, __amdgpu_buffer_rsrc_t rsrc, int soff, const unsigned* off) {
  using G = TileGeom<T, R, BK, KC, NT>;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    if (G::TOTAL % NT != 0 && threadIdx.x + i * NT >= G::TOTAL) break;
    regs[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off[i], soff, 0));
  }
}

// After a fast load: write the virtual all-ones operand row `ones_r` (fused bias gradient) into
// the staged registers. Applied right before the LDS store, when the loads have landed anyway.
// bits of 1.0 in one 16-bit element (bf16 0x3f80, f16 0x3c00)
template <typename T>
constexpr unsigned one16() { return std::is_same<T, f16_t>::value ? 0x3c00u : 0x3f80u; }
template <typename T>
DFM_INLINE unsigned one_bits() { return sizeof(T) == 2 ? one16<T>() : 0x3f800000u; }

template <typename T>
DFM_INLINE uint4 set_one(uint4 u, int e) {  // element e (0 <= e < VEC, or no-op) := 1.0
  unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (sizeof(T) == 2) {
      w[j] = (e == 2 * j) ? ((w[j] & 0xffff0000u) | one16<T>()) : w[j];
      w[j] = (e == 2 * j + 1) ? ((w[j] & 0x0000ffffu) | (one16<T>() << 16)) : w[j];
    } else {
      w[j] = (e == j) ? 0x3f800000u : w[j];
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <typename T, int R, int BK, bool KC, int NT>
DFM_INLINE void patch_ones(uint4* regs, int r0, int ones_r) {
  using G = TileGeom<T, R, BK, KC, NT>;
  constexpr int VEC = G::VEC;
  const unsigned one = sizeof(T) == 2 ? (one16<T>() | (one16<T>() << 16)) : 0x3f800000u;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    const int v = threadIdx.x + i * NT;
    if (G::TOTAL % NT != 0 && v >= G::TOTAL) break;
    if (KC) {
      if (r0 + v / (BK / VEC) == ones_r) regs[i] = make_uint4(one, one, one, one);
    } else {
      regs[i] = set_one<T>(regs[i], ones_r - (r0 + (v % (R / VEC)) * VEC));
    }
  }
}

// XOR swizzle of the 16-byte chunks of row k of a row-contiguous bf16 LDS tile (R elements per
// row, no pad): the 8 rows one ds_read_b64_tr_b16 lane group reads (k0 + 8g + q, g < 2, q < 4)
// land on 16 distinct 4-bank slots instead of 2-way conflicting, and the 8 consecutive lanes of a
// ds_write_b128 still hit distinct banks.
template <int R>
DFM_INLINE int tr_swz(int k) {
  if constexpr (R >= 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else if constexpr (R == 64) return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  else return 2 * ((k >> 3) & 1);
}

template <typename T, int R, int BK, bool KC, int NT>
DFM_INLINE void stage_store(const uint4* regs, T* lds) {
  using G = TileGeom<T, R, BK, KC, NT>;
  constexpr int VEC = G::VEC;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    const int v = threadIdx.x + i * NT;
    if (G::TOTAL % NT != 0 && v >= G::TOTAL) break;
    if (KC) {
      const int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
      *reinterpret_cast<uint4*>(lds + r * G::LD + kc) = regs[i];
    } else {
      const int k = v / (R / VEC), rc = (v % (R / VEC)) * VEC;
      if constexpr (sizeof(T) == 2)
        *reinterpret_cast<uint4*>(lds + k * G::LD + (((rc >> 3) ^ tr_swz<R>(k)) << 3)) = regs[i];
      else
        *reinterpret_cast<uint4*>(lds + k * G::LD + rc) = regs[i];
    }
  }
}

// ---- fragment reads
template <bool KC, int LD>
DFM_INLINE bf16x8_t frag_bf16(const bf16_t* lds, int r0, int k0, int lane) {
  if (KC) {
    const uint4 u = *reinterpret_cast<const uint4*>(lds + (r0 + (lane & 15)) * LD + k0 + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8_t, u);
  } else {
    const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
    typedef __attribute__((address_space(3))) short4_t lds_s4;
    const int k = k0 + 8 * g + q, r = r0 + 4 * p;  // LD == R (PADR = 0): swizzled 16-byte chunks
    const bf16_t* a0 = lds + k * LD + ((((r >> 3) ^ tr_swz<LD>(k)) << 3) | (r & 7));
    const bf16_t* a1 = lds + (k + 4) * LD + ((((r >> 3) ^ tr_swz<LD>(k + 4)) << 3) | (r & 7));
    short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
    short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a1));
    typedef __attribute__((ext_vector_type(8))) short short8_t;
    short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, s);
  }
}
template <bool KC, int LD>
DFM_INLINE float frag_f32(const float* lds, int r0, int k0, int lane) {
  if (KC) return lds[(r0 + (lane & 15)) * LD + k0 + (lane >> 4)];
  return lds[(k0 + (lane >> 4)) * LD + r0 + (lane & 15)];
}

// ---- epilogue (scalar element)
template <typename TO>
DFM_INLINE void epilogue_store(const GemmArgs& a, int b, int m, int n, float v) {
  if (n == a.N) {  // virtual ones column -> row sums (bias gradient)
    a.colsum[m] = a.colsum_acc ? a.colsum[m] + v : v;
    return;
  }
  const long ci = b * a.sc + (long)m * a.ldc + n;
  if (a.beta != 0.0f) v += a.beta * (a.c_f32 ? ((const float*)a.C)[ci] : ldf((const TO*)a.C + ci));
  if (a.bias) v += a.bias[n];
  if (n >= a.act_col0) {
    if (a.act == 3) {  // GELU; preact receives its derivative at the pre-activation
      float cdf, pdf;
      normal_cdf_pdf(v, cdf, pdf);
      if (a.preact) stf((TO*)a.preact + (long)m * a.ldpre + (n - a.act_col0), fmaf(v, pdf, cdf));
      v *= cdf;
    } else {
      if (a.preact) stf((TO*)a.preact + (long)m * a.ldpre + (n - a.act_col0), v);
      if (a.act == 1) v = gelu_f(v);
      else if (a.act == 2) v = fmaxf(v, 0.0f);
    }
  }
  if (a.C2) stf((TO*)a.C2 + (long)m * a.ldc2 + n, v * ldf((const TO*)a.mul2 + (long)m * a.ldmul2 + n));
  if (a.mul) {
    const float mv = ldf((const TO*)a.mul + (long)m * a.ldmul + n);
    v *= a.mul_gelu_grad ? gelu_grad_f(mv) : mv;
  }
  if (a.res) {
    float s = a.colscale ? a.colscale[n] : 1.0f;
    if (a.rowscale) s *= a.rowscale[m / a.rps];
    v = ldf((const TO*)a.res + (long)m * a.ldres + n) + s * v;
  }
  if (a.c_f32) ((float*)a.C)[ci] = v;
  else stf((TO*)a.C + ci, v);
}

// Epilogue inputs of one 8-column vector, loaded ahead of use (bf16 path) so a thread's loads for
// all of its vectors are in flight together.
template <typename TO>
struct EpiIn {
  Raw8<TO> mul, res, c, mul2;
};

template <typename TO>
DFM_INLINE void epi_load(const GemmArgs& a, int b, int m, int n, EpiIn<TO>& in) {
  if (a.beta != 0.0f && !a.c_f32) in.c = ldraw8<TO>((const TO*)a.C + b * a.sc + (long)m * a.ldc + n);
  if (a.mul) in.mul = ldraw8<TO>((const TO*)a.mul + (long)m * a.ldmul + n);
  if (a.C2) in.mul2 = ldraw8<TO>((const TO*)a.mul2 + (long)m * a.ldmul2 + n);
  if (a.res) in.res = ldraw8<TO>((const TO*)a.res + (long)m * a.ldres + n);
}

template <typename TO>
DFM_INLINE void epilogue8(const GemmArgs& a, int b, int m, int n, float* v, const EpiIn<TO>& in) {
  const long ci = b * a.sc + (long)m * a.ldc + n;
  float t[8];
  if (a.beta != 0.0f) {
    if (a.c_f32) ld8<float>((const float*)a.C + ci, t);
    else unpack8(in.c, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += a.beta * t[e];
  }
  if (a.bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += a.bias[n + e];
  }
  if (n >= a.act_col0 && a.act == 3) {  // GELU; preact receives its derivative at the pre-activation
    float dv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float cdf, pdf;
      normal_cdf_pdf(v[e], cdf, pdf);
      dv[e] = fmaf(v[e], pdf, cdf);
      v[e] *= cdf;
    }
    if (a.preact) st8<TO>((TO*)a.preact + (long)m * a.ldpre + (n - a.act_col0), dv);
  } else if (n >= a.act_col0) {  // act_col0 is a multiple of 8 whenever the vector path is taken
    if (a.preact) st8<TO>((TO*)a.preact + (long)m * a.ldpre + (n - a.act_col0), v);
    if (a.act == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
    } else if (a.act == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.0f);
    }
  }
  if (a.C2) {  // second output: the value before the multiplier times mul2
    float t2[8];
    unpack8(in.mul2, t2);
#pragma unroll
    for (int e = 0; e < 8; ++e) t2[e] *= v[e];
    st8<TO>((TO*)a.C2 + (long)m * a.ldc2 + n, t2);
  }
  if (a.mul) {
    unpack8(in.mul, t);
    if (a.mul_gelu_grad) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= gelu_grad_f(t[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= t[e];
    }
  }
  if (a.res) {
    unpack8(in.res, t);
    const float rs = a.rowscale ? a.rowscale[m / a.rps] : 1.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[e] + (a.colscale ? a.colscale[n + e] : 1.0f) * rs * v[e];
  }
  if (a.c_f32) st8<float>((float*)a.C + ci, v);
  else st8<TO>((TO*)a.C + ci, v);
}

// Epilogue of one BM x BN accumulator tile: -> LDS (fp32, RP rows per pass: two 8-column vectors
// per thread per pass) -> 8-column vectors with all of a pass's global loads issued together; or
// the fp32 split-K partial tile into the workspace. Ends with the LDS free (trailing barrier).
template <typename T, int BM, int BN, int NW, int WAVES_M>
DFM_INLINE void gemm_epilogue(const GemmArgs& a, float4_t (&acc)[BM / WAVES_M / 16][BN / (NW / WAVES_M) / 16],
                              char* smem, int bm, int bn, int b, int split) {
  constexpr int NT = 64 * NW;
  constexpr int WAVES_N = NW / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  constexpr int TPR = BN / 8;  // threads per row
  constexpr int RP = (2 * NT / TPR) < BM ? (2 * NT / TPR) : BM;
  constexpr int HALF = RP;
  constexpr int CLD = BN + 4;
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int half = 0; half < BM / RP; ++half) {
    __builtin_amdgcn_sched_barrier(0);  // keep each pass's loads in their pass (register pressure)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if ((wm * WM + i * 16) / RP != half) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WM + i * 16 + (lane >> 4) * 4 + r - half * RP;
          cs[row * CLD + col] = acc[i][j][r] * a.alpha;
        }
      }
    }
    lds_barrier();
    constexpr int ITEMS = (HALF * TPR + NT - 1) / NT;
    if (a.splits > 1) {  // fp32 partial tile -> workspace rows padded to ldw (16-byte stores)
#pragma unroll
      for (int it = 0; it < ITEMS; ++it) {
        const int idx = threadIdx.x + it * NT;
        const int row = idx / TPR, c8 = (idx % TPR) * 8;
        const int m = bm + half * HALF + row, n = bn + c8;
        if (idx >= HALF * TPR || m >= a.M || n >= a.Nw) continue;
        float4* wp = reinterpret_cast<float4*>(a.ws + (((long)split * a.batch + b) * a.M + m) * a.ldw + n);
        const float* cv = cs + row * CLD + c8;
        wp[0] = make_float4(cv[0], cv[1], cv[2], cv[3]);
        wp[1] = make_float4(cv[4], cv[5], cv[6], cv[7]);
      }
    } else {
      EpiIn<T> in[ITEMS];
      bool vec[ITEMS];
#pragma unroll
      for (int it = 0; it < ITEMS; ++it) {  // issue every vector's loads first
        const int idx = threadIdx.x + it * NT;
        const int row = idx / TPR, c8 = (idx % TPR) * 8;
        const int m = bm + half * HALF + row, n = bn + c8;
        vec[it] = idx < HALF * TPR && m < a.M && a.vec_ok && n + 8 <= a.N &&
                  (a.act_col0 <= n || a.act_col0 >= n + 8);
        if (vec[it]) epi_load<T>(a, b, m, n, in[it]);
      }
#pragma unroll
      for (int it = 0; it < ITEMS; ++it) {
        const int idx = threadIdx.x + it * NT;
        const int row = idx / TPR, c8 = (idx % TPR) * 8;
        const int m = bm + half * HALF + row, n = bn + c8;
        if (idx >= HALF * TPR || m >= a.M || n >= a.Nw) continue;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = cs[row * CLD + c8 + e];
        if (vec[it]) {
          epilogue8<T>(a, b, m, n, v, in[it]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (n + e < a.Nw) epilogue_store<T>(a, b, m, n + e, v[e]);
        }
      }
    }
    lds_barrier();
  }
}

// DEPTH 1: one register set (tile t+1 is requested while tile t is multiplied); DEPTH 2: two
// sets, for long k-loops where one tile of MFMA work cannot cover a global-load round trip.
// XCD-aware renumbering (bijective for any grid size; blocks id and id + 8 share an XCD): logical
// block lid of a grid of nblk runs on XCD (lid's run), so consecutive logical blocks share one L2.
DFM_INLINE int xcd_lid(int id, int nblk) {
  const int xcd = id & 7, q8 = nblk >> 3, r8 = nblk & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
}

// One output tile (tile, zs = batch * splits + split) of the register-staged MFMA GEMM.
template <typename T, int BM, int BN, int NW, int WAVES_M, int BK, bool AK, bool BKC, int DEPTH>
DFM_INLINE void gemm_tile(const GemmArgs& a, int tile, int zs, char* smem) {
  constexpr int NT = 64 * NW;
  constexpr int WAVES_N = NW / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int KSTEP = Mf<T>::KSTEP;
  using GA = TileGeom<T, BM, BK, AK, NT>;
  using GB = TileGeom<T, BN, BK, BKC, NT>;

  T* const lds_base = reinterpret_cast<T*>(smem);
#define LDS_A(i) (lds_base + (i) * GA::ELEMS)
#define LDS_B(i) (lds_base + 2 * GA::ELEMS + (i) * GB::ELEMS)

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int tiles_m = (a.M + BM - 1) / BM;  // tiles enumerate M tiles fastest
  // n_fast: consecutive blocks walk the column tiles of one row tile, so a tall A row block (large-M
  // forward / dgrad with several column tiles) is re-read from L2 rather than from HBM
  const int bm = (a.n_fast ? tile / a.tiles_n : tile % tiles_m) * BM;
  const int bn = (a.n_fast ? tile % a.tiles_n : tile / tiles_m) * BN;
  const int b = zs / a.splits, split = zs % a.splits;

  const int kper = ((a.K + a.splits - 1) / a.splits + BK - 1) / BK * BK;
  const int kbeg = split * kper;
  const int kend = min(a.K, kbeg + kper);
  const int ones_r = a.colsum != nullptr ? a.N : -1;

  const T* A = (const T*)a.A + (long)b * a.sa;
  const T* Bp = (const T*)a.B + (long)b * a.sb;

  float4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  // tiles [0, nfull) are whole BK slices of aligned operands: branch-free loads, two register
  // sets in flight (tile t+1 lands while tile t is multiplied, tile t+2 is already requested)
  const int nfull = (a.ala && a.alb) ? (kend - kbeg) / BK : 0;
  const bool patch = ones_r >= bn && ones_r < bn + BN;  // block holds the virtual ones column

  auto compute = [&](const T* la, const T* lb) {
#pragma unroll
    for (int ks = 0; ks < BK; ks += KSTEP) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag_bf16<AK, GA::LD>((const bf16_t*)la, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag_bf16<BKC, GB::LD>((const bf16_t*)lb, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mma16<T>(fa[i], fb[j], acc[i][j]);
      } else {
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag_f32<AK, GA::LD>((const float*)la, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag_f32<BKC, GB::LD>((const float*)lb, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  unsigned offa[GA::NVEC], offb[GB::NVEC];
  if (nfull > 0) {
    fast_offsets<T, BM, BK, AK, NT>(offa, a.lda, bm, a.M);
    fast_offsets<T, BN, BK, BKC, NT>(offb, a.ldb, bn, a.N);
  }
  // buffer descriptors over the operands: 32-bit per-lane offsets, the k-slice in soffset
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)Bp, 0, 0x7fffffff, 0x00020000);
  auto load_fast = [&](uint4* xa, uint4* xb, int kt) {
    const int k0 = kbeg + kt * BK;
    stage_load_fast<T, BM, BK, AK, NT>(xa, rsa, (int)((AK ? k0 : (long)k0 * a.lda) * sizeof(T)), offa);
    stage_load_fast<T, BN, BK, BKC, NT>(xb, rsb, (int)((BKC ? k0 : (long)k0 * a.ldb) * sizeof(T)), offb);
  };
  auto store_fast = [&](uint4* xa, uint4* xb, int buf) {
    if (patch) patch_ones<T, BN, BK, BKC, NT>(xb, bn, ones_r);
    stage_store<T, BM, BK, AK, NT>(xa, LDS_A(buf));
    stage_store<T, BN, BK, BKC, NT>(xb, LDS_B(buf));
  };

  uint4 ra0[GA::NVEC], rb0[GB::NVEC];
  uint4 ra1[DEPTH > 1 ? GA::NVEC : 1], rb1[DEPTH > 1 ? GB::NVEC : 1];
  int done = 0;
  if constexpr (DEPTH == 1) {
    if (nfull >= 1) {
      load_fast(ra0, rb0, 0);
      store_fast(ra0, rb0, 0);
      lds_barrier();
      int cur = 0;
      for (int kt = 0; kt + 1 < nfull; ++kt) {
        load_fast(ra0, rb0, kt + 1);
        compute(LDS_A(cur), LDS_B(cur));
        store_fast(ra0, rb0, cur ^ 1);
        lds_barrier();
        cur ^= 1;
      }
      compute(LDS_A(cur), LDS_B(cur));
      done = nfull;
    }
  } else if (nfull == 1) {
    load_fast(ra0, rb0, 0);
    store_fast(ra0, rb0, 0);
    lds_barrier();
    compute(LDS_A(0), LDS_B(0));
    done = 1;
  } else if (nfull >= 2) {
    load_fast(ra0, rb0, 0);
    load_fast(ra1, rb1, 1);
    store_fast(ra0, rb0, 0);
    lds_barrier();
    // invariant: LDS buffer 0 holds tile kt, set 1 holds tile kt+1 (in flight). Loads past the
    // last whole tile re-read it (in-bounds, L2-hot) so every load is unconditional.
    for (int kt = 0;; kt += 2) {
      load_fast(ra0, rb0, min(kt + 2, nfull - 1));
      compute(LDS_A(0), LDS_B(0));
      store_fast(ra1, rb1, 1);
      lds_barrier();
      if (kt + 2 >= nfull) {
        compute(LDS_A(1), LDS_B(1));
        done = kt + 2;
        break;
      }
      load_fast(ra1, rb1, min(kt + 3, nfull - 1));
      compute(LDS_A(1), LDS_B(1));
      store_fast(ra0, rb0, 0);
      lds_barrier();
      if (kt + 3 >= nfull) {
        compute(LDS_A(0), LDS_B(0));
        done = kt + 3;
        break;
      }
    }
  }
  // guarded tail: the partial last slice, or every slice of unaligned operands
  for (int kt = done; kt < nk; ++kt) {
    uint4 rta[GA::NVEC], rtb[GB::NVEC];
    lds_barrier();
    const int k0 = kbeg + kt * BK;
    stage_load<T, BM, BK, AK, NT>(rta, A, a.lda, bm, k0, a.M, kend, a.ala);
    stage_load<T, BN, BK, BKC, NT>(rtb, Bp, a.ldb, bn, k0, a.N, kend, a.alb, ones_r);
    stage_store<T, BM, BK, AK, NT>(rta, LDS_A(0));
    stage_store<T, BN, BK, BKC, NT>(rtb, LDS_B(0));
    lds_barrier();
    compute(LDS_A(0), LDS_B(0));
  }
  lds_barrier();  // the epilogue reuses the operand LDS
#undef LDS_A
#undef LDS_B

  gemm_epilogue<T, BM, BN, NW, WAVES_M>(a, acc, smem, bm, bn, b, split);
}

// DEPTH 1: one register set (tile t+1 is requested while tile t is multiplied); DEPTH 2: two
// sets, for long k-loops where one tile of MFMA work cannot cover a global-load round trip.
template <typename T, int BM, int BN, int NW, int WAVES_M, int BK, bool AK, bool BKC, int DEPTH>
__global__ __launch_bounds__(64 * NW) void gemm_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int tile = blockIdx.x, zs = blockIdx.z;  // grid.x enumerates the output tiles
  if (a.xcd_map) {
    // the tiles of one split-K slice — which read the same K range of both operands — run on one
    // XCD, so the operand slices they share are re-read from that XCD's L2 instead of by all eight
    const int lid = xcd_lid(blockIdx.z * gridDim.x + blockIdx.x, gridDim.x * gridDim.z);
    tile = lid % gridDim.x;
    zs = lid / gridDim.x;
  }
  gemm_tile<T, BM, BN, NW, WAVES_M, BK, AK, BKC, DEPTH>(a, tile, zs, smem);
}

// ---------------------------------------------------------------- grouped GEMM
// Up to GMAX independent GEMMs of one tile configuration in ONE launch (the weight gradients of a
// Block's backward, which are independent of each other and of the data-gradient chain): problem q
// owns the blocks [start[q], start[q+1]) (start a multiple of 8, so the XCD renumbering inside a
// problem sees the hardware XCD of each block); its tiles x batch x splits run as in gemm_kernel.
// Sharing the chip between the problems lets each one use fewer split-K slices, and the split-K
// partials of all problems are combined by ONE grouped reduction launch.
constexpr int GMAX = 8;
struct GemmGroup {
  GemmArgs p[GMAX];
  int start[GMAX + 1];
  int n;
};

static_assert(sizeof(GemmGroup) <= 4096, "the problem table travels as a kernel argument");

DFM_INLINE int group_problem(const GemmGroup& g, int b) {
  int q = 0;
#pragma unroll
  for (int i = 1; i < GMAX; ++i)
    if (i < g.n && b >= g.start[i]) q = i;
  return q;
}

// Four waves per SIMD = two blocks per CU (at most 128 VGPRs; the second launch bound is waves per EU):
// the weight-gradient k-loops are latency-bound with one 8-wave
// block per CU, and a second resident block doubles the operand bytes in flight.
template <typename T, int BM, int BN, int NW, int WAVES_M, int BK, bool AK, bool BKC, int DEPTH>
__global__ __launch_bounds__(64 * NW, 4) void gemm_group_kernel(GemmGroup g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int q = group_problem(g, b);
  const GemmArgs& a = g.p[q];  // read in place from the kernel-argument segment (uniform scalar loads)
  const int ntile = a.tiles_m * a.tiles_n, nblk = ntile * a.batch * a.splits;
  const int local = b - g.start[q];
  if (local >= nblk) return;  // padding up to the next multiple of 8
  const int lid = xcd_lid(local, nblk);
  gemm_tile<T, BM, BN, NW, WAVES_M, BK, AK, BKC, DEPTH>(a, lid % ntile, lid / ntile, smem);
}

// Deterministic split-K combine: each block owns 256/G consecutive outputs and G lanes per output
// walk the splits in a fixed order (G = 4 when there are many splits, so short outputs x long
// split counts still fill the chip), then the G partial sums meet in LDS.
template <typename T, int G>
DFM_INLINE void splitk_reduce_block(const GemmArgs& a, long blk) {
  constexpr int PER = 256 / G;
  __shared__ float red[G][PER];
  const long total = (long)a.batch * a.M * a.ldw;  // padded workspace elements per split
  const int o = threadIdx.x % PER, g = threadIdx.x / PER;
  const long idx = blk * PER + o;
  float v = 0.f;
  if (idx < total) {  // splits g, g + G, ... in order, 8 loads in flight
    const float* p = a.ws + idx;
    int s = g;
    for (; s + 7 * G < a.splits; s += 8 * G) {
      float t[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = p[(long)(s + i * G) * total];
#pragma unroll
      for (int i = 0; i < 8; ++i) v += t[i];
    }
    if (s < a.splits) {  // the tail: every load issued before the first add (clamped index, masked
      float t[8];        // add), the same order of additions
#pragma unroll
      for (int i = 0; i < 8; ++i) t[i] = p[(long)min(s + i * G, a.splits - 1) * total];
#pragma unroll
      for (int i = 0; i < 8; ++i) v = s + i * G < a.splits ? v + t[i] : v;
    }
  }
  if (G > 1) {
    red[g][o] = v;
    __syncthreads();
    if (g != 0) return;
#pragma unroll
    for (int i = 1; i < G; ++i) v += red[i][o];
  }
  if (idx >= total) return;
  const int n = idx % a.ldw;
  if (n >= a.Nw) return;
  const long bm = idx / a.ldw;
  const int m = bm % a.M, b = bm / a.M;
  epilogue_store<T>(a, b, m, n, v);
}

template <typename T, int G>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a) {
  splitk_reduce_block<T, G>(a, blockIdx.x);
}

// grouped combine: problem q (with splits > 1) owns reduction blocks [start[q], start[q+1])
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_group_kernel(GemmGroup g) {
  const int q = group_problem(g, blockIdx.x);
  const GemmArgs& a = g.p[q];
  if (a.splits <= 1) return;
  splitk_reduce_block<T, 4>(a, blockIdx.x - g.start[q]);
}

// ---------------------------------------------------------------- LDS-DMA pipelined GEMM (bf16)
// For k-loops of >= 2 whole 64-deep slices over 16-byte aligned operands. Operand tiles go global ->
// LDS by global_load_lds_dwordx4 (no register staging, so few VGPRs and several blocks per CU)
// into an NS-deep ring of stages; each wave waits only for its own DMAs of the slice it is about
// to read with a COUNTED vmcnt (NS-2 slices stay in flight across every barrier; with NS = 2 the
// next slice's DMA overlaps this slice's MFMAs) and the raw s_barrier publishes them. LDS images are
// unpadded with XOR-swizzled 16-byte chunks (an LDS-DMA writes lane-linearly, so the swizzle is
// applied to each lane's SOURCE address): k-contiguous tiles [R][64] hold chunk c of row r at
// position c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 fragments); row-contiguous tiles [64][R]
// use tr_swz (read with ds_read_b64_tr_b16). Blocks are renumbered so consecutive logical blocks
// share an XCD (and its L2): the column tiles of one row tile (n_fast) or the tiles of one split.
constexpr int GBK = 64;

DFM_INLINE int kc_swz(int r) { return (r >> 1) & 7; }

template <int R, bool KC>
struct GImg {
  static constexpr int CHUNKS = R * GBK / 8;           // 16-byte chunks per tile
  static constexpr int BYTES = CHUNKS * 16;
  static constexpr int CPR = KC ? GBK / 8 : R / 8;     // chunks per image row
  // image position q -> (image row, chunk of the source row stored there)
  DFM_INLINE static void at(int q, int& row, int& chunk) {
    row = q / CPR;
    const int p = q % CPR;
    chunk = KC ? (p ^ kc_swz(row)) : (p ^ tr_swz<R>(row));
  }
};

DFM_INLINE bf16x8_t frag_kc_swz(const bf16_t* lds, int r0, int k0, int lane) {
  const int r = r0 + (lane & 15), c = (k0 >> 3) + (lane >> 4);
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(lds + r * GBK + ((c ^ kc_swz(r)) << 3)));
}

constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
template <int N>
DFM_INLINE void wait_vm() { __builtin_amdgcn_s_waitcnt(vmcnt_imm(N)); }
DFM_INLINE void wait_lgkm0() { __builtin_amdgcn_s_waitcnt((15) | (3 << 14) | (7 << 4) | (0 << 8)); }

// One block's work of the ring GEMM: logical block lid (XCD-renumbered) of problem a.
template <typename T, int BM, int BN, int NW, int WAVES_M, bool AK, bool BKC, int NS>
DFM_INLINE void glds_block(const GemmArgs& a, int lid, char* smem) {
  constexpr int NT = 64 * NW;
  constexpr int WAVES_N = NW / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  using IA = GImg<BM, AK>;
  using IB = GImg<BN, BKC>;
  constexpr int WIA = IA::CHUNKS / 64, WIB = IB::CHUNKS / 64;  // wave-instructions per tile
  static_assert((WIA + WIB) % NW == 0, "every wave must issue the same number of DMAs per slice");
  constexpr int J = (WIA + WIB) / NW;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  static_assert(NS >= 2, "ring too shallow");
  (void)NT;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int tiles = a.tiles_m * a.tiles_n;
  const int tile = lid % tiles, zs = lid / tiles;
  const int bm = (a.n_fast ? tile / a.tiles_n : tile % a.tiles_m) * BM;
  const int bn = (a.n_fast ? tile % a.tiles_n : tile / a.tiles_m) * BN;
  const int b = zs / a.splits, split = zs % a.splits;

  const int kper = ((a.K + a.splits - 1) / a.splits + GBK - 1) / GBK * GBK;
  const int kbeg = split * kper;
  const int kend = min(a.K, kbeg + kper);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;
  const int nfull = (kend - kbeg) / GBK;  // >= 2 whenever the host picks this kernel, except short splits
  const int ones_r = a.colsum != nullptr ? a.N : -1;

  const T* A = (const T*)a.A + (long)b * a.sa;
  const T* Bp = (const T*)a.B + (long)b * a.sb;

  // per DMA j of this lane: source of slice 0, per-slice step (elements), LDS offset in a stage,
  // and (virtual ones column) the element of the chunk to overwrite with 1.0 after it lands
  const T* src[J];
  long step[J];
  int dst[J], ones_e[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int g = j * NW + wid;  // wave-uniform
    const bool isA = g < WIA;
    const int gq = (isA ? g : g - WIA) * 64 + lane;
    int row, chunk;
    ones_e[j] = -1;
    if (isA) {
      IA::at(gq, row, chunk);
      if (AK) {
        const int r = min(bm + row, a.M - 1);
        src[j] = A + (long)r * a.lda + kbeg + chunk * 8;
        step[j] = GBK;
      } else {
        const int c = bm + chunk * 8;
        src[j] = A + (long)(kbeg + row) * a.lda + (c < a.M ? c : 0);
        step[j] = (long)GBK * a.lda;
      }
      dst[j] = g * 1024;
    } else {
      if (BKC) {
        IB::at(gq, row, chunk);
        const int r = min(bn + row, a.N - 1);
        src[j] = Bp + (long)r * a.ldb + kbeg + chunk * 8;
        step[j] = GBK;
      } else {
        IB::at(gq, row, chunk);
        const int c = bn + chunk * 8;
        src[j] = Bp + (long)(kbeg + row) * a.ldb + (c < a.N ? c : 0);
        step[j] = (long)GBK * a.ldb;
        if (ones_r >= c && ones_r < c + 8) ones_e[j] = ones_r - c;
      }
      dst[j] = IA::BYTES + (g - WIA) * 1024;
    }
  }
  const bool patch = ones_r >= bn && ones_r < bn + BN;  // block-uniform

#ifndef DFM_RING_ASM_DMA
#define DFM_RING_ASM_DMA 1
#endif
#if DFM_RING_ASM_DMA
  // The DMA as inline asm (measured 471.5 / 472.9 vs 470.1 / 470.9 images/s): the compiler no longer
  // sees an LDS write in flight, so it stops draining the ring (s_waitcnt vmcnt(0)) before the
  // transposing fragment reads; ordering comes from the counted waits, the barrier and the compiler
  // fences below. m0 is written here only (the ring kernels have no other m0 user, checked in their ISA).
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const T* gp = src[j] + t * step[j];
      const unsigned l = __builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(smem + stage * STAGE + dst[j]));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(l), "v"(gp) : "memory", "m0");
#pragma clang diagnostic pop
    }
  };
#define DFM_CFENCE() asm volatile("" ::: "memory")
#else
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int j = 0; j < J; ++j)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src[j] + t * step[j]),
                                       (void __attribute__((address_space(3)))*)(smem + stage * STAGE + dst[j]),
                                       16, 0, 0);
  };
#define DFM_CFENCE() ((void)0)
#endif
  auto patch_ones = [&](int stage) {  // after this wave's DMAs of the stage landed
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (ones_e[j] >= 0)
        reinterpret_cast<unsigned short*>(smem + stage * STAGE + dst[j] + lane * 16)[ones_e[j]] = (unsigned short)one16<T>();
  };

  float4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  auto read_frags = [&](int stage, bf16x8_t (&fa)[2][TM], bf16x8_t (&fb)[2][TN]) {
    const bf16_t* la = reinterpret_cast<const bf16_t*>(smem + stage * STAGE);
    const bf16_t* lb = reinterpret_cast<const bf16_t*>(smem + stage * STAGE + IA::BYTES);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[h][i] = AK ? frag_kc_swz(la, wm * WM + i * 16, 32 * h, lane)
                      : frag_bf16<false, BM>(la, wm * WM + i * 16, 32 * h, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[h][j] = BKC ? frag_kc_swz(lb, wn * WN + j * 16, 32 * h, lane)
                       : frag_bf16<false, BN>(lb, wn * WN + j * 16, 32 * h, lane);
    }
  };
  auto mma = [&](const bf16x8_t (&fa)[2][TM], const bf16x8_t (&fb)[2][TN], int h) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mma16<T>(fa[h][i], fb[h][j], acc[i][j]);
  };
  auto compute = [&](int stage) {
    bf16x8_t fa[2][TM], fb[2][TN];
    read_frags(stage, fa, fb);
    mma(fa, fb, 0);
    mma(fa, fb, 1);
  };

  // Software pipeline across the barrier. Iteration u enters with slice u's fragments in
  // registers; k-step 0 MFMAs -> wait for slice u+1's DMAs -> barrier (slice u+1 visible, stage
  // u % NS free) -> DMA slice u+NS into it -> read slice u+1's fragments -> k-step 1 MFMAs, so
  // the LDS reads of the next slice overlap this slice's MFMAs instead of every wave reading,
  // then every wave multiplying, in lockstep.
  {
    // ring: wait for slice t (NS-2 slices stay in flight) -> barrier -> DMA slice t+NS-1 into the
    // stage read last iteration -> multiply slice t. Measured on the step's GEMM census: a 2-stage
    // ring at 3-4 blocks per CU (blocks overlap each other's barrier/LDS phases) beats a 4-stage
    // ring at 1 block per CU, with or without fragment reads pipelined across the barrier.
#pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (t < nfull) issue(t, t);
    for (int t = 0; t < nfull; ++t) {
      const int stage = t % NS;
      const int rem = nfull - 1 - t;
      if (NS > 2 && rem >= NS - 2) wait_vm<J * (NS > 2 ? NS - 2 : 0)>();
      else if (NS > 3 && rem == 1) wait_vm<J>();
      else wait_vm<0>();
      DFM_CFENCE();
      if (patch) patch_ones(stage);
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      DFM_CFENCE();
      if (t + NS - 1 < nfull) issue(t + NS - 1, (t + NS - 1) % NS);
      compute(stage);
    }
  }
  wait_vm<0>();
  DFM_CFENCE();
  __syncthreads();
#undef DFM_CFENCE
  // guarded tail: the partial last slice (zero fill past kend), staged through registers into stage 0
  for (int kt = nfull; kt < nk; ++kt) {
    const int k0 = kbeg + kt * GBK;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int g = j * NW + wid;
      const bool isA = g < WIA;
      const int gq = (isA ? g : g - WIA) * 64 + lane;
      int row, chunk;
      uint4 v;
      if (isA) {
        IA::at(gq, row, chunk);
        v = AK ? load_vec<T, true>(A, a.lda, bm + row, k0 + chunk * 8, a.M, kend, true, -1)
               : load_vec<T, false>(A, a.lda, bm + chunk * 8, k0 + row, a.M, kend, true, -1);
      } else {
        IB::at(gq, row, chunk);
        v = BKC ? load_vec<T, true>(Bp, a.ldb, bn + row, k0 + chunk * 8, a.N, kend, true, ones_r)
                : load_vec<T, false>(Bp, a.ldb, bn + chunk * 8, k0 + row, a.N, kend, true, ones_r);
      }
      *reinterpret_cast<uint4*>(smem + dst[j] + lane * 16) = v;
    }
    __syncthreads();
    compute(0);
    __syncthreads();
  }
  gemm_epilogue<T, BM, BN, NW, WAVES_M>(a, acc, smem, bm, bn, b, split);
}

template <typename T, int BM, int BN, int NW, int WAVES_M, bool AK, bool BKC, int NS, int MINB>
__global__ __launch_bounds__(64 * NW, MINB) void gemm_glds_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // XCD-aware renumbering (bijective for any grid size): blocks id and id + 8 share an XCD
  glds_block<T, BM, BN, NW, WAVES_M, AK, BKC, NS>(a, xcd_lid(blockIdx.x, gridDim.x), smem);
}

// Up to GMAX independent ring GEMMs (k-contiguous A: forwards and input gradients of one Block phase,
// e.g. q | q_cut | l with e_fore) in ONE launch: problem q owns blocks [start[q], start[q+1]) as in
// gemm_group_kernel, so the short k-loops of the stage-2 / 3 shapes share one ramp and one tail.
template <typename T, int BM, int BN, int NW, int WAVES_M, bool AK, bool BKC, int NS, int MINB>
__global__ __launch_bounds__(64 * NW, MINB) void gemm_glds_group_kernel(GemmGroup g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int q = group_problem(g, blockIdx.x);
  const GemmArgs& a = g.p[q];
  const int nblk = a.tiles_m * a.tiles_n * a.batch * a.splits;
  const int local = blockIdx.x - g.start[q];
  if (local >= nblk) return;  // padding up to the next multiple of 8
  glds_block<T, BM, BN, NW, WAVES_M, AK, BKC, NS>(a, xcd_lid(local, nblk), smem);
}

template <typename T, int BM, int BN, int NW, int WM_, bool AK, bool BKC, int NS, int MINB>
int launch_glds(GemmArgs& a, hipStream_t s) {
  using IA = GImg<BM, AK>;
  using IB = GImg<BN, BKC>;
  constexpr int RP = (128 * NW / (BN / 8)) < BM ? (128 * NW / (BN / 8)) : BM;
  const size_t lds = std::max((size_t)NS * (IA::BYTES + IB::BYTES), (size_t)RP * (BN + 4) * sizeof(float));
  auto kern = gemm_glds_kernel<T, BM, BN, NW, WM_, AK, BKC, NS, MINB>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  a.tiles_m = cdiv(a.M, BM);
  a.tiles_n = cdiv(a.Nw, BN);
  a.n_fast = a.M >= a.N;
  const long grid = (long)a.tiles_m * a.tiles_n * a.batch * a.splits;
  DFM_LAUNCH(kern, dim3((unsigned)grid), dim3(64 * NW), lds, s, a);
  DFM_LAUNCH_CHECK();
  if (a.splits > 1) {
    const long total = (long)a.batch * a.M * a.ldw;
    if (a.splits >= 8)
      DFM_LAUNCH((splitk_reduce_kernel<T, 4>), dim3(cdiv(total, 64)), dim3(256), 0, s, a);
    else
      DFM_LAUNCH((splitk_reduce_kernel<T, 1>), dim3(cdiv(total, 256)), dim3(256), 0, s, a);
    DFM_LAUNCH_CHECK();
  }
  return DFM_OK;
}

template <typename T, int BM, int BN, int NW, int WM_, int NS, int MINB>
int glds_ak(GemmArgs& a, bool bk, hipStream_t s) {
  if (bk) return launch_glds<T, BM, BN, NW, WM_, true, true, NS, MINB>(a, s);
  return launch_glds<T, BM, BN, NW, WM_, true, false, NS, MINB>(a, s);
}

template <typename T, int BM, int BN, int NW, int WM_, int BK, bool AK, bool BKC, int DEPTH>
int launch_cfg(GemmArgs& a, hipStream_t s) {
  using GA = TileGeom<T, BM, BK, AK, 64 * NW>;
  using GB = TileGeom<T, BN, BK, BKC, 64 * NW>;
  const size_t lds_op = (size_t)2 * (GA::ELEMS + GB::ELEMS) * sizeof(T);
  constexpr int RP = (128 * NW / (BN / 8)) < BM ? (128 * NW / (BN / 8)) : BM;  // epilogue rows per pass
  const size_t lds_c = (size_t)RP * (BN + 4) * sizeof(float);
  const size_t lds = lds_op > lds_c ? lds_op : lds_c;
  a.tiles_n = cdiv(a.Nw, BN);
  a.n_fast = a.tiles_n > 1 && a.M >= a.Nw;
  dim3 grid(cdiv(a.M, BM) * a.tiles_n, 1, a.batch * a.splits);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<T, BM, BN, NW, WM_, BK, AK, BKC, DEPTH>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  DFM_LAUNCH((gemm_kernel<T, BM, BN, NW, WM_, BK, AK, BKC, DEPTH>), grid, dim3(64 * NW), lds, s, a);
  DFM_LAUNCH_CHECK();
  if (a.splits > 1) {
    const long total = (long)a.batch * a.M * a.ldw;
    if (a.splits >= 8)
      DFM_LAUNCH((splitk_reduce_kernel<T, 4>), dim3(cdiv(total, 64)), dim3(256), 0, s, a);
    else
      DFM_LAUNCH((splitk_reduce_kernel<T, 1>), dim3(cdiv(total, 256)), dim3(256), 0, s, a);
    DFM_LAUNCH_CHECK();
  }
  return DFM_OK;
}

template <typename T, int BM, int BN, int NW, int WM_, int BK, int DEPTH>
int launch_layout(GemmArgs& a, bool ak, bool bk, hipStream_t s) {
  if (ak && bk) return launch_cfg<T, BM, BN, NW, WM_, BK, true, true, DEPTH>(a, s);
  if (ak && !bk) return launch_cfg<T, BM, BN, NW, WM_, BK, true, false, DEPTH>(a, s);
  if (!ak && bk) return launch_cfg<T, BM, BN, NW, WM_, BK, false, true, DEPTH>(a, s);
  return launch_cfg<T, BM, BN, NW, WM_, BK, false, false, DEPTH>(a, s);
}

template <typename T, int BM, int BN, int NW, int WM_, int BK>
int launch_depth(GemmArgs& a, bool ak, bool bk, hipStream_t s) {
  const int kper = (a.K + a.splits - 1) / a.splits;
  const long blocks = (long)cdiv(a.M, BM) * cdiv(a.Nw, BN) * a.batch * a.splits;
  // two register sets cost occupancy: only worth it for long k-loops on a grid that leaves CUs
  // with a single block anyway
  if (kper >= 8 * BK && blocks <= 512) return launch_layout<T, BM, BN, NW, WM_, BK, 2>(a, ak, bk, s);
  return launch_layout<T, BM, BN, NW, WM_, BK, 1>(a, ak, bk, s);
}

void pick_tile(const DfmGemmDesc* d, int& BM, int& BN) {
  const int Nw = d->N + (d->colsum ? 1 : 0);
  BM = 128;
  BN = Nw <= 32 ? 32 : (Nw <= 64 ? 64 : 128);
}

// Split-K: enough blocks to put one long-K block on every CU (~256), but at least 512 reduction
// elements per split, rounded down to a power of two (fitted on the DFormer-B step's GEMM census,
// tools/gemm_sweep.py).
int choose_splits(const DfmGemmDesc* d, int elem_bytes) {
  if (d->split_k >= 1) return d->split_k;
  int BM, BN;
  pick_tile(d, BM, BN);
  const int Nw = d->N + (d->colsum ? 1 : 0);
  const long tiles = (long)cdiv(d->M, BM) * cdiv(Nw, BN) * (d->batch > 0 ? d->batch : 1);
  if (elem_bytes == 4 && d->batch > 1 && tiles < 64 && d->K >= 256) {
    // batched fp32 products with one tile per batch over a long K (the NMF's R x R Gram products,
    // ham_head.py:88-109): ~512 blocks of >= 128 reduction elements instead of one serial k-loop
    // per batch (one 64 x 64 x 512 tile took 28 us)
    long s = std::min((512 + tiles - 1) / tiles, (long)d->K / 128);
    int p = 1;
    while (2L * p <= s && p < 1024) p *= 2;
    return p;
  }
  if (d->K < 1024 || tiles >= 256) return 1;
  // (~256 blocks: 475.9-476.7 images/s vs 469.4-469.7 at 128 and 473.4-473.8 at 512)
  long s = std::min((256 + tiles - 1) / tiles, (long)d->K / 512);
  int p = 1;
  while (2L * p <= s && p < 1024) p *= 2;
  return p;
}

#include "gemm_wide.h"

template <typename T>
bool al16(const void* p, long ld) {
  return p == nullptr || (((uintptr_t)p % 16 == 0) && (ld % 8 == 0));
}

template <typename T>
int gemm_typed(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s) {
  constexpr int VEC = Mf<T>::VEC;
  GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.ws = (float*)ws;
  a.M = d->M; a.N = d->N; a.K = d->K; a.batch = d->batch > 0 ? d->batch : 1;
  a.Nw = d->N + (d->colsum ? 1 : 0);
  a.ldw = (a.Nw + 7) & ~7;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c;
  a.alpha = d->alpha; a.beta = d->beta; a.c_f32 = d->c_f32;
  a.bias = d->bias; a.act = d->act; a.preact = d->preact; a.ldpre = d->ldpre;
  a.mul = d->mul; a.ldmul = d->ldmul; a.res = d->res; a.ldres = d->ldres; a.mul_gelu_grad = d->mul_gelu_grad;
  a.colscale = d->colscale; a.rowscale = d->rowscale; a.act_col0 = d->act_col0;
  a.rps = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  a.colsum = d->colsum; a.colsum_acc = d->colsum_accumulate;
  a.mul2 = d->mul2; a.ldmul2 = d->ldmul2; a.C2 = d->out2; a.ldc2 = d->ldout2;
  a.xcd_map = 1;
  int BM, BN;
  pick_tile(d, BM, BN);
  a.splits = choose_splits(d, sizeof(T));
  if (a.splits > 1) DFM_CHECK_ARG(ws != nullptr, "dfm_gemm: split-K needs a workspace");
  // fast (buffer-load) tiles need 16-byte aligned rows and one matrix within a 2 GiB descriptor
  const double ext_a = ((double)(d->a_kcontig ? d->M : d->K) * d->lda) * sizeof(T);
  const double ext_b = ((double)(d->b_kcontig ? d->N : d->K) * d->ldb) * sizeof(T);
  a.ala = (d->lda % VEC == 0) && ((uintptr_t)A % 16 == 0) && (a.batch == 1 || d->stride_a % VEC == 0) &&
          ext_a < 2147483647.0;
  a.alb = (d->ldb % VEC == 0) && ((uintptr_t)B % 16 == 0) && (a.batch == 1 || d->stride_b % VEC == 0) &&
          ext_b < 2147483647.0;
  a.vec_ok = al16<T>(C, d->ldc) && (a.batch == 1 || d->stride_c % 8 == 0) && al16<T>(d->preact, d->ldpre) &&
             al16<T>(d->mul, d->ldmul) && al16<T>(d->res, d->ldres) && (d->act_col0 % 8 == 0) &&
             al16<T>(d->mul2, d->ldmul2) && al16<T>(d->out2, d->ldout2);
  const bool ak = d->a_kcontig, bk = d->b_kcontig;
  const bool small_k = sizeof(T) == 2 ? d->K <= 128 : d->K <= 64;
  // (a persistent M-streaming kernel for large M x short K, column tiles <= 64, was measured slower
  // on the step than one tile per block: 452.7-454.0 vs 455.2 images/s — its static tile walk
  // finishes late when the concurrent ConvFFN stream holds CUs)
  // bf16 k-contiguous A on the LDS-DMA ring: split-K off (one unsplit 64x64 ring block per tile beats
  // the split + reduction at 4,800 rows x K >= 1024: 16.8 vs 34.8 us, profiles/r04_glds_variants.txt)
  // (the ring kernel writes the virtual ones column of a bias-gradient colsum for a row-contiguous B
  // only; a k-contiguous B with colsum takes the register-staged kernel)
  bool glds_ok = sizeof(T) == 2 && ak && a.ala && a.alb && !(d->colsum && bk);
  if (glds_ok && d->split_k < 1) a.splits = 1;
  glds_ok = glds_ok && (d->K + a.splits - 1) / a.splits >= 2 * GBK;  // >= 2 whole k-slices per split
  // tall short-K GEMMs with more than one 128-column slice (gemm_wide.h): measured per shape on the
  // DFormer-B step's census (profiles/r04_wide_gemm_ab.txt) it wins from 65,536 rows and N >= 144
  // (stage-0 fc1 104 vs 138 us, stage-1 fc2 input gradient x GELU' 106 vs 124 us) and loses on
  // narrower outputs (a 128-column slice half empty) and on the 19,200-row stage-2 shapes
  if constexpr (sizeof(T) == 2) {
    if (wide_eligible<T>(a, d)) return wide_launch<T>(a, d, s);
  }
  // LDS-DMA ring kernel: bf16 with a k-contiguous A (forward, dgrad) and >= 2 whole k-slices. Routing
  // fitted on the DFormer-B step's GEMM census (tools/gemm_sweep.py --replay): it wins on the forward
  // except wide-N x short-K, and on input gradients from K = 128 up (64x64 tiles: 418.5-419.4
  // images/s vs 415.4-416.0 from K = 640); with a row-contiguous A (weight gradients) the
  // register-staged kernel stays ahead (a 3/4-stage ring there measured 386.3 vs 408 images/s).
  // 64x64 tiles for every width: the stage-1..3 shapes are latency-bound and gain from twice the
  // blocks more than they lose in B-tile reuse (421.5 vs 418.1-418.5 images/s with 64x128). Bigger
  // tiles chosen per shape (128x128 from 65,536 rows, 128x64 / 64x128 elsewhere: 1 ms less GEMM time
  // per step replayed in isolation, tools/gemm_variants.py) measured flat on the step (37.45-37.59
  // ms/step either way, profiles/r04_glds_variants.txt).
  if constexpr (sizeof(T) == 2) {  // the LDS-DMA ring kernel: bf16 and fp16
    // (wide-N x K = 256 forward GEMMs, the stage-2 fc1, on the ring too: 477.2 -> 480.7 images/s)
    const bool route = ak && (bk ? !(a.Nw > 512 && d->K <= 128) : d->K >= 128);
    if (glds_ok && route) {
      if (BN == 32) return glds_ak<T, 128, 32, 4, 4, 2, 3>(a, bk, s);
      // the decoder's 1x1 convs (76,800 rows x 512-896 x 512-896): 128 x 128 tiles, 8 waves
      // (438.7-438.4 -> 439.0-440.3 images/s on one box; 65-93 vs 81-127 us per launch alone)
      if (a.splits == 1 && d->M >= 65536 && a.Nw >= 512 && d->K >= 512) return glds_ak<T, 128, 128, 8, 2, 2, 2>(a, bk, s);
      return glds_ak<T, 64, 64, 4, 2, 2, 4>(a, bk, s);
    }
  }
  if (small_k) {
    constexpr int BKs = sizeof(T) == 2 ? 32 : 16;
    if (BN == 32) return launch_layout<T, 128, 32, 4, 4, BKs, 1>(a, ak, bk, s);
    if (BN == 64) return launch_layout<T, 128, 64, 4, 2, BKs, 1>(a, ak, bk, s);
    return launch_layout<T, 128, 128, 8, 2, BKs, 1>(a, ak, bk, s);
  }
  constexpr int BKl = sizeof(T) == 2 ? 64 : 32;
  if (BN == 32) return launch_depth<T, 128, 32, 4, 4, BKl>(a, ak, bk, s);
  if (BN == 64) return launch_depth<T, 128, 64, 4, 2, BKl>(a, ak, bk, s);
  return launch_depth<T, 128, 128, 8, 2, BKl>(a, ak, bk, s);
}

// ---- grouped launch (host)
// The group's split-K choice: every problem gets split-K slices in proportion to its share of the
// group's work (tiles x K), so the ~512 blocks of the launch each reduce about the same K range (at
// least 512 elements); d->split_k >= 1 forces a problem's count.
void group_splits(int n, const DfmGemmDesc* d, int* splits) {
  // ~512 blocks (one round at two blocks per CU): measured on the step 481.5 / 482.2 images/s vs
  // 472.7 / 473.4 at 1,024 (half the fp32 split-K partials written and re-read by the combine),
  // 480.5 / 480.8 at 384, 478.5 / 479.2 at 256, 447 at 128, 467 at 2,048; the 512-element minimum
  // per block measured flat against 256 / 1,024
  constexpr double target = 512.0;
  double work = 0;
  for (int q = 0; q < n; ++q) {
    const int Nw = d[q].N + (d[q].colsum ? 1 : 0);
    work += (double)cdiv(d[q].M, 128) * cdiv(Nw, 128) * (d[q].batch > 0 ? d[q].batch : 1) * d[q].K;
  }
  const double per_blk = std::max(512.0, work / target);
  for (int q = 0; q < n; ++q) {
    if (d[q].split_k >= 1) {
      splits[q] = d[q].split_k;
      continue;
    }
    const double want = d[q].K / per_blk;
    int p2 = 1;
    while (2.0 * p2 <= want && p2 < 256) p2 *= 2;
    splits[q] = p2;
  }
}

size_t group_ws_bytes(const DfmGemmDesc* d, int splits) {
  if (splits <= 1) return 0;
  const long ldw = (d->N + (d->colsum ? 1 : 0) + 7) & ~7L;
  return (size_t)splits * (d->batch > 0 ? d->batch : 1) * d->M * ldw * sizeof(float);
}

template <typename T>
void fill_args(GemmArgs& a, const DfmGemmDesc* d, const void* A, const void* B, void* C, float* ws, int splits) {
  constexpr int VEC = Mf<T>::VEC;
  a = GemmArgs{};
  a.A = A; a.B = B; a.C = C; a.ws = ws;
  a.M = d->M; a.N = d->N; a.K = d->K; a.batch = d->batch > 0 ? d->batch : 1;
  a.Nw = d->N + (d->colsum ? 1 : 0);
  a.ldw = (a.Nw + 7) & ~7;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c;
  a.alpha = d->alpha; a.beta = d->beta; a.c_f32 = d->c_f32;
  a.bias = d->bias; a.act = d->act; a.preact = d->preact; a.ldpre = d->ldpre;
  a.mul = d->mul; a.ldmul = d->ldmul; a.res = d->res; a.ldres = d->ldres; a.mul_gelu_grad = d->mul_gelu_grad;
  a.colscale = d->colscale; a.rowscale = d->rowscale; a.act_col0 = d->act_col0;
  a.rps = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  a.colsum = d->colsum; a.colsum_acc = d->colsum_accumulate;
  a.mul2 = d->mul2; a.ldmul2 = d->ldmul2; a.C2 = d->out2; a.ldc2 = d->ldout2;
  a.splits = splits;
  const double ext_a = ((double)(d->a_kcontig ? d->M : d->K) * d->lda) * sizeof(T);
  const double ext_b = ((double)(d->b_kcontig ? d->N : d->K) * d->ldb) * sizeof(T);
  a.ala = (d->lda % VEC == 0) && ((uintptr_t)A % 16 == 0) && (a.batch == 1 || d->stride_a % VEC == 0) &&
          ext_a < 2147483647.0;
  a.alb = (d->ldb % VEC == 0) && ((uintptr_t)B % 16 == 0) && (a.batch == 1 || d->stride_b % VEC == 0) &&
          ext_b < 2147483647.0;
  a.vec_ok = al16<T>(C, d->ldc) && (a.batch == 1 || d->stride_c % 8 == 0) && al16<T>(d->preact, d->ldpre) &&
             al16<T>(d->mul, d->ldmul) && al16<T>(d->res, d->ldres) && (d->act_col0 % 8 == 0) &&
             al16<T>(d->mul2, d->ldmul2) && al16<T>(d->out2, d->ldout2);
}

template <typename T, bool AK, bool BKC>
int group_launch(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C, char* ws,
                 hipStream_t s) {
  constexpr int BM = 128, BN = 128, NW = 8, WM_ = 2, BK = sizeof(T) == 2 ? 64 : 32, DEPTH = 2;
  using GA = TileGeom<T, BM, BK, AK, 64 * NW>;
  using GB = TileGeom<T, BN, BK, BKC, 64 * NW>;
  const size_t lds_op = (size_t)2 * (GA::ELEMS + GB::ELEMS) * sizeof(T);
  constexpr int RP = (128 * NW / (BN / 8)) < BM ? (128 * NW / (BN / 8)) : BM;
  const size_t lds = std::max(lds_op, (size_t)RP * (BN + 4) * sizeof(float));
  auto kern = gemm_group_kernel<T, BM, BN, NW, WM_, BK, AK, BKC, DEPTH>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  int splits[GMAX];
  group_splits(n, d, splits);
  GemmGroup g;
  GemmGroup r;  // the same problems with the reduction's block ranges
  g.n = r.n = n;
  g.start[0] = r.start[0] = 0;
  size_t off = 0;
  bool any_split = false;
  for (int q = 0; q < n; ++q) {
    fill_args<T>(g.p[q], &d[q], A[q], B[q], C[q], splits[q] > 1 ? (float*)(ws + off) : nullptr, splits[q]);
    off += group_ws_bytes(&d[q], splits[q]);
    g.p[q].xcd_map = 1;
    g.p[q].tiles_m = cdiv(d[q].M, BM);
    g.p[q].tiles_n = cdiv(g.p[q].Nw, BN);
    // forward / input-gradient problems (k-contiguous A, tall): the column tiles of one row tile run
    // back to back so the A row block is re-read from L2 (as launch_cfg); weight gradients keep row order
    g.p[q].n_fast = AK && g.p[q].tiles_n > 1 && d[q].M >= g.p[q].Nw;
    const int nblk = g.p[q].tiles_m * g.p[q].tiles_n * g.p[q].batch * splits[q];
    g.start[q + 1] = g.start[q] + (nblk + 7) / 8 * 8;
    r.p[q] = g.p[q];
    const long total = (long)g.p[q].batch * g.p[q].M * g.p[q].ldw;
    r.start[q + 1] = r.start[q] + (splits[q] > 1 ? (int)cdiv(total, 64) : 0);
    any_split = any_split || splits[q] > 1;
  }
  DFM_LAUNCH(kern, dim3((unsigned)g.start[n]), dim3(64 * NW), lds, s, g);
  DFM_LAUNCH_CHECK();
  if (any_split) {
    DFM_LAUNCH(splitk_reduce_group_kernel<T>, dim3((unsigned)r.start[n]), dim3(256), 0, s, r);
    DFM_LAUNCH_CHECK();
  }
  return DFM_OK;
}

// k-contiguous-A problems whose operands suit the ring kernel (16-byte aligned, >= 2 whole k-slices)
// go to gemm_glds_group_kernel, unsplit, in 64 x 64 tiles (the single-GEMM route's tile for these shapes)
template <typename T, bool BKC>
int group_launch_glds(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                      hipStream_t s) {
  constexpr int BM = 64, BN = 64, NW = 4, WM_ = 2, NS = 2, MINB = 4;  // (3 stages at 3 blocks per CU: no gain)
  using IA = GImg<BM, true>;
  using IB = GImg<BN, BKC>;
  constexpr int RP = (128 * NW / (BN / 8)) < BM ? (128 * NW / (BN / 8)) : BM;
  const size_t lds = std::max((size_t)NS * (IA::BYTES + IB::BYTES), (size_t)RP * (BN + 4) * sizeof(float));
  auto kern = gemm_glds_group_kernel<T, BM, BN, NW, WM_, true, BKC, NS, MINB>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  GemmGroup g;
  g.n = n;
  g.start[0] = 0;
  for (int q = 0; q < n; ++q) {
    fill_args<T>(g.p[q], &d[q], A[q], B[q], C[q], nullptr, 1);
    g.p[q].tiles_m = cdiv(d[q].M, BM);
    g.p[q].tiles_n = cdiv(g.p[q].Nw, BN);
    g.p[q].n_fast = d[q].M >= d[q].N;
    const int nblk = g.p[q].tiles_m * g.p[q].tiles_n * g.p[q].batch;
    g.start[q + 1] = g.start[q] + (nblk + 7) / 8 * 8;
  }
  DFM_LAUNCH(kern, dim3((unsigned)g.start[n]), dim3(64 * NW), lds, s, g);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T>
bool glds_group_member(const DfmGemmDesc* d, const void* A, const void* B) {
  if (sizeof(T) != 2 || !d->a_kcontig) return false;
  GemmArgs a;
  fill_args<T>(a, d, A, B, nullptr, nullptr, 1);
  return a.ala && a.alb && d->K >= 2 * GBK && d->split_k <= 1 && !d->colsum;
}

template <typename T>
int gemm_group_typed(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                     void* ws, hipStream_t s) {
  const bool ak = d[0].a_kcontig, bk = d[0].b_kcontig;
  if (ak) {
    // forwards / input gradients: the ring-kernel members as one grouped launch, the rest (short K,
    // unaligned operands, fp32) one by one on their own single-GEMM route (sharing the workspace)
    DfmGemmDesc gd[GMAX];
    const void *ga[GMAX], *gb[GMAX];
    void* gc[GMAX];
    int m = 0;
    for (int q = 0; q < n; ++q) {
      if (glds_group_member<T>(&d[q], A[q], B[q])) {
        gd[m] = d[q];
        ga[m] = A[q], gb[m] = B[q], gc[m] = C[q];
        ++m;
        continue;
      }
      DfmGemmDesc one = d[q];
      one.workspace_bytes = d[0].workspace_bytes;
      if (int st = gemm_typed<T>(&one, A[q], B[q], C[q], ws, s)) return st;
    }
    if constexpr (sizeof(T) == 2) {
      if (m == 1) return gemm_typed<T>(&gd[0], ga[0], gb[0], gc[0], ws, s);
      if (m > 1) return bk ? group_launch_glds<T, true>(m, gd, ga, gb, gc, s) : group_launch_glds<T, false>(m, gd, ga, gb, gc, s);
    }
    return DFM_OK;
  }
  // (weight gradients on the ring kernel in 128 x 128 tiles measured 472.3 / 472.5 vs 472.8 / 473.0
  // images/s: the register-staged kernel stays)
  if (ak && bk) return group_launch<T, true, true>(n, d, A, B, C, (char*)ws, s);
  if (ak) return group_launch<T, true, false>(n, d, A, B, C, (char*)ws, s);
  if (bk) return group_launch<T, false, true>(n, d, A, B, C, (char*)ws, s);
  return group_launch<T, false, false>(n, d, A, B, C, (char*)ws, s);
}

// per-dtype instantiations live in gemm_bf16.hip / gemm_f16.hip / gemm_f32.hip (one translation unit
// each, so the three dtype sets of tile templates compile in parallel)
}  // namespace

int dfm_gemm_bf16(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s);
int dfm_gemm_f16(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s);
int dfm_gemm_f32(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s);
int dfm_gemm_group_bf16(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                        void* ws, hipStream_t s);
int dfm_gemm_group_f16(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                       void* ws, hipStream_t s);
int dfm_gemm_group_f32(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                       void* ws, hipStream_t s);
