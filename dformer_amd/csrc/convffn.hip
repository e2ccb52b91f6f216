// Fused ConvFFN for gfx950 — DFormer's MLP (models/encoders/DFormer.py:48-67) inside the Block
// residual (DFormer.py:173-179):
//
//   out = x + rowscale * ls * (fc2(GELU(DW3x3(h) + bpos + h)) + b2),   h = fc1(xn) + b1
//
// One workgroup owns a TH x TW tile of output pixels of one image. The tile's xn rows plus their
// 1-pixel halo are staged in LDS once; the workgroup then walks the hidden channels in chunks of
// HC: the chunk's W1 rows / W2 columns are staged in LDS, fc1 runs on tile + halo (MFMA,
// h^T = W1c xn^T, so each lane holds 4 consecutive channels of one pixel) -> LDS; depthwise 3x3 +
// bias + identity + GELU on 8-channel vectors from LDS (zero padding = zero rows for halo pixels
// outside the image) -> LDS; fc2 of the chunk (MFMA, out^T += W2c g^T) accumulates in registers
// over all chunks. The [P, r*C] hidden activation never leaves the CU: HBM sees xn and x read
// once (+ the halo rows of neighbouring tiles, L2) and out / f written once.
//
// Backward (convffn_bwd_kernel, below) recomputes h / hpre per tile from xn.
#include <algorithm>

#include "common.h"

namespace {

constexpr int NTH = 256;  // threads per workgroup (4 waves)

// ---- MFMA fragment helpers, both operands "k-contiguous per row": lane l holds
// A[row l&15][k0 + KL*(l>>4) .. +KL] and B[k0 + KL*(l>>4) .. +KL][col l&15]; C/D: col = l&15,
// rows 4*(l>>4) .. +4 (dtype-independent on gfx950).
template <typename T> struct MM;
template <> struct MM<bf16_t> {
  static constexpr int KS = 32, KL = 8;
  using frag = bf16x8_t;
  static DFM_INLINE frag zero() { return __builtin_bit_cast(frag, make_uint4(0, 0, 0, 0)); }
  static DFM_INLINE frag load(const bf16_t* p) { return __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(p)); }
  static DFM_INLINE float4_t mma(float4_t c, frag a, frag b) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MM<float> {
  static constexpr int KS = 4, KL = 1;
  using frag = float;
  static DFM_INLINE frag zero() { return 0.f; }
  static DFM_INLINE frag load(const float* p) { return *p; }
  static DFM_INLINE float4_t mma(float4_t c, frag a, frag b) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
};

// 4 consecutive values -> LDS (8 bytes bf16 / 16 bytes f32)
DFM_INLINE void st4(bf16_t* p, const float* v) {
  const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}
DFM_INLINE void st4(float* p, const float* v) { *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]); }

struct FfnArgs {
  int B, H, W, C, hid;
  int tiles_y, tiles_x;
  const void* xn;
  long ldxn;
  const void* x;
  long ldx;
  const void* w1;  // [hid][C] compute dtype
  const float* b1;
  const float* wpos;  // [hid][9]
  const float* bpos;
  const void* w2;  // [C][hid] compute dtype
  const float* b2;
  const float* ls;
  const float* rowscale;  // [B] or null
  void* out;
  long ldout;
  void* f;
  long ldf;
};

// LDS pitch (elements) of a row of `n` elements: +16 bytes, so the 8-byte MFMA-layout writes of 16
// consecutive rows and the 16-byte fragment / vector reads spread over the banks
template <typename T> constexpr int lpitch(int n) { return n + 16 / (int)sizeof(T); }

// Copy rows x cols (cols % (16/sizeof(T)) == 0) into LDS with pitch lp; rowptr(r) == nullptr -> zeros.
template <typename T, int NT, typename F>
DFM_INLINE void stage_rows(T* lds, int lp, int rows, int cols, F rowptr) {
  constexpr int V = 16 / sizeof(T);
  const int vpr = cols / V;
  for (int i = threadIdx.x; i < rows * vpr; i += NT) {
    const int r = i / vpr, c = (i - r * vpr) * V;
    const T* src = rowptr(r);
    const uint4 v = src ? *reinterpret_cast<const uint4*>(src + c) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(lds + r * lp + c) = v;
  }
}

// MFMA over k in [0, K) with A rows / B rows k-contiguous in LDS (pitch lpa / lpb):
// acc[it] += A[i0 + 16 it + l&15][k] B[j0 + l&15][k]  (C/D: rows i, cols j)
template <typename T, int NI>
DFM_INLINE void mma_rows(float4_t (&acc)[NI], const T* A, int lpa, const T* B, int lpb, int K, int lane) {
  using M = MM<T>;
  const int kq = M::KL * (lane >> 4);
  const T* brow = B + (lane & 15) * lpb;
  const T* arow = A + (lane & 15) * lpa;
  for (int k0 = 0; k0 < K; k0 += M::KS) {
    const int k = k0 + kq;
    const bool ok = k < K;
    const typename M::frag b = ok ? M::load(brow + k) : M::zero();
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const typename M::frag av = ok ? M::load(arow + it * 16 * lpa + k) : M::zero();
      acc[it] = M::mma(acc[it], av, b);
    }
  }
}

// A rows x cols block (cols % (16/sizeof(T)) == 0, row stride ld in global) split over NT threads as
// 16-byte vectors: load() issues the global loads into registers, store() writes them to LDS later,
// so a chunk's operands travel while the previous chunk computes.
template <typename T, int NT, int NV>
struct Prefetch2D {
  static constexpr int V = 16 / sizeof(T);
  uint4 v[NV];
  DFM_INLINE void load(const T* src, long ld, int rows, int cols) {
    const int vpr = cols / V;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = threadIdx.x + j * NT;
      if (i < rows * vpr) {
        const int r = i / vpr, c = (i - r * vpr) * V;
        v[j] = *reinterpret_cast<const uint4*>(src + r * ld + c);
      }
    }
  }
  DFM_INLINE void store(T* lds, int lp, int rows, int cols) const {
    const int vpr = cols / V;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int i = threadIdx.x + j * NT;
      if (i < rows * vpr) {
        const int r = i / vpr, c = (i - r * vpr) * V;
        *reinterpret_cast<uint4*>(lds + r * lp + c) = v[j];
      }
    }
  }
};

// Per-chunk fp32 parameters of HC hidden channels starting at c0, in LDS as
//   pb[0, HC) = b1, pb[HC, 2 HC) = bpos, pb[2 HC + t HC + ch] = wpos[c0 + ch][t] (tap-major).
template <int HC, int NT>
struct ParamPrefetch {
  static constexpr int N4 = (2 * HC + 9 * HC) / 4;  // float4 units: b1, bpos, wpos[HC][9]
  static_assert(N4 <= NT, "one float4 per thread");
  float4 v;
  DFM_INLINE void load(const float* b1, const float* bpos, const float* wpos, int c0) {
    const int i = threadIdx.x;
    if (i < HC / 4) v = reinterpret_cast<const float4*>(b1 + c0)[i];
    else if (i < HC / 2) v = reinterpret_cast<const float4*>(bpos + c0)[i - HC / 4];
    else if (i < N4) v = reinterpret_cast<const float4*>(wpos + (long)c0 * 9)[i - HC / 2];
  }
  DFM_INLINE void store(float* pb) const {
    const int i = threadIdx.x;
    if (i < HC / 2) {
      reinterpret_cast<float4*>(pb)[i] = v;
    } else if (i < N4) {
      const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = (i - HC / 2) * 4 + e, ch = idx / 9, t = idx - ch * 9;
        pb[2 * HC + t * HC + ch] = f[e];
      }
    }
  }
};

// 3x3 depthwise + bias + identity on 8 channels, taps from the LDS parameter block: img points at
// channel 0 of the group in an LDS image with pitch LP and HW pixels per image row; base = the
// top-left neighbour; pw = &pb[2 HC + ch0] (tap t at pw[t * HC]), pbias = &pb[HC + ch0] or null.
template <typename T, int LP, int HW, int HC, bool FLIP>
DFM_INLINE void dw_unit_lds(const T* img, int base, const float* pw, const float* pbias, float (&sv)[8]) {
  float cv[8];
  ld8<T>(img + (base + HW + 1) * LP, cv);
  if (pbias) {
    float bv[8];
    ld8<float>(pbias, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) sv[e] = bv[e] + cv[e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) sv[e] = cv[e];
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    float nv[8], wv[8];
    const int tt = FLIP ? 8 - t : t;  // FLIP: the transposed conv (backward-data) of the same taps
    ld8<T>(img + (base + (t / 3) * HW + t % 3) * LP, nv);
    ld8<float>(pw + tt * HC, wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) sv[e] = fmaf(wv[e], nv[e], sv[e]);
  }
}

template <typename T, int NTHR>
struct FfnBase {
  static constexpr int NT = NTHR;
  static constexpr int NWV = NTHR / 64;
};

template <typename T, int CT, int TH, int TW, int HC, int NTHR>
struct FfnGeom : FfnBase<T, NTHR> {
  static constexpr int HW2 = TW + 2;
  static constexpr int NH = (TH + 2) * (TW + 2);  // tile + 1-pixel halo
  static constexpr int NHP = (NH + 15) / 16 * 16;
  static constexpr int TP = TH * TW;
  static constexpr int XP = lpitch<T>(CT);  // xn / W1 row pitch
  static constexpr int HP = lpitch<T>(HC);  // h / g / W2-chunk row pitch
  static constexpr int SP = CT + 4;         // fp32 epilogue staging pitch
  static constexpr size_t o_w1 = (size_t)NHP * XP * sizeof(T);
  static constexpr size_t o_w2 = o_w1 + (size_t)HC * XP * sizeof(T);
  static constexpr size_t o_h = o_w2 + (size_t)CT * HP * sizeof(T);
  static constexpr size_t o_g = o_h + (size_t)NHP * HP * sizeof(T);
  static constexpr size_t o_p = o_g + (size_t)TP * HP * sizeof(T);
  static constexpr size_t lds_main = o_p + (size_t)11 * HC * sizeof(float);
  static constexpr size_t lds_stage = (size_t)TP * SP * sizeof(float);
  static constexpr size_t lds = lds_main > lds_stage ? lds_main : lds_stage;
};

// ---------------------------------------------------------------- forward
template <typename T, int CT, int TH, int TW, int HC, int NTHR>
__global__ __launch_bounds__(NTHR) void convffn_fwd_kernel(FfnArgs a) {
  using G = FfnGeom<T, CT, TH, TW, HC, NTHR>;
  constexpr int NT = G::NT, NWV = G::NWV, TP = G::TP, XP = G::XP, HP = G::HP;
  constexpr int PT = TP / 16;                    // pixel tiles of fc2
  constexpr int PTW = (PT + NWV - 1) / NWV;      // per wave
  constexpr int OT = CT / 16;                    // output-channel tiles of fc2
  constexpr int G8 = HC / 8;                     // 8-channel groups of the depthwise stage
  constexpr int NT1 = G::NHP / 16;               // fc1 pixel tiles (tile + halo)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);            // [NHP][XP] xn on tile + halo
  T* w1s = reinterpret_cast<T*>(smem + G::o_w1);  // [HC][XP] W1 rows of the chunk
  T* w2s = reinterpret_cast<T*>(smem + G::o_w2);  // [CT][HP] W2[:, chunk]
  T* hs = reinterpret_cast<T*>(smem + G::o_h);   // [NHP][HP] h chunk
  T* gs = reinterpret_cast<T*>(smem + G::o_g);   // [TP][HP] GELU output chunk

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, tid = threadIdx.x;
  const int tile = blockIdx.x;
  const int b = tile / (a.tiles_y * a.tiles_x);
  const int ty = (tile / a.tiles_x) % a.tiles_y, tx = tile % a.tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int C = a.C, hid = a.hid;
  const T* xn = (const T*)a.xn;
  const T* w1 = (const T*)a.w1;
  const T* w2 = (const T*)a.w2;
  auto inside = [&](int yy, int xx) { return yy >= 0 && yy < a.H && xx >= 0 && xx < a.W; };
  auto halo_ok = [&](int q) {
    const int yy = y0 - 1 + q / G::HW2, xx = x0 - 1 + q % G::HW2;
    return q < G::NH && inside(yy, xx);
  };

  float* pb = reinterpret_cast<float*>(smem + G::o_p);  // [11][HC] b1 | bpos | wpos (tap-major)
  constexpr int VEC = 16 / sizeof(T);
  Prefetch2D<T, NT, (HC * CT / VEC + NT - 1) / NT> pw1, pw2;
  ParamPrefetch<HC, NT> ppar;
  auto fetch = [&](int c) {
    pw1.load(w1 + (long)c * C, C, HC, C);
    pw2.load(w2 + c, hid, C, HC);
    ppar.load(a.b1, a.bpos, a.wpos, c);
  };
  auto put = [&]() {
    pw1.store(w1s, XP, HC, C);
    pw2.store(w2s, HP, C, HC);
    ppar.store(pb);
  };
  fetch(0);
  stage_rows<T, NT>(xs, XP, G::NHP, C, [&](int q) -> const T* {
    const int yy = y0 - 1 + q / G::HW2, xx = x0 - 1 + q % G::HW2;
    return (q < G::NH && inside(yy, xx)) ? xn + ((long)(b * a.H + yy) * a.W + xx) * a.ldxn : nullptr;
  });
  put();

  float4_t acc[PTW][OT];
#pragma unroll
  for (int i = 0; i < PTW; ++i)
#pragma unroll
    for (int j = 0; j < OT; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  const int g = tid % G8;
  __syncthreads();

  for (int c0 = 0; c0 < hid; c0 += HC) {
    const bool more = c0 + HC < hid;
    if (more) fetch(c0 + HC);  // next chunk's operands in flight under this chunk's work
    // ---- fc1 on tile + halo: h^T[hidden][pixel] = W1c xn^T -> hs[pixel][hidden]
#pragma unroll 1
    for (int jt = wid; jt < NT1; jt += NWV) {
      float4_t h[HC / 16];
#pragma unroll
      for (int it = 0; it < HC / 16; ++it) h[it] = float4_t{0.f, 0.f, 0.f, 0.f};
      mma_rows<T, HC / 16>(h, w1s, XP, xs + jt * 16 * XP, XP, C, lane);
      const int q = jt * 16 + (lane & 15);
      const bool val = halo_ok(q);
#pragma unroll
      for (int it = 0; it < HC / 16; ++it) {
        const int ch = it * 16 + 4 * (lane >> 4);
        const float4 bb = *reinterpret_cast<const float4*>(pb + ch);
        const float v[4] = {val ? h[it][0] + bb.x : 0.f, val ? h[it][1] + bb.y : 0.f, val ? h[it][2] + bb.z : 0.f,
                            val ? h[it][3] + bb.w : 0.f};
        st4(hs + q * HP + ch, v);
      }
    }
    __syncthreads();
    // ---- depthwise 3x3 + bias + identity + GELU: hs -> gs, one (pixel, 8-channel) unit at a time
#pragma unroll 1
    for (int u = tid; u < TP * G8; u += NT) {
      const int p = u / G8;
      float sv[8];
      dw_unit_lds<T, HP, G::HW2, HC, false>(hs + g * 8, (p / TW) * G::HW2 + p % TW, pb + 2 * HC + g * 8,
                                             pb + HC + g * 8, sv);
#pragma unroll
      for (int e = 0; e < 8; ++e) sv[e] = gelu_f(sv[e]);
      st8<T>(gs + p * HP + g * 8, sv);
    }
    __syncthreads();
    // ---- fc2 chunk: out^T[c][p] += W2c[c][k] g^T[k][p]
#pragma unroll
    for (int i = 0; i < PTW; ++i) {
      const int pj = wid + i * NWV;
      if (pj < PT) mma_rows<T, OT>(acc[i], w2s, HP, gs + pj * 16 * HP, HP, HC, lane);
    }
    if (more) {
      __syncthreads();  // this chunk's reads of w1s / w2s / pb are done
      put();
      __syncthreads();
    }
  }
  __syncthreads();  // chunk images dead: the fp32 staging tile reuses the LDS
  float* st = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pj = wid + i * NWV;
    if (pj >= PT) break;
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const float v[4] = {acc[i][ot][0], acc[i][ot][1], acc[i][ot][2], acc[i][ot][3]};
      st4(st + (pj * 16 + (lane & 15)) * G::SP + ot * 16 + 4 * (lane >> 4), v);
    }
  }
  __syncthreads();
  const float rs = a.rowscale ? a.rowscale[b] : 1.f;
  const int CG = C / 8;
  for (int u = tid; u < TP * CG; u += NT) {
    const int p = u / CG, c = (u % CG) * 8;
    const int yy = y0 + p / TW, xx = x0 + p % TW;
    if (!inside(yy, xx)) continue;
    const long row = (long)(b * a.H + yy) * a.W + xx;
    float v[8], xv[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = st[p * G::SP + c + e] + a.b2[c + e];
    st8<T>((T*)a.f + row * a.ldf + c, v);
    ld8<T>((const T*)a.x + row * a.ldx + c, xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = xv[e] + a.ls[c + e] * rs * v[e];
    st8<T>((T*)a.out + row * a.ldout + c, o);
  }
}

// ---------------------------------------------------------------- backward
// Given df = dout * ls * rowscale (the residual's chain rule, dfm_residual_bwd) the tile stages xn
// on tile + 2-pixel halo and df on tile + 1-pixel halo in LDS, then per hidden chunk recomputes h
// (fc1, MFMA) on tile + 2 halo, forms dg = df W2 on tile + 1 halo (MFMA), hpre = DW3(h) + bpos + h
// and g = GELU(hpre) (VALU), dhpre = dg * GELU'(hpre), dh = DW3^T(dhpre) + dhpre on the tile,
// dxn += dh W1 (MFMA, accumulated over the chunks) and the depthwise weight / bias gradient
// partials sum_p dhpre[p] h[p + tap]. It writes g and dh ([P, hid], the inputs of the fc2 / fc1
// weight-gradient GEMMs), dxn ([P, C]) and one [hid][10] partial per workgroup; hpre / dhpre never
// reach HBM.
struct FfnBwdArgs {
  int B, H, W, C, hid;
  int tiles_y, tiles_x;
  const void* xn;
  long ldxn;
  const void* df;
  long lddf;
  const void* w1;   // [hid][C]
  const float* b1;
  const float* wpos;
  const float* bpos;
  const void* w2t;  // [hid][C]  (fc2 weight, transposed)
  const void* w1t;  // [C][hid]  (fc1 weight, transposed)
  void* g;          // [P][ldg] GELU output
  long ldg;
  void* dh;         // [P][lddh] fc1-output gradient
  long lddh;
  void* dxn;        // [P][lddxn]
  long lddxn;
  float* part;      // [nblk][hid * 10] depthwise weight (9) + bias (1) gradient partials
};

template <typename T, int CT, int TH, int TW, int HC, int NTHR>
struct FfnBwdGeom : FfnBase<T, NTHR> {
  static constexpr int HW2 = TW + 2, HW4 = TW + 4;
  static constexpr int NH1 = (TH + 2) * (TW + 2);
  static constexpr int NH1P = (NH1 + 15) / 16 * 16;
  static constexpr int NH2 = (TH + 4) * (TW + 4);
  static constexpr int NH2P = (NH2 + 15) / 16 * 16;
  static constexpr int TP = TH * TW;
  static constexpr int XP = lpitch<T>(CT);
  static constexpr int HP = lpitch<T>(HC);
  static constexpr int SP = CT + 4;
  static constexpr int G8 = HC / 8;
  static constexpr int NPAIR = G8 * 10;              // (8-channel group, tap|bias) pairs
  static constexpr int NSL = NTHR / NPAIR > 3 ? 3 : NTHR / NPAIR;  // pixel slices of the dw-gradient reduction
  static constexpr size_t o_df = (size_t)NH2P * XP * sizeof(T);
  static constexpr size_t o_w1 = o_df + (size_t)NH1P * XP * sizeof(T);
  static constexpr size_t o_w2t = o_w1 + (size_t)HC * XP * sizeof(T);
  static constexpr size_t o_w1t = o_w2t + (size_t)HC * XP * sizeof(T);
  static constexpr size_t o_h = o_w1t + (size_t)CT * HP * sizeof(T);
  static constexpr size_t o_d = o_h + (size_t)(NH2P > TP ? NH2P : TP) * HP * sizeof(T);
  static constexpr size_t o_r = o_d + (size_t)NH1P * HP * sizeof(T);
  static constexpr size_t o_p = o_r + (size_t)NSL * NPAIR * 8 * sizeof(float);
  static constexpr size_t lds_main = o_p + (size_t)11 * HC * sizeof(float);
  static constexpr size_t lds_stage = (size_t)TP * SP * sizeof(float);
  static constexpr size_t lds = lds_main > lds_stage ? lds_main : lds_stage;
};

template <typename T, int CT, int TH, int TW, int HC, int NTHR>
__global__ __launch_bounds__(NTHR, 2) void convffn_bwd_kernel(FfnBwdArgs a) {
  using G = FfnBwdGeom<T, CT, TH, TW, HC, NTHR>;
  constexpr int NT = G::NT, NWV = G::NWV, TP = G::TP, XP = G::XP, HP = G::HP, G8 = G::G8;
  constexpr int PT = TP / 16;
  constexpr int PTW = (PT + NWV - 1) / NWV;
  constexpr int OT = CT / 16;
  constexpr int NT2 = G::NH2P / 16;  // fc1 pixel tiles (tile + 2 halo)
  constexpr int NT1 = G::NH1P / 16;  // dg pixel tiles (tile + 1 halo)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);                 // [NH2P][XP] xn on tile + 2 halo
  T* dfs = reinterpret_cast<T*>(smem + G::o_df);      // [NH1P][XP] df on tile + 1 halo
  T* w1s = reinterpret_cast<T*>(smem + G::o_w1);      // [HC][XP] W1 rows of the chunk
  T* w2ts = reinterpret_cast<T*>(smem + G::o_w2t);    // [HC][XP] W2^T rows of the chunk
  T* w1ts = reinterpret_cast<T*>(smem + G::o_w1t);    // [CT][HP] W1^T[:, chunk]
  T* hs = reinterpret_cast<T*>(smem + G::o_h);        // [NH2P][HP] h; later [TP][HP] dh
  T* ds = reinterpret_cast<T*>(smem + G::o_d);        // [NH1P][HP] dg -> dhpre
  float* red = reinterpret_cast<float*>(smem + G::o_r);  // [NSL][NPAIR][8]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, tid = threadIdx.x;
  const int tile = blockIdx.x;
  const int b = tile / (a.tiles_y * a.tiles_x);
  const int ty = (tile / a.tiles_x) % a.tiles_y, tx = tile % a.tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int C = a.C, hid = a.hid;
  const T* xn = (const T*)a.xn;
  const T* df = (const T*)a.df;
  const T* w1 = (const T*)a.w1;
  const T* w2t = (const T*)a.w2t;
  const T* w1t = (const T*)a.w1t;
  const int g = tid % G8;
  auto pix = [&](int yy, int xx) { return (long)(b * a.H + yy) * a.W + xx; };
  auto inside = [&](int yy, int xx) { return yy >= 0 && yy < a.H && xx >= 0 && xx < a.W; };

  float* pb = reinterpret_cast<float*>(smem + G::o_p);  // [11][HC] b1 | bpos | wpos (tap-major)
  constexpr int VEC = 16 / sizeof(T);
  Prefetch2D<T, NT, (HC * CT / VEC + NT - 1) / NT> pw1, pw2t, pw1t;
  ParamPrefetch<HC, NT> ppar;
  auto fetch = [&](int c) {
    pw1.load(w1 + (long)c * C, C, HC, C);
    pw2t.load(w2t + (long)c * C, C, HC, C);
    pw1t.load(w1t + c, hid, C, HC);
    ppar.load(a.b1, a.bpos, a.wpos, c);
  };
  auto put = [&]() {
    pw1.store(w1s, XP, HC, C);
    pw2t.store(w2ts, XP, HC, C);
    pw1t.store(w1ts, HP, C, HC);
    ppar.store(pb);
  };
  fetch(0);
  stage_rows<T, NT>(xs, XP, G::NH2P, C, [&](int q) -> const T* {
    const int yy = y0 - 2 + q / G::HW4, xx = x0 - 2 + q % G::HW4;
    return (q < G::NH2 && inside(yy, xx)) ? xn + pix(yy, xx) * a.ldxn : nullptr;
  });
  stage_rows<T, NT>(dfs, XP, G::NH1P, C, [&](int q) -> const T* {
    const int yy = y0 - 1 + q / G::HW2, xx = x0 - 1 + q % G::HW2;
    return (q < G::NH1 && inside(yy, xx)) ? df + pix(yy, xx) * a.lddf : nullptr;
  });
  put();

  float4_t acc[PTW][OT];  // dxn^T[c][p]
#pragma unroll
  for (int i = 0; i < PTW; ++i)
#pragma unroll
    for (int j = 0; j < OT; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (int c0 = 0; c0 < hid; c0 += HC) {
    const bool more = c0 + HC < hid;
    if (more) fetch(c0 + HC);  // next chunk's operands in flight under this chunk's work
    // ---- [1] h on tile + 2 halo -> hs ; [2] dg on tile + 1 halo -> ds
#pragma unroll 1
    for (int jt = wid; jt < NT2 + NT1; jt += NWV) {
      float4_t h[HC / 16];
#pragma unroll
      for (int it = 0; it < HC / 16; ++it) h[it] = float4_t{0.f, 0.f, 0.f, 0.f};
      if (jt < NT2) {
        mma_rows<T, HC / 16>(h, w1s, XP, xs + jt * 16 * XP, XP, C, lane);
        const int q = jt * 16 + (lane & 15);
        const int yy = y0 - 2 + q / G::HW4, xx = x0 - 2 + q % G::HW4;
        const bool val = q < G::NH2 && inside(yy, xx);
#pragma unroll
        for (int it = 0; it < HC / 16; ++it) {
          const int ch = it * 16 + 4 * (lane >> 4);
          const float4 bb = *reinterpret_cast<const float4*>(pb + ch);
          const float v[4] = {val ? h[it][0] + bb.x : 0.f, val ? h[it][1] + bb.y : 0.f, val ? h[it][2] + bb.z : 0.f,
                              val ? h[it][3] + bb.w : 0.f};
          st4(hs + q * HP + ch, v);
        }
      } else {
        const int j1 = jt - NT2;
        mma_rows<T, HC / 16>(h, w2ts, XP, dfs + j1 * 16 * XP, XP, C, lane);
        const int q = j1 * 16 + (lane & 15);
#pragma unroll
        for (int it = 0; it < HC / 16; ++it) {
          const float v[4] = {h[it][0], h[it][1], h[it][2], h[it][3]};
          st4(ds + q * HP + it * 16 + 4 * (lane >> 4), v);
        }
      }
    }
    __syncthreads();
    // ---- [3] hpre = DW3(h) + bpos + h on tile + 1 halo; g = GELU(hpre) (tile pixels -> HBM);
    //          dhpre = dg * GELU'(hpre) in place (df rows outside the image are zero)
#pragma unroll 1
    for (int u = tid; u < G::NH1 * G8; u += NT) {
      const int q = u / G8;
      const int qy = q / G::HW2, qx = q % G::HW2;
      float sv[8], dv[8], gv[8];
      dw_unit_lds<T, HP, G::HW4, HC, false>(hs + g * 8, qy * G::HW4 + qx, pb + 2 * HC + g * 8, pb + HC + g * 8, sv);
      ld8<T>(ds + q * HP + g * 8, dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float cdf, pdf;
        normal_cdf_pdf(sv[e], cdf, pdf);
        gv[e] = sv[e] * cdf;
        dv[e] *= fmaf(sv[e], pdf, cdf);
      }
      st8<T>(ds + q * HP + g * 8, dv);
      const int yy = y0 - 1 + qy, xx = x0 - 1 + qx;
      if (qy >= 1 && qy <= TH && qx >= 1 && qx <= TW && inside(yy, xx))
        st8<T>((T*)a.g + pix(yy, xx) * a.ldg + c0 + g * 8, gv);
    }
    __syncthreads();
    // ---- [4] depthwise weight / bias gradient partials: sum_p dhpre[p] * h[p + (dy-1, dx-1)]
    {
      const int pr = tid % G::NPAIR, sl = tid / G::NPAIR;
      if (sl < G::NSL) {
        const int gg = pr / 10, t = pr % 10;
        const int off = t < 9 ? (t / 3) * G::HW4 + t % 3 : G::HW4 + 1;
        float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int p = sl; p < TP; p += G::NSL) {
          const int py = p / TW, px = p % TW;
          float dv[8], hv[8];
          ld8<T>(ds + ((py + 1) * G::HW2 + px + 1) * HP + gg * 8, dv);
          if (t < 9) {
            ld8<T>(hs + ((py + 1) * G::HW4 + px + 1 + off) * HP + gg * 8, hv);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) hv[e] = 1.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) s8[e] = fmaf(dv[e], hv[e], s8[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(sl * G::NPAIR + pr) * 8 + e] = s8[e];
      }
    }
    // ---- [5] dh = DW3^T(dhpre) + dhpre on the tile (flipped taps, identity, no bias)
    {
      constexpr int NU = (TP * G8 + NT - 1) / NT;
      float dhv[NU][8];
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        const int p = min((tid + j * NT) / G8, TP - 1);
        const int pc = (p / TW + 1) * G::HW2 + p % TW + 1;  // the pixel in ds coordinates
        // dh[p] = dhpre[p] + sum_t w[t] dhpre[p - (t/3 - 1, t%3 - 1)]: the flipped 3x3 around p
        dw_unit_lds<T, HP, G::HW2, HC, true>(ds + g * 8, pc - G::HW2 - 1, pb + 2 * HC + g * 8, nullptr, dhv[j]);
      }
      __syncthreads();  // [4] reads of hs done: dh overwrites it; red complete
      for (int i = tid; i < G::NPAIR * 8; i += NT) {
        const int pr = i / 8, e = i % 8, gg = pr / 10, t = pr % 10;
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < G::NSL; ++sl) v += red[(sl * G::NPAIR + pr) * 8 + e];
        a.part[(long)blockIdx.x * hid * 10 + (long)(c0 + gg * 8 + e) * 10 + t] = v;
      }
#pragma unroll
      for (int j = 0; j < NU; ++j) {
        const int u = tid + j * NT;
        if (u >= TP * G8) break;
        const int p = u / G8;
        const int yy = y0 + p / TW, xx = x0 + p % TW;
        st8<T>(hs + p * HP + g * 8, dhv[j]);
        if (inside(yy, xx)) st8<T>((T*)a.dh + pix(yy, xx) * a.lddh + c0 + g * 8, dhv[j]);
      }
    }
    __syncthreads();
    // ---- [6] dxn^T[c][p] += W1^T[c][chunk] dh^T
#pragma unroll
    for (int i = 0; i < PTW; ++i) {
      const int pj = wid + i * NWV;
      if (pj < PT) mma_rows<T, OT>(acc[i], w1ts, HP, hs + pj * 16 * HP, HP, HC, lane);
    }
    __syncthreads();  // this chunk's reads of the weight chunks, pb and hs (dh) are done
    if (more) {
      put();
      __syncthreads();
    }
  }
  __syncthreads();
  float* st = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pj = wid + i * NWV;
    if (pj >= PT) break;
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const float v[4] = {acc[i][ot][0], acc[i][ot][1], acc[i][ot][2], acc[i][ot][3]};
      st4(st + (pj * 16 + (lane & 15)) * G::SP + ot * 16 + 4 * (lane >> 4), v);
    }
  }
  __syncthreads();
  const int CG = C / 8;
  for (int u = tid; u < TP * CG; u += NT) {
    const int p = u / CG, c = (u % CG) * 8;
    const int yy = y0 + p / TW, xx = x0 + p % TW;
    if (!inside(yy, xx)) continue;
    st8<T>((T*)a.dxn + pix(yy, xx) * a.lddxn + c, st + p * G::SP + c);
  }
}

// ---------------------------------------------------------------- launch configurations
// (tile, hidden chunk, threads) per channel-width class, sized so two workgroups fit a CU's LDS
// for bf16 (fp32, the parity path, runs one per CU).
template <typename T, int CT> struct FwdCfg { static constexpr int TH = 8, TW = CT <= 64 ? 16 : 8, HC = 32, NT = 256; };
template <typename T, int CT> struct BwdCfg { static constexpr int TH = CT <= 128 ? 8 : 4, TW = 8, HC = 32, NT = 256; };
// fp32 (the parity path) doubles every LDS image: smaller backward tiles, and C > 128 unsupported
template <> struct BwdCfg<float, 128> { static constexpr int TH = 4, TW = 4, HC = 32, NT = 256; };
template <> struct FwdCfg<float, 256> { static constexpr int TH = 1, TW = 1, HC = 32, NT = 256; };  // unused
template <> struct BwdCfg<float, 256> { static constexpr int TH = 1, TW = 1, HC = 32, NT = 256; };  // unused

constexpr int HC_ALL = 32;  // every configuration walks the hidden dim in chunks of 32

template <typename T, int CT>
int launch_fwd(FfnArgs& a, hipStream_t s) {
  using Cf = FwdCfg<T, CT>;
  using G = FfnGeom<T, CT, Cf::TH, Cf::TW, Cf::HC, Cf::NT>;
  static_assert(G::lds <= 160 * 1024, "LDS");
  auto kern = convffn_fwd_kernel<T, CT, Cf::TH, Cf::TW, Cf::HC, Cf::NT>;
  a.tiles_y = cdiv(a.H, Cf::TH);
  a.tiles_x = cdiv(a.W, Cf::TW);
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  DFM_LAUNCH(kern, dim3((unsigned)nblk), dim3(Cf::NT), G::lds, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, int CT>
int launch_bwd(FfnBwdArgs& a, hipStream_t s) {
  using Cf = BwdCfg<T, CT>;
  using G = FfnBwdGeom<T, CT, Cf::TH, Cf::TW, Cf::HC, Cf::NT>;
  static_assert(G::lds <= 160 * 1024, "LDS");
  auto kern = convffn_bwd_kernel<T, CT, Cf::TH, Cf::TW, Cf::HC, Cf::NT>;
  a.tiles_y = cdiv(a.H, Cf::TH);
  a.tiles_x = cdiv(a.W, Cf::TW);
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  DFM_LAUNCH(kern, dim3((unsigned)nblk), dim3(Cf::NT), G::lds, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, int CT>
long bwd_blocks(int B, int H, int W) {
  return (long)B * cdiv(H, BwdCfg<T, CT>::TH) * cdiv(W, BwdCfg<T, CT>::TW);
}

template <typename T>
long bwd_nblk(int B, int H, int W, int C) {
  if (C <= 32) return bwd_blocks<T, 32>(B, H, W);
  if (C <= 64) return bwd_blocks<T, 64>(B, H, W);
  if (C <= 128) return bwd_blocks<T, 128>(B, H, W);
  if constexpr (sizeof(T) == 2) return bwd_blocks<T, 256>(B, H, W);
  return 0;
}

template <typename T>
int bwd_dispatch(FfnBwdArgs& a, hipStream_t s) {
  if (a.C <= 32) return launch_bwd<T, 32>(a, s);
  if (a.C <= 64) return launch_bwd<T, 64>(a, s);
  if (a.C <= 128) return launch_bwd<T, 128>(a, s);
  if constexpr (sizeof(T) == 2) return launch_bwd<T, 256>(a, s);
  return DFM_ERR_ARG;
}

template <typename T>
int fwd_dispatch(FfnArgs& a, hipStream_t s) {
  if (a.C <= 32) return launch_fwd<T, 32>(a, s);
  if (a.C <= 64) return launch_fwd<T, 64>(a, s);
  if (a.C <= 128) return launch_fwd<T, 128>(a, s);
  if constexpr (sizeof(T) == 2) return launch_fwd<T, 256>(a, s);
  return DFM_ERR_ARG;
}

bool al16p(const void* p, long ld, int es) { return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0); }

}  // namespace

extern "C" int dfm_convffn_supported(int dtype, int C, int hid) {
  if (dtype != DFM_BF16 && dtype != DFM_F32) return 0;
  return C >= 8 && C <= (dtype == DFM_BF16 ? 256 : 128) && C % 8 == 0 && hid > 0 && hid % HC_ALL == 0;
}

extern "C" int dfm_convffn_fwd(int dtype, int B, int H, int W, int C, int hid, const void* xn, long ldxn,
                               const void* x, long ldx, const void* w1, const float* b1, const float* wpos,
                               const float* bpos, const void* w2, const float* b2, const float* ls,
                               const float* rowscale, void* out, long ldout, void* f, long ldf, dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, C, hid), "dfm_convffn_fwd: unsupported C=%d hid=%d dtype=%d", C, hid,
                dtype);
  DFM_CHECK_ARG(xn && x && w1 && b1 && wpos && bpos && w2 && b2 && ls && out && f, "dfm_convffn_fwd: null argument");
  const int es = dtype == DFM_BF16 ? 2 : 4;
  DFM_CHECK_ARG(al16p(xn, ldxn, es) && al16p(x, ldx, es) && al16p(out, ldout, es) && al16p(f, ldf, es) &&
                    al16p(w1, C, es) && al16p(w2, hid, es) && al16p(b1, 0, 4) && al16p(bpos, 0, 4) &&
                    al16p(wpos, 0, 4),
                "dfm_convffn_fwd: rows must be 16-byte aligned");
  if ((long)B * H * W == 0) return DFM_OK;
  FfnArgs a{};
  a.B = B; a.H = H; a.W = W; a.C = C; a.hid = hid;
  a.xn = xn; a.ldxn = ldxn; a.x = x; a.ldx = ldx;
  a.w1 = w1; a.b1 = b1; a.wpos = wpos; a.bpos = bpos; a.w2 = w2; a.b2 = b2;
  a.ls = ls; a.rowscale = rowscale; a.out = out; a.ldout = ldout; a.f = f; a.ldf = ldf;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return fwd_dispatch<bf16_t>(a, s);
  return fwd_dispatch<float>(a, s);
}

extern "C" size_t dfm_convffn_bwd_workspace(int dtype, int B, int H, int W, int C, int hid) {
  const long nblk = dtype == DFM_BF16 ? bwd_nblk<bf16_t>(B, H, W, C) : bwd_nblk<float>(B, H, W, C);
  return (size_t)nblk * hid * 10 * sizeof(float);
}

extern "C" int dfm_convffn_bwd(int dtype, int B, int H, int W, int C, int hid, const void* xn, long ldxn,
                               const void* df, long lddf, const void* w1, const float* b1, const float* wpos,
                               const float* bpos, const void* w2t, const void* w1t, void* g, long ldg, void* dh,
                               long lddh, void* dxn, long lddxn, float* dwpos, float* dbpos, void* workspace,
                               dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, C, hid), "dfm_convffn_bwd: unsupported C=%d hid=%d dtype=%d", C, hid,
                dtype);
  DFM_CHECK_ARG(xn && df && w1 && b1 && wpos && bpos && w2t && w1t && g && dh && dxn && dwpos && dbpos && workspace,
                "dfm_convffn_bwd: null argument");
  const int es = dtype == DFM_BF16 ? 2 : 4;
  DFM_CHECK_ARG(al16p(xn, ldxn, es) && al16p(df, lddf, es) && al16p(g, ldg, es) && al16p(dh, lddh, es) &&
                    al16p(dxn, lddxn, es) && al16p(w1, C, es) && al16p(w2t, C, es) && al16p(w1t, hid, es) &&
                    al16p(b1, 0, 4) && al16p(bpos, 0, 4) && al16p(wpos, 0, 4),
                "dfm_convffn_bwd: rows must be 16-byte aligned");
  if ((long)B * H * W == 0) return DFM_OK;
  FfnBwdArgs a{};
  a.B = B; a.H = H; a.W = W; a.C = C; a.hid = hid;
  a.xn = xn; a.ldxn = ldxn; a.df = df; a.lddf = lddf;
  a.w1 = w1; a.b1 = b1; a.wpos = wpos; a.bpos = bpos; a.w2t = w2t; a.w1t = w1t;
  a.g = g; a.ldg = ldg; a.dh = dh; a.lddh = lddh; a.dxn = dxn; a.lddxn = lddxn;
  a.part = (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  const int rc = dtype == DFM_BF16 ? bwd_dispatch<bf16_t>(a, s) : bwd_dispatch<float>(a, s);
  if (rc != DFM_OK) return rc;
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  DFM_LAUNCH(partial_sum_kernel<2>, dim3(cdiv((long)hid * 10, 64)), dim3(1024), 0, s, (int)nblk, (long)hid * 10,
             (const float*)workspace, dwpos, dbpos, 10L, 0);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
