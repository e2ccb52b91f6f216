// Fused ConvFFN (K4) for gfx950 — DFormer's MLP (models/encoders/DFormer.py:48-67) inside the Block
// residual (DFormer.py:173-179):
//
//   out = x + rowscale[b] * ls * f,   f = fc2(g) + b2,   g = GELU(hpre),
//   hpre = DW3x3(h) + bpos + h,       h = fc1(LN(x)) + b1          (rows = NHWC pixels)
//
// FORWARD (ffn_fwd_kernel): one workgroup per TH x TW tile of output pixels; the [P, R] hidden
// activation is produced and consumed on the CU in chunks of HC channels (the depthwise conv is
// per channel, so a hidden chunk needs only its own channels of h on the tile + 1-pixel halo):
//   prologue  LN of x on the tile + halo -> Xs (LDS, 16-bit), mean / rstd of the tile saved
//   per chunk [A] h^T = W1c xn^T + b1 (MFMA 16x16x32), zero outside the image -> Hs (LDS)
//             [B] every lane computes DW3x3 + bpos + identity and GELU for exactly the 1 pixel x 8
//                 channels it holds as the B operand of out^T += W2c g^T (MFMA): g goes from the VALU
//                 straight into the matrix core; the lane's centre tap of h is stored to HBM (the one
//                 hidden tensor the backward reads)
//   epilogue  f = acc + b2 (saved for the layer-scale gradient), out = x + rowscale * ls * f.
// HBM per pixel: read C (x, + halo from L2), write 2C (out, f) + R (h) elements + 8 B; the unfused
// chain moved 5 hidden tensors (fc1 out, GELU, GELU', and their reads).
//
// BACKWARD, hidden part (ffn_bwd_kernel): one workgroup per (strip of tiles, hidden chunk). Per tile:
//   [A] dg^T = W2c^T df^T on the tile + 1-pixel halo (MFMA; W2c^T held in registers for the strip)
//   [B] hpre recomputed from h (tile + 2-pixel halo, LDS), GELU / GELU' from one erf evaluation,
//       dhpre = dg GELU'(hpre) -> LDS; the depthwise weight / bias gradient sums ride in registers
//       (each lane owns 4 hidden channels for the whole strip)
//   [C] dh = DW3x3^T(dhpre) + dhpre on the tile -> HBM (for the fc1 input gradient GEMM) and LDS
//   [D] dW2^T += g^T df, dW1 += dh^T LN(x) (MFMA, K = pixels, operands read with
//       ds_read_b64_tr_b16 from [pixel][channel] LDS images), accumulated in registers over the strip
// and writes per-strip partials that one fixed-order grouped sum reduces (deterministic). The fc1
// input gradient (dh W1), the LayerNorm backward and the residual / layer-scale backward are the
// library's GEMM / LN / residual entry points, issued by dfm_convffn_bwd.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

// ---- 16-bit element helpers (bf16_t / f16_t storage)
template <typename T> DFM_INLINE float lo16(uint32_t w);
template <typename T> DFM_INLINE float hi16(uint32_t w);
template <> DFM_INLINE float lo16<bf16_t>(uint32_t w) { return __uint_as_float(w << 16); }
template <> DFM_INLINE float hi16<bf16_t>(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
template <> DFM_INLINE float lo16<f16_t>(uint32_t w) { return h2f((uint16_t)(w & 0xffffu)); }
template <> DFM_INLINE float hi16<f16_t>(uint32_t w) { return h2f((uint16_t)(w >> 16)); }
template <typename T> DFM_INLINE uint32_t pack2(float a, float b) {
  return (uint32_t)bits16<T>(a) | ((uint32_t)bits16<T>(b) << 16);
}
template <typename T> DFM_INLINE void ld4h(const T* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = lo16<T>(u.x); v[1] = hi16<T>(u.x); v[2] = lo16<T>(u.y); v[3] = hi16<T>(u.y);
}
template <typename T> DFM_INLINE void st4h(T* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]));
}
template <typename T> DFM_INLINE void unpack8w(const uint4 u, float* v) {
  v[0] = lo16<T>(u.x); v[1] = hi16<T>(u.x); v[2] = lo16<T>(u.y); v[3] = hi16<T>(u.y);
  v[4] = lo16<T>(u.z); v[5] = hi16<T>(u.z); v[6] = lo16<T>(u.w); v[7] = hi16<T>(u.w);
}
DFM_INLINE bf16x8_t as_frag(uint4 u) { return __builtin_bit_cast(bf16x8_t, u); }
template <typename T> DFM_INLINE bf16x8_t ldfrag(const T* p) { return as_frag(*reinterpret_cast<const uint4*>(p)); }

// A / B fragment of v_mfma_f32_16x16x32 with K along the ROWS of a [k][n] 16-bit LDS image (pitch
// in elements, a multiple of 4): lane l gets image[k0 + 8 (l >> 4) + j][n0 + (l & 15)], j < 8, read
// by two ds_read_b64_tr_b16 (each 16-lane group transposes a 4-row x 16-column block).
template <typename T>
DFM_INLINE bf16x8_t tr_frag(const T* img, int pitch, int k0, int n0, int lane) {
  typedef __attribute__((address_space(3))) short4_t lds_s4;
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const T* a0 = img + (k0 + 8 * (lane >> 4) + q) * pitch + n0 + 4 * p;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0 + 4 * pitch));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  const short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, s);
}

struct FfnFwdArgs {
  int B, H, W, R;
  float eps;
  long rps;  // rows per rowscale entry (H * W)
  int tiles_x, tiles_y;
  const void* x;
  const float* lnw;
  const float* lnb;
  const void* w1;  // [R][C]
  const float* b1;
  const float* wpos;  // [R][9]
  const float* bpos;
  const void* w2;  // [C][R]
  const float* b2;
  const float* ls;
  const float* rowscale;  // [B] or NULL
  void* out;
  void* f;
  void* h;   // [P][R] saved for the backward
  void* xn;  // [P][C] LN(x), or NULL
  void* gout;   // [P][R] GELU(hpre), or NULL (with gdout: the op-level backward's saved operands)
  void* gdout;  // [P][R] GELU'(hpre), or NULL
  float* mean;
  float* rstd;
};

// Forward geometry: TH x TW pixel tiles with T * C = 4096 (a wave's partial out^T is 64 fp32 registers
// per lane: 8 x 16 tiles at C = 32, 8 x 8 at 64, 4 x 8 at 128, 4 x 4 at 256); each of the 4 waves owns
// every 4th hidden chunk of HC channels
// and keeps its own partial out^T[C, T] in registers, so the chunk loop has no workgroup barrier:
// a wave computes h for its chunk (tile + 1 halo, MFMA) into its private LDS buffer and reads it back
// for the depthwise conv (wave-local LDS hand-off). The four partials are summed in a fixed order at
// the end (deterministic).
template <int C, int HC, int TH_, int TW_>
struct FwdGeom {
  static constexpr int TH = TH_, TW = TW_, T = TH * TW;
  static constexpr int EW = TW + 2, T1 = (TH + 2) * EW, T1P = (T1 + 15) / 16 * 16;
  static constexpr int XP = C + 8, HP = HC + 8;  // LDS pitches (elements): 16-byte rows, staggered banks
  static constexpr int RB1 = HC / 16, CB1 = T1P / 16, KS1 = C / 32;
  static constexpr int RB2 = C / 16, CB2 = T / 16, KS2 = HC / 32;
  static constexpr int XS = T1P * XP, HS = T1P * HP, PS = 10 * HC;  // elements / floats
  static constexpr int RED = T * C;                                   // floats of one partial
  static constexpr size_t BODY = (size_t)(XS + 4 * HS) * 2 + (size_t)4 * PS * 4;
  static constexpr size_t LDS = BODY > (size_t)2 * RED * 4 ? BODY : (size_t)2 * RED * 4;
  static_assert(T % 16 == 0 && HC % 32 == 0 && C % 32 == 0, "tile geometry");
};

template <typename T, int C, int HC, int TH_, int TW_, bool SAVEG>
__global__ __launch_bounds__(256, 2) void ffn_fwd_kernel(FfnFwdArgs a) {
  using G = FwdGeom<C, HC, TH_, TW_>;
  constexpr int TH = G::TH, TW = G::TW;
  extern __shared__ __align__(16) unsigned char smem[];
  T* Xs = reinterpret_cast<T*>(smem);  // [T1P][XP] LN(x) of tile + halo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, lq = lane >> 4;
  T* Hw = Xs + G::XS + wave * G::HS;  // this wave's [T1P][HP] h chunk
  float* Pw = reinterpret_cast<float*>(Xs + G::XS + 4 * G::HS) + wave * G::PS;  // its taps + bias
  int t = blockIdx.x;
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  const int b = t / a.tiles_y;
  const int y0 = ty * TH, x0 = tx * TW;
  const int H = a.H, W = a.W, R = a.R;
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const T* __restrict__ w1 = static_cast<const T*>(a.w1);
  const T* __restrict__ w2 = static_cast<const T*>(a.w2);
  T* __restrict__ hsave = static_cast<T*>(a.h);

  // ---- prologue: LayerNorm of the tile + 1-pixel halo (DFormer.py:58, eps 1e-6) into Xs; all of a
  //      thread's rows are loaded before any is normalised (one round trip)
  {
    constexpr int GL = C / 8 < 64 ? C / 8 : 64, RPP = 256 / GL, NV = C / 8 / GL;
    constexpr int NR = (G::T1P + RPP - 1) / RPP;
    const int gl = tid % GL;
    float4 lg[NV][2], lb[NV][2];
#pragma unroll
    for (int nv = 0; nv < NV; ++nv) {
      const int c = 8 * (gl + nv * GL);
      lg[nv][0] = *reinterpret_cast<const float4*>(a.lnw + c);
      lg[nv][1] = *reinterpret_cast<const float4*>(a.lnw + c + 4);
      lb[nv][0] = *reinterpret_cast<const float4*>(a.lnb + c);
      lb[nv][1] = *reinterpret_cast<const float4*>(a.lnb + c + 4);
    }
    uint4 raw[NR][NV];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int e = r * RPP + tid / GL;
      const int yy = y0 + e / G::EW - 1, xx = x0 + e % G::EW - 1;
      const bool in = e < G::T1 && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const long p = ((long)b * H + yy) * W + xx;
#pragma unroll
      for (int nv = 0; nv < NV; ++nv)
        raw[r][nv] = in ? *reinterpret_cast<const uint4*>(x + p * C + 8 * (gl + nv * GL)) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int e = r * RPP + tid / GL;
      const int ey = e / G::EW, ex = e % G::EW;
      const int yy = y0 + ey - 1, xx = x0 + ex - 1;
      const bool in = e < G::T1 && yy >= 0 && yy < H && xx >= 0 && xx < W;
      float v[NV][8];
      float s = 0.f;
#pragma unroll
      for (int nv = 0; nv < NV; ++nv) {
        unpack8w<T>(raw[r][nv], v[nv]);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[nv][j];
      }
      const float mu = group_sum<GL>(s) / C;
      float q = 0.f;
#pragma unroll
      for (int nv = 0; nv < NV; ++nv)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = in ? v[nv][j] - mu : 0.f;
          q += d * d;
        }
      const float rs = rsqrtf(group_sum<GL>(q) / C + a.eps);
      if (e < G::T1P) {
#pragma unroll
        for (int nv = 0; nv < NV; ++nv) {
          const float gw[8] = {lg[nv][0].x, lg[nv][0].y, lg[nv][0].z, lg[nv][0].w,
                               lg[nv][1].x, lg[nv][1].y, lg[nv][1].z, lg[nv][1].w};
          const float bw[8] = {lb[nv][0].x, lb[nv][0].y, lb[nv][0].z, lb[nv][0].w,
                               lb[nv][1].x, lb[nv][1].y, lb[nv][1].z, lb[nv][1].w};
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = in ? (v[nv][j] - mu) * rs * gw[j] + bw[j] : 0.f;
          st8<T>(Xs + e * G::XP + 8 * (gl + nv * GL), o);
        }
        if (in && ey >= 1 && ey <= TH && ex >= 1 && ex <= TW) {
          const long p = ((long)b * H + yy) * W + xx;
          if (gl == 0) {
            a.mean[p] = mu;
            a.rstd[p] = rs;
          }
          if (a.xn) {
#pragma unroll
            for (int nv = 0; nv < NV; ++nv)
              *reinterpret_cast<uint4*>(static_cast<T*>(a.xn) + p * C + 8 * (gl + nv * GL)) =
                  *reinterpret_cast<const uint4*>(Xs + e * G::XP + 8 * (gl + nv * GL));
          }
        }
      }
    }
  }
  __syncthreads();

  float4_t acc[G::CB2][G::RB2];  // this wave's partial out^T over its chunks
#pragma unroll
  for (int i = 0; i < G::CB2; ++i)
#pragma unroll
    for (int r = 0; r < G::RB2; ++r) acc[i][r] = float4_t{0.f, 0.f, 0.f, 0.f};

  const int nch = R / HC;
  // the next chunk's taps (+ W1 fragments when they are few) are loaded into registers under this
  // chunk's depthwise / GELU phase; the chunk's W2 fragments under its fc1 phase
  constexpr int NTP = (G::PS + 63) / 64;
  constexpr bool PREW1 = G::RB1 * G::KS1 <= 4;
  float tp[NTP];
  bf16x8_t wpf[PREW1 ? G::RB1 : 1][PREW1 ? G::KS1 : 1];
  auto load_taps = [&](int c0) {  // unconditional loads (clamped index): no branch for the wait to settle in
#pragma unroll
    for (int k = 0; k < NTP; ++k) {
      const int i = min(lane + 64 * k, G::PS - 1);
      const int tap = i / HC, j = i % HC;
      const float wv = a.wpos[(long)(c0 + j) * 9 + min(tap, 8)];
      const float bv = a.bpos[c0 + j];
      tp[k] = tap < 9 ? wv + (tap == 4 ? 1.f : 0.f) : bv;
    }
  };
  auto load_w1 = [&](int c0) {
    if constexpr (PREW1) {
#pragma unroll
      for (int rb = 0; rb < G::RB1; ++rb)
#pragma unroll
        for (int ks = 0; ks < G::KS1; ++ks) wpf[rb][ks] = ldfrag(w1 + (long)(c0 + 16 * rb + l15) * C + 32 * ks + 8 * lq);
    }
  };
  // W2c fragments of the chunk: loaded one chunk ahead, under the previous chunk's GELU phase (when
  // the double set fits in registers: C <= 128), else at the chunk's start
  constexpr bool PREW2 = G::RB2 * G::KS2 <= 8;
  bf16x8_t wb[G::RB2][G::KS2], wbn[PREW2 ? G::RB2 : 1][PREW2 ? G::KS2 : 1];
  auto load_w2 = [&](int c0, auto& dst) {
#pragma unroll
    for (int r = 0; r < G::RB2; ++r)
#pragma unroll
      for (int ks = 0; ks < G::KS2; ++ks) dst[r][ks] = ldfrag(w2 + (long)(16 * r + l15) * R + c0 + 32 * ks + 8 * lq);
  };
  if (wave < nch) {
    load_taps(wave * HC);
    load_w1(wave * HC);
    if constexpr (PREW2) load_w2(wave * HC, wb);
  }
  for (int ch = wave; ch < nch; ch += 4) {
    const int c0 = ch * HC;
    if constexpr (!PREW2) load_w2(c0, wb);
#pragma unroll
    for (int k = 0; k < NTP; ++k)
      if (G::PS % 64 == 0 || lane + 64 * k < G::PS) Pw[lane + 64 * k] = tp[k];
    // [A] h^T[HC, T1P] = W1c[HC, C] xn^T  (+ b1; zero outside the image) -> Hw[pixel][channel]
#pragma unroll
    for (int rb = 0; rb < G::RB1; ++rb) {
      bf16x8_t wa[G::KS1];
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks)
        wa[ks] = PREW1 ? wpf[PREW1 ? rb : 0][PREW1 ? ks : 0] : ldfrag(w1 + (long)(c0 + 16 * rb + l15) * C + 32 * ks + 8 * lq);
      const float4 bias = *reinterpret_cast<const float4*>(a.b1 + c0 + 16 * rb + 4 * lq);
#pragma unroll
      for (int cb = 0; cb < G::CB1; ++cb) {
        const int e = 16 * cb + l15;
        float4_t hacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < G::KS1; ++ks) hacc = mma16<T>(wa[ks], ldfrag(Xs + e * G::XP + 32 * ks + 8 * lq), hacc);
        const int ey = e / G::EW, ex = e % G::EW;
        const int yy = y0 + ey - 1, xx = x0 + ex - 1;
        const bool in = e < G::T1 && yy >= 0 && yy < H && xx >= 0 && xx < W;
        float hv[4] = {hacc[0] + bias.x, hacc[1] + bias.y, hacc[2] + bias.z, hacc[3] + bias.w};
        if (!in) hv[0] = hv[1] = hv[2] = hv[3] = 0.f;
        st4h<T>(Hw + e * G::HP + 16 * rb + 4 * lq, hv);
      }
    }
    // wave-local hand-off: this wave's own LDS writes are complete once lgkmcnt drains
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (ch + 4 < nch) {
      load_taps(c0 + 4 * HC);
      load_w1(c0 + 4 * HC);
      if constexpr (PREW2) load_w2(c0 + 4 * HC, wbn);
    }
    // the tile's h (the centre tap) is saved first: the stores then complete under the GELU phase
    // instead of being waited on by the next chunk's first load-use (one counter covers both)
#pragma unroll
    for (int cb = 0; cb < G::CB2; ++cb) {
      const int p = 16 * cb + l15, py = p / TW, px = p % TW;
      const int yy = y0 + py, xx = x0 + px;
#pragma unroll
      for (int ks = 0; ks < G::KS2; ++ks) {
        const int cc = 32 * ks + 8 * lq;
        const uint4 u = *reinterpret_cast<const uint4*>(Hw + ((py + 1) * G::EW + px + 1) * G::HP + cc);
        if (yy < H && xx < W) *reinterpret_cast<uint4*>(hsave + (((long)b * H + yy) * W + xx) * R + c0 + cc) = u;
      }
    }
    // [B] g = GELU(DW3x3(h) + bpos + h) for (1 pixel, 8 channels) per lane = its B fragment of
    //     out^T[C, T] += W2c[C, HC] g^T
#pragma unroll
    for (int cb = 0; cb < G::CB2; ++cb) {
      const int p = 16 * cb + l15, py = p / TW, px = p % TW;
      const long pix = ((long)b * H + y0 + py) * W + x0 + px;
      const bool pin = y0 + py < H && x0 + px < W;
#pragma unroll
      for (int ks = 0; ks < G::KS2; ++ks) {
        const int cc = 32 * ks + 8 * lq;
        // DW3x3 + bias on channel pairs (v_pk_fma_f32), GELU / GELU' packed too (normal_cdf_pdf2)
        float2_t hp2[4];
        {
          const float4 p0 = *reinterpret_cast<const float4*>(Pw + 9 * HC + cc);
          const float4 p1 = *reinterpret_cast<const float4*>(Pw + 9 * HC + cc + 4);
          hp2[0] = float2_t{p0.x, p0.y}; hp2[1] = float2_t{p0.z, p0.w};
          hp2[2] = float2_t{p1.x, p1.y}; hp2[3] = float2_t{p1.z, p1.w};
        }
        const T* hb = Hw + (py * G::EW + px) * G::HP + cc;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const uint4 u = *reinterpret_cast<const uint4*>(hb + ((tap / 3) * G::EW + tap % 3) * G::HP);
          float hv[8];
          unpack8w<T>(u, hv);
          const float4 q0 = *reinterpret_cast<const float4*>(Pw + tap * HC + cc);
          const float4 q1 = *reinterpret_cast<const float4*>(Pw + tap * HC + cc + 4);
          const float2_t wv[4] = {float2_t{q0.x, q0.y}, float2_t{q0.z, q0.w}, float2_t{q1.x, q1.y},
                                  float2_t{q1.z, q1.w}};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            hp2[j] = __builtin_elementwise_fma(wv[j], float2_t{hv[2 * j], hv[2 * j + 1]}, hp2[j]);
        }
        float g[8];
        if constexpr (SAVEG) {  // GELU and GELU' from one erf, both stored for the op-level backward
          float gd[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float2_t cdf, pdf;
            normal_cdf_pdf2(hp2[j], cdf, pdf);
            const float2_t gg = hp2[j] * cdf, dd = __builtin_elementwise_fma(hp2[j], pdf, cdf);
            g[2 * j] = gg.x; g[2 * j + 1] = gg.y;
            gd[2 * j] = dd.x; gd[2 * j + 1] = dd.y;
          }
          if (pin) {
            st8<T>(static_cast<T*>(a.gout) + pix * R + c0 + cc, g);
            st8<T>(static_cast<T*>(a.gdout) + pix * R + c0 + cc, gd);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float2_t cdf, pdf;
            normal_cdf_pdf2(hp2[j], cdf, pdf);
            const float2_t gg = hp2[j] * cdf;
            g[2 * j] = gg.x; g[2 * j + 1] = gg.y;
          }
        }
        const bf16x8_t gf = pack16x8<T>(g);
#pragma unroll
        for (int r = 0; r < G::RB2; ++r) acc[cb][r] = mma16<T>(wb[r][ks], gf, acc[cb][r]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next chunk's phase A rewrites Hw / Pw: this wave's reads of them must have completed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (PREW2) {
      if (ch + 4 < nch) {
#pragma unroll
        for (int r = 0; r < G::RB2; ++r)
#pragma unroll
          for (int ks = 0; ks < G::KS2; ++ks) wb[r][ks] = wbn[r < G::RB2 ? r : 0][ks];
      }
    }
  }

  // ---- fixed-order sum of the 4 partials: (w0 + w2) + (w1 + w3) in LDS (the body buffers are dead)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // 2 x [T * C] floats, element (cb, r, lane, j)
  auto slot = [&](int buf, int cb, int r, int j) { return buf * G::RED + ((cb * G::RB2 + r) * 4 + j) * 64 + lane; };
  if (wave >= 2) {
#pragma unroll
    for (int cb = 0; cb < G::CB2; ++cb)
#pragma unroll
      for (int r = 0; r < G::RB2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[slot(wave - 2, cb, r, j)] = acc[cb][r][j];
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int cb = 0; cb < G::CB2; ++cb)
#pragma unroll
      for (int r = 0; r < G::RB2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[cb][r][j] += red[slot(wave, cb, r, j)];
  }
  __syncthreads();
  if (wave == 1) {
#pragma unroll
    for (int cb = 0; cb < G::CB2; ++cb)
#pragma unroll
      for (int r = 0; r < G::RB2; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[slot(0, cb, r, j)] = acc[cb][r][j];
  }
  __syncthreads();
  if (wave != 0) return;
  // ---- epilogue (wave 0): f = acc + b2; out = x + rowscale * ls * f   (4 channels x 1 pixel per block)
  T* __restrict__ out = static_cast<T*>(a.out);
  T* __restrict__ fo = static_cast<T*>(a.f);
#pragma unroll
  for (int cb = 0; cb < G::CB2; ++cb) {
    const int p = 16 * cb + l15, py = p / TW, px = p % TW;
    const int yy = y0 + py, xx = x0 + px;
    const bool in = yy < H && xx < W;
    const long pg = ((long)b * H + (in ? yy : 0)) * W + (in ? xx : 0);
    const float rsc = a.rowscale ? a.rowscale[pg / a.rps] : 1.f;
#pragma unroll
    for (int r = 0; r < G::RB2; ++r) {
      const int c = 16 * r + 4 * lq;
      const float4 bb = *reinterpret_cast<const float4*>(a.b2 + c);
      const float4 ll = *reinterpret_cast<const float4*>(a.ls + c);
      float v[4] = {acc[cb][r][0] + red[slot(0, cb, r, 0)] + bb.x, acc[cb][r][1] + red[slot(0, cb, r, 1)] + bb.y,
                    acc[cb][r][2] + red[slot(0, cb, r, 2)] + bb.z, acc[cb][r][3] + red[slot(0, cb, r, 3)] + bb.w};
      if (!in) continue;
      float xv[4];
      ld4h<T>(x + pg * C + c, xv);
      st4h<T>(fo + pg * C + c, v);
      const float lv[4] = {ll.x, ll.y, ll.z, ll.w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = xv[j] + lv[j] * rsc * v[j];
      st4h<T>(out + pg * C + c, o);
    }
  }
}

// ============================================================================ backward (hidden part)
struct FfnBwdArgs {
  int B, H, W, R;
  int tiles_x, tiles_y, ntiles;
  int nstrip, tiles_per_strip;
  const void* h;   // [P][R] saved by the forward
  const void* df;  // [P][C] gradient of f (dout * rowscale * ls)
  const void* w2;  // [C][R]
  const float* wpos;
  const float* bpos;
  void* dh;          // [P][R]
  float* part_w2;    // [nstrip][C * R]   dW2[c][r]
  float* part_b2;    // [nstrip][C]
};


// 16-byte piece p of image row r sits at position p ^ swz(r) of that row
template <int NPR> DFM_INLINE int swz(int r) {
  if constexpr (NPR >= 8) return r & 7;
  else if constexpr (NPR == 4) return (r >> 2) & 3;
  else return 0;
}
// element offset of (row, element e) in an unpadded swizzled image of NPR 16-byte pieces per row
template <int NPR> DFM_INLINE int sw_off(int row, int e) {
  return row * NPR * 8 + (((e >> 3) ^ swz<NPR>(row)) << 3) + (e & 7);
}
// MFMA fragment, K along the rows of a swizzled image (row(k): the image row of k)
template <int NPR, typename RowF>
DFM_INLINE bf16x8_t tr_frag_sw(const bf16_t* img, int k0, int n0, int lane, RowF rowf) {
  typedef __attribute__((address_space(3))) short4_t lds_s4;
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int k = k0 + 8 * (lane >> 4) + q;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + sw_off<NPR>(rowf(k), n0 + 4 * p)));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + sw_off<NPR>(rowf(k + 4), n0 + 4 * p)));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  const short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, s);
}

// ============================================================================ backward, dhpre pass
// ffn_dhpre_kernel: one workgroup per (strip of tiles, hidden chunk); per tile (8 x 8; 4 x 8 at C = 256):
//   [A] dg^T = W2c^T df^T on the tile (MFMA; W2c^T in registers for the strip)
//   [B] hpre = DW3x3(h) + bpos + h from h on tile + 1 halo (LDS), GELU / GELU' from one erf,
//       dhpre = dg GELU'(hpre) -> HBM (16-bit, as the op-level chain stores it); g -> LDS
//   [D] dW2^T += g^T df (MFMA, K = pixels, ds_read_b64_tr_b16), accumulated over the strip
// h and df of the NEXT tile are DMA'd into double-buffered LDS images while this tile is computed.
// The depthwise input / weight gradients (dfm_dwconv_bwd) and the fc1 GEMMs follow in
// dfm_convffn_bwd. No halo pixel's GELU is recomputed.
template <int C, int HC, int TH_, int TW_>
struct DhGeom {
  static constexpr int TH = TH_, TW = TW_, T = TH * TW;
  static constexpr int EW1 = TW + 2, T1 = (TH + 2) * EW1;
  static constexpr int RB = HC / 16, CBT = T / 16, KS1 = C / 32;
  static constexpr int NPAIR = (CBT * RB + 3) / 4;  // (row block, column block) pairs per wave in [A] / [B]
  static constexpr int CB3 = C / 16, KS3 = T / 32;
  static constexpr int NCB3 = (CB3 * RB + 3) / 4;
  static constexpr int HP = HC + 8, HSL = HP / 8, PC = C / 8;
  static constexpr int NSH = T1 * HSL, NSD = T * PC;  // DMA slots per tile
  static constexpr int HS = T1 * HP, DS = T * C, GS = T * HP;  // elements
  static constexpr size_t LDS = (size_t)(2 * HS + 2 * DS + GS) * 2 + (size_t)(10 * HC) * 4;
  static_assert(HC % 32 == 0 && C % 32 == 0 && 4 % RB == 0 && (CBT * RB) % 4 == 0, "geometry");
};

// zero page for LDS-DMA slots outside the image: 64 x 16 bytes indexed by lane, so the requests spread
// over L2 channels instead of all hitting one line
__device__ __attribute__((aligned(16))) const unsigned int g_ffn_zero16[256] = {};

template <typename T, int C, int HC, int TH_, int TW_>
__global__ __launch_bounds__(256, 2) void ffn_dhpre_kernel(FfnBwdArgs a) {
  using G = DhGeom<C, HC, TH_, TW_>;
  constexpr int TH = G::TH, TW = G::TW, HP = G::HP;
  extern __shared__ __align__(16) unsigned char smem[];
  bf16_t* Hs = reinterpret_cast<bf16_t*>(smem);  // 2 x [T1][HP]  h chunk, tile + 1 halo (padded rows)
  bf16_t* Ds = Hs + 2 * G::HS;                     // 2 x [T][C]    df of the tile (swizzled pieces)
  bf16_t* Gs = Ds + 2 * G::DS;                     // [T][HP]       g of the tile
  float* Ps = reinterpret_cast<float*>(Gs + G::GS);  // [10][HC] taps (identity in the centre) + bias
  float* red = reinterpret_cast<float*>(smem);       // end of strip only
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, lq = lane >> 4;
  const int H = a.H, W = a.W, R = a.R;
  const int nch = R / HC;
  const int xcd = blockIdx.x & 7, j8 = blockIdx.x >> 3;
  const int chunk = j8 % nch;
  const int strip = (j8 / nch) * 8 + xcd;
  if (strip >= a.nstrip) return;
  const int c0 = chunk * HC;
  const T* __restrict__ hg = static_cast<const T*>(a.h);
  const T* __restrict__ dfg = static_cast<const T*>(a.df);
  const T* __restrict__ w2 = static_cast<const T*>(a.w2);
  T* __restrict__ dhp_g = static_cast<T*>(a.dh);  // dhpre out
  const void* zero = (const void*)g_ffn_zero16;

  for (int i = tid; i < 10 * HC; i += 256) {
    const int tap = i / HC, j = i % HC;
    Ps[i] = tap < 9 ? a.wpos[(long)(c0 + j) * 9 + tap] + (tap == 4 ? 1.f : 0.f) : a.bpos[c0 + j];
  }
  const int rb = wave % G::RB;
  const int chl = 16 * rb + 4 * lq;  // the lane's 4 hidden channels (within the chunk) in [A] / [B]
  bf16x8_t wa[G::KS1];  // W2c^T[HC, C] as A fragments: row = hidden channel 16 rb + l15, k = c
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks) {
    typedef __attribute__((ext_vector_type(8))) unsigned short us8;
    us8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_bit_cast(unsigned short, w2[(long)(32 * ks + 8 * lq + j) * R + c0 + 16 * rb + l15]);
    wa[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
  float4_t aw2[G::NCB3];
#pragma unroll
  for (int i = 0; i < G::NCB3; ++i) aw2[i] = float4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int RS2 = 256 / C;
  float db2 = 0.f;

  const int t_begin = strip * a.tiles_per_strip;
  const int t_end = min(a.ntiles, t_begin + a.tiles_per_strip);
  auto tile_xy = [&](int tile, int& b, int& y0, int& x0) {
    const int tx = tile % a.tiles_x, r = tile / a.tiles_x;
    x0 = tx * TW;
    y0 = (r % a.tiles_y) * TH;
    b = r / a.tiles_y;
  };
  auto issue = [&](int tile, int buf) {
    int b, y0, x0;
    tile_xy(tile, b, y0, x0);
    int ln = lane;
    asm volatile("" : "+v"(ln));  // opaque: the per-lane address math is redone here, not kept live
    unsigned char* hbase = smem + buf * G::HS * 2;
    for (int wi = wave; wi * 64 < G::NSH; wi += 4) {
      const int q = wi * 64 + ln;
      if (q < G::NSH) {
        const int row = q / G::HSL, slot = q - row * G::HSL;
        const int yy = y0 + row / G::EW1 - 1, xx = x0 + row % G::EW1 - 1;
        const void* src = static_cast<const unsigned char*>(zero) + 16 * ln;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)  // a pad slot re-reads the pixel's first piece
          src = hg + (((long)b * H + yy) * W + xx) * R + c0 + 8 * (slot < HC / 8 ? slot : 0);
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(hbase + wi * 1024), 16, 0, 0);
      }
    }
    unsigned char* dbase = smem + (2 * G::HS + buf * G::DS) * 2;
    for (int wi = wave; wi * 64 < G::NSD; wi += 4) {
      const int q = wi * 64 + ln;
      if (q < G::NSD) {
        const int row = q / G::PC, pos = q - row * G::PC, piece = pos ^ swz<G::PC>(row);
        const int yy = y0 + row / TW, xx = x0 + row % TW;
        const void* src = static_cast<const unsigned char*>(zero) + 16 * ln;
        if (yy < H && xx < W) src = dfg + (((long)b * H + yy) * W + xx) * C + 8 * piece;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(dbase + wi * 1024), 16, 0, 0);
      }
    }
  };

  if (t_begin < t_end) issue(t_begin, 0);
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int cur = (tile - t_begin) & 1;
    int b, y0, x0;
    tile_xy(tile, b, y0, x0);
    const bf16_t* Hc = Hs + cur * G::HS;
    const bf16_t* Dc = Ds + cur * G::DS;
    __builtin_amdgcn_s_waitcnt(0);  // this tile's DMAs (and everything older)
    __builtin_amdgcn_s_barrier();
    if (tile + 1 < t_end) issue(tile + 1, cur ^ 1);  // in flight under this tile
    // ---- [A] + [B], one (row block, column block) pair at a time
#pragma unroll 1
    for (int i = 0; i < G::NPAIR; ++i) {
      const int cb = wave / G::RB + i * (4 / G::RB);
      const int pi = 16 * cb + l15, py = pi / TW, px = pi % TW;  // tile pixel of this lane
      float4_t dg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) dg = mma16<T>(wa[ks], ldfrag(Dc + sw_off<G::PC>(pi, 32 * ks + 8 * lq)), dg);
      const bf16_t* hb = Hc + (py * G::EW1 + px) * HP + chl;  // tap (0, 0); tap t at + off(t)
      float hp[4];
      {
        const float4 bp = *reinterpret_cast<const float4*>(Ps + 9 * HC + chl);
        hp[0] = bp.x; hp[1] = bp.y; hp[2] = bp.z; hp[3] = bp.w;
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        float hv[4];
        ld4h<T>(reinterpret_cast<const T*>(hb + ((tap / 3) * G::EW1 + tap % 3) * HP), hv);
        const float4 wt = *reinterpret_cast<const float4*>(Ps + tap * HC + chl);
        hp[0] = fmaf(wt.x, hv[0], hp[0]);
        hp[1] = fmaf(wt.y, hv[1], hp[1]);
        hp[2] = fmaf(wt.z, hv[2], hp[2]);
        hp[3] = fmaf(wt.w, hv[3], hp[3]);
      }
      float g[4], dhp[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float cdf, pdf;
        normal_cdf_pdf(hp[j], cdf, pdf);
        g[j] = hp[j] * cdf;
        dhp[j] = dg[j] * fmaf(hp[j], pdf, cdf);
      }
      const bool in = y0 + py < H && x0 + px < W;
      if (in) st4h<T>(dhp_g + (((long)b * H + y0 + py) * W + x0 + px) * R + c0 + chl, dhp);
      else g[0] = g[1] = g[2] = g[3] = 0.f;
      st4h<T>(reinterpret_cast<T*>(Gs + pi * HP + chl), g);
    }
    if (chunk == 0) {  // db2 = sum df over the strip
      const int c = tid % C;
      for (int pi = tid / C; pi < G::T; pi += RS2)
        db2 += Num<T>::to_f(reinterpret_cast<const T*>(Dc)[sw_off<G::PC>(pi, c)]);
    }
    lds_barrier();
    // ---- [D] dW2^T[HC, C] += g^T df (K = tile pixels)
    auto id_row = [](int k) { return k; };
#pragma unroll
    for (int i = 0; i < G::NCB3; ++i) {
      const int cb = wave / G::RB + i * (4 / G::RB);
      if ((G::CB3 * G::RB) % 4 != 0 && cb >= G::CB3) break;
#pragma unroll
      for (int ks = 0; ks < G::KS3; ++ks)
        aw2[i] = mma16<T>(tr_frag(Gs, HP, 32 * ks, 16 * rb, lane), tr_frag_sw<G::PC>(Dc, 32 * ks, 16 * cb, lane, id_row),
                          aw2[i]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // ---- per-strip partials
  const long S = strip;
#pragma unroll
  for (int i = 0; i < G::NCB3; ++i) {
    const int cb = wave / G::RB + i * (4 / G::RB);
    if ((G::CB3 * G::RB) % 4 != 0 && cb >= G::CB3) break;
    const int c = 16 * cb + l15;
    *reinterpret_cast<float4*>(a.part_w2 + S * C * R + (long)c * R + c0 + chl) =
        make_float4(aw2[i][0], aw2[i][1], aw2[i][2], aw2[i][3]);
  }
  if (chunk == 0) {
    red[tid] = db2;
    __syncthreads();
    if (tid < C) {
      float s = 0.f;
      for (int t2 = tid; t2 < 256; t2 += C) s += red[t2];
      a.part_b2[S * C + tid] = s;
    }
  }
}

// ============================================================================ host side
template <int C> struct FfnCfg;  // hidden chunk and tile shapes per channel count
template <> struct FfnCfg<32> {
  static constexpr int FHC = 32, FTH = 8, FTW = 16, BHC = 32, DTH = 8, DTW = 8;
};
template <> struct FfnCfg<64> {
  static constexpr int FHC = 32, FTH = 8, FTW = 8, BHC = 32, DTH = 8, DTW = 8;
};
template <> struct FfnCfg<128> {
  static constexpr int FHC = 32, FTH = 4, FTW = 8, BHC = 32, DTH = 8, DTW = 8;
};
template <> struct FfnCfg<256> {
  static constexpr int FHC = 32, FTH = 4, FTW = 4, BHC = 32, DTH = 4, DTW = 8;
};

bool ffn_shape_ok(int C, int R) {
  return (C == 32 || C == 64 || C == 128 || C == 256) && R % 128 == 0;
}

template <typename T, int C, int TH, int TW>
int ffn_fwd_launch_t(const DfmConvFFNDesc* d, FfnFwdArgs a, hipStream_t s) {
  using Cf = FfnCfg<C>;
  using G = FwdGeom<C, Cf::FHC, TH, TW>;
  auto kern = a.gout ? ffn_fwd_kernel<T, C, Cf::FHC, TH, TW, true> : ffn_fwd_kernel<T, C, Cf::FHC, TH, TW, false>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ffn_fwd_kernel<T, C, Cf::FHC, TH, TW, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
    (void)hipFuncSetAttribute((const void*)ffn_fwd_kernel<T, C, Cf::FHC, TH, TW, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
    attr = true;
  }
  a.tiles_x = (int)cdiv(d->W, G::TW);
  a.tiles_y = (int)cdiv(d->H, G::TH);
  const long grid = (long)d->B * a.tiles_x * a.tiles_y;
  DFM_LAUNCH(kern, dim3((unsigned)grid), dim3(256), G::LDS, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, int C>
int ffn_fwd_launch(const DfmConvFFNDesc* d, FfnFwdArgs a, hipStream_t s) {
  using Cf = FfnCfg<C>;
  // the 8 x 16 tile at C = 32 spills with the GELU outputs: 8 x 8 then (half-size tiles everywhere
  // measured 467.8 / 468.4 vs 468.5 / 469.9 images/s)
  if constexpr (C == 32) {
    if (a.gout) return ffn_fwd_launch_t<T, C, 8, 8>(d, a, s);
  }
  return ffn_fwd_launch_t<T, C, Cf::FTH, Cf::FTW>(d, a, s);
}

struct BwdPlan {
  int tiles_x, tiles_y, ntiles, nstrip, tps, nch;
  size_t lds;
};

template <int C>
BwdPlan ffn_dh_plan(const DfmConvFFNDesc* d) {
  using Cf = FfnCfg<C>;
  using G = DhGeom<C, Cf::BHC, Cf::DTH, Cf::DTW>;
  BwdPlan p;
  p.tiles_x = (int)cdiv(d->W, G::TW);
  p.tiles_y = (int)cdiv(d->H, G::TH);
  p.ntiles = d->B * p.tiles_x * p.tiles_y;
  p.nch = d->hidden / Cf::BHC;
  // about 4 workgroups per CU over (strip, chunk): the tile loop's DMA waits overlap across them
  int ns = (1024 + p.nch - 1) / p.nch;
  ns = std::max(8, std::min((ns + 7) / 8 * 8, (p.ntiles + 7) / 8 * 8));
  p.tps = (p.ntiles + ns - 1) / ns;
  p.nstrip = (p.ntiles + p.tps - 1) / p.tps;
  p.lds = G::LDS;
  return p;
}

BwdPlan dh_plan(const DfmConvFFNDesc* d) {
  switch (d->C) {
    case 32: return ffn_dh_plan<32>(d);
    case 64: return ffn_dh_plan<64>(d);
    case 128: return ffn_dh_plan<128>(d);
    default: return ffn_dh_plan<256>(d);
  }
}

template <typename T, int C>
int ffn_dh_launch(const BwdPlan& p, FfnBwdArgs a, hipStream_t s) {
  using Cf = FfnCfg<C>;
  auto kern = ffn_dhpre_kernel<T, C, Cf::BHC, Cf::DTH, Cf::DTW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds);
    attr = true;
  }
  a.tiles_x = p.tiles_x;
  a.tiles_y = p.tiles_y;
  a.ntiles = p.ntiles;
  a.nstrip = p.nstrip;
  a.tiles_per_strip = p.tps;
  const long grid = (long)(p.nstrip + 7) / 8 * 8 * p.nch;
  DFM_LAUNCH(kern, dim3((unsigned)grid), dim3(256), p.lds, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

#define FFN_C_SWITCH(C, FN, ...)            \
  [&]() -> int {                            \
    switch (C) {                            \
      case 32: return FN<T, 32>(__VA_ARGS__);  \
      case 64: return FN<T, 64>(__VA_ARGS__);  \
      case 128: return FN<T, 128>(__VA_ARGS__); \
      default: return FN<T, 256>(__VA_ARGS__); \
    }                                       \
  }()

struct BwdWs {
  size_t df, dh, du, pw2, pb2, res, ln, gemm, dhp, dw, wg, total;
};

DfmGemmDesc du_desc(const DfmConvFFNDesc* d) {
  // du[P, C] = dh[P, R] W1[R, C]   (nn.Linear fc1 input gradient: A k-contiguous, B row-contiguous)
  DfmGemmDesc g{};
  const long P = (long)d->B * d->H * d->W;
  g.M = (int)P;
  g.N = d->C;
  g.K = d->hidden;
  g.batch = 1;
  g.a_kcontig = 1;
  g.b_kcontig = 0;
  g.lda = d->hidden;
  g.ldb = d->C;
  g.ldc = d->C;
  g.alpha = 1.f;
  g.beta = 0.f;
  g.rows_per_scale = 1;
  return g;
}

DfmGemmDesc w1_desc(const DfmConvFFNDesc* d) {
  // dW1[R, C] = dh^T xn (+ db1 = column sums of dh): K = pixels, both operands row-contiguous
  DfmGemmDesc g{};
  const long P = (long)d->B * d->H * d->W;
  g.M = d->hidden;
  g.N = d->C;
  g.K = (int)P;
  g.batch = 1;
  g.a_kcontig = 0;
  g.b_kcontig = 0;
  g.lda = d->hidden;
  g.ldb = d->C;
  g.ldc = d->C;
  g.alpha = 1.f;
  g.beta = 0.f;
  g.c_f32 = 1;
  g.rows_per_scale = 1;
  return g;
}

BwdWs bwd_ws(int dtype, const DfmConvFFNDesc* d) {
  const size_t es = dtype == DFM_F32 ? 4 : 2;
  const long P = (long)d->B * d->H * d->W;
  BwdWs w{};
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  w.df = al(es * P * d->C);
  w.dh = al(es * P * d->hidden);
  w.du = al(es * P * d->C);
  w.res = al(dfm_residual_bwd_workspace(P, d->C));
  w.ln = al(dfm_layernorm_bwd_workspace(P, d->C));
  DfmGemmDesc g = du_desc(d);
  w.gemm = al(dfm_gemm_workspace_size(&g));
  // dhpre (+ dW2 / db2 strip partials), depthwise weight-gradient partials, fc1 weight-gradient GEMM
  const BwdPlan q = dh_plan(d);
  w.pw2 = al((size_t)q.nstrip * d->C * d->hidden * 4);
  w.pb2 = al((size_t)q.nstrip * d->C * 4);
  w.dhp = al(es * P * d->hidden);
  w.dw = al(dfm_dwconv_bwd_weight_workspace(d->B, d->H, d->W, d->hidden, 3));
  DfmGemmDesc gw = w1_desc(d);
  gw.colsum = reinterpret_cast<float*>(16);  // sized with its bias-gradient column (only nullness is read)
  w.wg = al(dfm_gemm_workspace_size(&gw));
  w.total = w.df + w.dh + w.du + w.pw2 + w.pb2 + w.res + w.ln + w.gemm + w.dhp + w.dw + w.wg;
  return w;
}

}  // namespace

extern "C" int dfm_convffn_supported(int dtype, const DfmConvFFNDesc* d) {
  return d && (dtype == DFM_BF16 || dtype == DFM_F16) && d->B > 0 && d->H > 0 && d->W > 0 &&
         ffn_shape_ok(d->C, d->hidden);
}

extern "C" int dfm_convffn_fwd(int dtype, const DfmConvFFNDesc* d, const void* x, const float* ln_w,
                               const float* ln_b, const void* w1, const float* b1, const float* wpos,
                               const float* bpos, const void* w2, const float* b2, const float* ls,
                               const float* rowscale, void* out, void* f, void* h, void* xn, float* mean,
                               float* rstd, void* gelu_out, void* gelu_grad, dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, d), "dfm_convffn_fwd: unsupported dtype %d / shape (C %d, hidden %d)",
                dtype, d ? d->C : -1, d ? d->hidden : -1);
  DFM_CHECK_ARG(x && ln_w && ln_b && w1 && b1 && wpos && bpos && w2 && b2 && ls && out && f && h && mean && rstd,
                "dfm_convffn_fwd: null argument");
  DFM_CHECK_ARG(!gelu_out == !gelu_grad, "dfm_convffn_fwd: gelu_out and gelu_grad go together");
  FfnFwdArgs a{};
  a.B = d->B; a.H = d->H; a.W = d->W; a.R = d->hidden;
  a.eps = d->ln_eps;
  a.rps = (long)d->H * d->W;
  a.x = x; a.lnw = ln_w; a.lnb = ln_b; a.w1 = w1; a.b1 = b1; a.wpos = wpos; a.bpos = bpos;
  a.w2 = w2; a.b2 = b2; a.ls = ls; a.rowscale = rowscale;
  a.out = out; a.f = f; a.h = h; a.xn = xn; a.mean = mean; a.rstd = rstd;
  a.gout = gelu_out; a.gdout = gelu_grad;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) {
    using T = bf16_t;
    return FFN_C_SWITCH(d->C, ffn_fwd_launch, d, a, s);
  }
  using T = f16_t;
  return FFN_C_SWITCH(d->C, ffn_fwd_launch, d, a, s);
}

extern "C" size_t dfm_convffn_bwd_workspace_size(int dtype, const DfmConvFFNDesc* d) {
  if (!dfm_convffn_supported(dtype, d)) return 0;
  return bwd_ws(dtype, d).total;
}

extern "C" int dfm_convffn_bwd(int dtype, const DfmConvFFNDesc* d, const void* dout, const void* x, const void* h,
                               const void* xn, const void* f, const float* mean, const float* rstd,
                               const float* ln_w, const float* ln_b, const void* w1, const float* wpos,
                               const float* bpos, const void* w2, const float* ls, const float* rowscale, void* dx,
                               float* dln_w, float* dln_b, float* dw1, float* db1, float* dwpos, float* dbpos,
                               float* dw2, float* db2, float* dls, void* workspace, size_t workspace_bytes,
                               dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, d), "dfm_convffn_bwd: unsupported dtype %d / shape (C %d, hidden %d)",
                dtype, d ? d->C : -1, d ? d->hidden : -1);
  DFM_CHECK_ARG(dout && x && h && xn && f && mean && rstd && ln_w && ln_b && w1 && wpos && bpos && w2 && ls && dx &&
                    dln_w && dln_b && dw1 && db1 && dwpos && dbpos && dw2 && db2 && dls && workspace,
                "dfm_convffn_bwd: null argument");
  const BwdWs w = bwd_ws(dtype, d);
  DFM_CHECK_ARG(workspace_bytes >= w.total, "dfm_convffn_bwd: workspace %zu < %zu bytes", workspace_bytes, w.total);
  hipStream_t s = (hipStream_t)stream;
  const long P = (long)d->B * d->H * d->W;
  const int C = d->C, R = d->hidden;
  char* ws = (char*)workspace;
  void* df = ws; ws += w.df;
  void* dh = ws; ws += w.dh;
  void* du = ws; ws += w.du;
  float* pw2 = (float*)ws; ws += w.pw2;
  float* pb2 = (float*)ws; ws += w.pb2;
  void* wres = ws; ws += w.res;
  void* wln = ws; ws += w.ln;
  void* wgemm = ws; ws += w.gemm;
  void* dhp = ws; ws += w.dhp;
  void* wdw = ws; ws += w.dw;
  void* wwg = ws;
  DfmPartialSum sums[12];
  int ns = 0;
  // residual / layer-scale backward: df = dout * ls * rowscale, dls = sum dout * f * rowscale
  int rc = dfm_residual_bwd(dtype, P, C, dout, C, f, C, ls, rowscale, (long)d->H * d->W, df, C, dls, wres, &sums[ns],
                            stream);
  if (rc != DFM_OK) return rc;
  if (sums[ns].part) ++ns;
  FfnBwdArgs a{};
  a.B = d->B; a.H = d->H; a.W = d->W; a.R = R;
  a.h = h; a.df = df; a.w2 = w2;
  a.wpos = wpos; a.bpos = bpos;
  a.part_w2 = pw2; a.part_b2 = pb2;
  // dhpre (+ dW2, db2) -> depthwise input / weight gradients -> fc1 weight gradient (+ db1)
  const BwdPlan p = dh_plan(d);
  a.dh = dhp;
  if (dtype == DFM_BF16) {
    using T = bf16_t;
    rc = FFN_C_SWITCH(C, ffn_dh_launch, p, a, s);
  } else {
    using T = f16_t;
    rc = FFN_C_SWITCH(C, ffn_dh_launch, p, a, s);
  }
  if (rc != DFM_OK) return rc;
  sums[ns++] = DfmPartialSum{pw2, dw2, nullptr, (long)C * R, 0, p.nstrip, 0, 0};
  sums[ns++] = DfmPartialSum{pb2, db2, nullptr, (long)C, 0, p.nstrip, 0, 0};
  rc = dfm_dwconv_bwd(dtype, d->B, d->H, d->W, R, 3, h, R, dhp, R, wpos, 1, dh, R, 0, dwpos, dbpos, wdw, &sums[ns],
                      stream);
  if (rc != DFM_OK) return rc;
  if (sums[ns].part) ++ns;
  DfmGemmDesc gw = w1_desc(d);
  gw.colsum = db1;
  gw.workspace_bytes = (long)w.wg;
  rc = dfm_gemm(dtype, &gw, dh, xn, dw1, wwg, stream);
  if (rc != DFM_OK) return rc;
  // fc1 input gradient du = dh W1, then the LayerNorm backward with the residual's dout
  DfmGemmDesc g = du_desc(d);
  g.workspace_bytes = (long)w.gemm;
  rc = dfm_gemm(dtype, &g, dh, w1, du, wgemm, stream);
  if (rc != DFM_OK) return rc;
  rc = dfm_layernorm_bwd(dtype, P, C, x, C, du, C, ln_w, mean, rstd, dout, C, dx, C, 0, dln_w, dln_b, wln, &sums[ns],
                         stream);
  if (rc != DFM_OK) return rc;
  if (sums[ns].part) ++ns;
  return dfm_partial_sum_group(ns, sums, stream);
}
