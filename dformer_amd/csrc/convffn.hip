// Fused ConvFFN for gfx950 — DFormer's MLP (models/encoders/DFormer.py:48-67) inside the Block
// residual (DFormer.py:173-179):
//
//   out = x + rowscale * ls * f,   f = fc2(GELU(DW3x3(h) + bpos + h)) + b2,   h = fc1(xn) + b1
//
// A workgroup owns a TH x 16 tile of output pixels of one image (one 16-pixel MFMA tile per tile
// row) and walks the hidden channels in chunks of HC = 32. The [P, hid] hidden activation never
// leaves the CU in the forward pass:
//   [A] fc1 on tile + 1-pixel halo: h^T = W1c xn^T (MFMA), + b1, zero outside the image -> LDS as
//       fp32 "channel planes" hs[plane = ch / 8][pixel][ch % 8] (a plane stride = 4 mod 64 dwords
//       makes the depthwise reads below bank-conflict free);
//   [B] every lane computes the depthwise 3x3 (+ bias, identity folded into the centre tap) and GELU
//       for exactly the 8 (bf16 / f16) hidden channels x 1 pixel that it must hold as the B operand of
//       the fc2 MFMA (lane l: pixel l & 15, channels 8 (l >> 4) .. + 8), so g goes from VALU registers
//       straight into v_mfma_f32_16x16x32 without an LDS round trip; out^T += W2c g^T accumulates in
//       registers over all chunks.
// The next chunk's weights are fetched into registers under [A] / [B] (and double-buffered in LDS
// where it fits two workgroups per CU).
//
// Backward (one 512-thread workgroup per CU, TH = 8): per chunk [A] recomputes h on tile + 2-pixel
// halo and dg = df W2c on tile + 1 halo (MFMA), [B] hpre = DW3(h) + bpos + h, g = GELU(hpre) (tile
// pixels -> HBM for the fc2 weight-gradient GEMM), dhpre = dg GELU'(hpre) (in LDS), [C] dh = DW3^T
// (dhpre) + dhpre on the tile straight into the B fragments of dxn^T += W1c^T dh^T (MFMA) and to HBM
// (fc1 weight-gradient GEMM); the depthwise weight / bias gradient partials of the tile ride along
// in [B]. Weights are read in their natural layouts (w1 [hid][C], w2 [C][hid]) and transposed while
// staged into LDS.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int HC = 32;  // hidden channels per chunk
constexpr int TW = 16;  // tile width = one 16-pixel MFMA tile per tile row

// ---- MFMA operand traits: 16-bit types use v_mfma_f32_16x16x32_{bf16,f16} (lane l holds A[l&15]
// [8(l>>4) .. +8], B[8(l>>4) .. +8][l&15]); float32 (the parity path) v_mfma_f32_16x16x4_f32 (lane l
// holds A[l&15][l>>4], B[l>>4][l&15]). C/D: lane l holds rows 4(l>>4) .. +4 of column l&15.
template <typename T> struct FT {
  using frag = bf16x8_t;
  static constexpr int KS = 32;
  static constexpr int PAD = 16;  // row pitch = K + 16 elements (= 16 mod 32): conflict-free b128 fragments
  static DFM_INLINE frag ld(const T* row, int k0, int lane) {
    return __builtin_bit_cast(frag, *reinterpret_cast<const uint4*>(row + k0 + 8 * (lane >> 4)));
  }
  static DFM_INLINE float4_t mma(frag a, frag b, float4_t c) { return mma16<T>(a, b, c); }
};
template <> struct FT<float> {
  using frag = float;
  static constexpr int KS = 4;
  static constexpr int PAD = 4;
  static DFM_INLINE frag ld(const float* row, int k0, int lane) { return row[k0 + (lane >> 4)]; }
  static DFM_INLINE float4_t mma(frag a, frag b, float4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// The hidden channel m (0..7) of a lane's 8 in the MFMA B-operand layout of a 32-channel chunk:
// 16-bit: 8 consecutive channels per lane quarter; float32: k-step m, channel 4 m + quarter.
template <typename T> DFM_INLINE int lane_ch(int kq, int m) { return sizeof(T) == 2 ? 8 * kq + m : 4 * m + kq; }

// 8 floats -> B fragment(s): 16-bit: one 8 x 16-bit vector; float32: element m is k-step m's operand
template <typename T> DFM_INLINE typename FT<T>::frag to_frag(const float* v, int m) {
  if constexpr (sizeof(T) == 2) return pack16x8<T>(v);
  else return v[m];
}

// fp32 channel planes: plane p holds channels 8p .. 8p + 7 of every pixel row (32 bytes per row).
// Plane stride = rows * 8 + RES floats. RES = 4: the lane groups of a ds_read_b128 in the MFMA
// operand layout (16 consecutive pixels x 4 planes) hit 16 distinct 4-bank slots. RES = 16: the
// 32-lane groups of a ds_read_b64 over (2 consecutive pixels x 16 channel pairs) hit 32 distinct
// 2-bank slots (the backward's per-channel-pair depthwise phase).
template <int ROWS, int RES = 4> struct Planes {
  static constexpr int PS = ROWS * 8 + RES;  // ROWS * 8 is a multiple of 64 (ROWS % 8 == 0)
  static constexpr int FLOATS = 4 * PS;  // HC / 8 planes
  static DFM_INLINE int at(int row, int ch) { return (ch >> 3) * PS + row * 8 + (ch & 7); }
};

// 8 consecutive floats of channels ch .. ch + 7 (ch % 8 == 0) of one plane row
DFM_INLINE void ld8p(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// The lane's 8 channels of one pixel row of a plane image (16-bit: one contiguous group; fp32: strided)
template <typename T, int ROWS>
DFM_INLINE void ld_lane8(const float* img, int row, int kq, float* v) {
  if constexpr (sizeof(T) == 2) {
    ld8p(img + Planes<ROWS>::at(row, 8 * kq), v);
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = img[Planes<ROWS>::at(row, lane_ch<T>(kq, m))];
  }
}

// 4 consecutive elements (8 bytes for 16-bit types, 16 for float32) <-> floats
template <typename T> DFM_INLINE void ld4(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = Num<T>::to_f(e[r]);
  } else {
    const float4 u = *reinterpret_cast<const float4*>(p);
    v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
  }
}
template <typename T> DFM_INLINE void st4g(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    T e[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) e[r] = Num<T>::from_f(v[r]);
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(e);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Per-chunk fp32 parameters in LDS: pb[0, HC) = b1, pb[HC, 2 HC) = bpos, pb[2 HC + t HC + ch] = tap t
// of channel ch (tap-major), with the identity of `DW3(h) + h` folded into the centre tap (t = 4).
constexpr int PB = 11 * HC;

template <typename T> DFM_INLINE void ld_lane8_par(const float* pb, int kq, float* v) {
  if constexpr (sizeof(T) == 2) {
    ld8p(pb + 8 * kq, v);
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = pb[lane_ch<T>(kq, m)];
  }
}

// Register-staged prefetch of one chunk of weights / parameters (issued under the previous chunk's
// work, stored to LDS after it). Rows beyond C are zero-filled.
//   W1c = w1[c0 .. c0 + HC][0 .. C)        -> dst1[j][c]   (pitch XP)
//   W2c = w2[0 .. C)[c0 .. c0 + HC)        -> dst2[c][j]   (pitch WP)
//   b1, bpos, wpos (+1 on the centre tap)  -> pb
template <typename T, int CT, int NT>
struct ChunkPrefetch {
  static constexpr int V = 16 / sizeof(T);                 // elements per 16-byte vector
  static constexpr int N1 = HC * CT / V, N2 = CT * HC / V;  // vectors of W1c / W2c
  static constexpr int R1 = (N1 + NT - 1) / NT, R2 = (N2 + NT - 1) / NT;
  static constexpr int NP = PB;                            // parameter floats
  static constexpr int RP = (NP + NT - 1) / NT;
  uint4 w1[R1], w2[R2];
  float par[RP];

  DFM_INLINE void load(const T* __restrict__ gw1, const T* __restrict__ gw2, const float* __restrict__ b1,
                       const float* __restrict__ bpos, const float* __restrict__ wpos, int C, int hid, int c0) {
#pragma unroll
    for (int i = 0; i < R1; ++i) {
      const int v = threadIdx.x + i * NT;
      const int j = v / (CT / V), c = (v % (CT / V)) * V;
      w1[i] = (v < N1 && c < C) ? *reinterpret_cast<const uint4*>(gw1 + (long)(c0 + j) * C + c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < R2; ++i) {
      const int v = threadIdx.x + i * NT;
      const int c = v / (HC / V), j = (v % (HC / V)) * V;
      w2[i] = (v < N2 && c < C) ? *reinterpret_cast<const uint4*>(gw2 + (long)c * hid + c0 + j) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int e = threadIdx.x + i * NT;
      float v = 0.f;
      if (e < HC) v = b1[c0 + e];
      else if (e < 2 * HC) v = bpos[c0 + e - HC];
      else if (e < NP) {
        const int t = (e - 2 * HC) / HC, ch = (e - 2 * HC) % HC;
        v = wpos[(long)(c0 + ch) * 9 + t] + (t == 4 ? 1.0f : 0.0f);
      }
      par[i] = v;
    }
  }

  template <int XP, int WP>
  DFM_INLINE void store(T* dst1, T* dst2, float* pb) const {
#pragma unroll
    for (int i = 0; i < R1; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= N1) break;
      const int j = v / (CT / V), c = (v % (CT / V)) * V;
      *reinterpret_cast<uint4*>(dst1 + j * XP + c) = w1[i];
    }
#pragma unroll
    for (int i = 0; i < R2; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= N2) break;
      const int c = v / (HC / V), j = (v % (HC / V)) * V;
      *reinterpret_cast<uint4*>(dst2 + c * WP + j) = w2[i];
    }
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int e = threadIdx.x + i * NT;
      if (e < NP) pb[e] = par[i];
    }
  }
};

// Rows x C of NHWC activations (row r of the halo image = pixel (y0 + r / rw, x0 + r % rw) of image b,
// zero outside the image or past `rows`) -> LDS with pitch XP; columns C .. CT zero-filled.
template <typename T, int CT, int XP, int NT>
DFM_INLINE void stage_halo(T* dst, const T* __restrict__ src, long ld, int rows, int rows_pad, int rw, int b, int y0,
                           int x0, int H, int W, int C) {
  constexpr int V = 16 / sizeof(T);
  constexpr int VPR = CT / V;
  for (int i = threadIdx.x; i < rows_pad * VPR; i += NT) {
    const int r = i / VPR, c = (i % VPR) * V;
    const int yy = y0 + r / rw, xx = x0 + r % rw;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < rows && c < C && yy >= 0 && yy < H && xx >= 0 && xx < W)
      v = *reinterpret_cast<const uint4*>(src + ((long)(b * H + yy) * W + xx) * ld + c);
    *reinterpret_cast<uint4*>(dst + r * XP + c) = v;
  }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not its global
// loads. __syncthreads()' fence drains vmcnt, which would wait for the next chunk's weight prefetch
// at every barrier and expose its L2 round trip once per chunk; the inline asm (memory clobber) also
// keeps the compiler from moving LDS accesses across it.
DFM_INLINE void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// XCD-aware tile order: neighbouring tiles (which share halo rows) run on one XCD's L2.
DFM_INLINE int xcd_tile(int id, int n) {
  const int xcd = id & 7, q8 = n >> 3, r8 = n & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
}

struct FfnArgs {
  int B, H, W, C, hid;
  int tiles_y, tiles_x;
  const void* xn;
  long ldxn;
  const void* x;
  long ldx;
  const void* w1;  // [hid][C]
  const float* b1;
  const float* wpos;  // [hid][9]
  const float* bpos;
  const void* w2;  // [C][hid]
  const float* b2;
  const float* ls;
  const float* rowscale;  // [B] or null
  void* out;
  long ldout;
  void* f;
  long ldf;
};

// ---------------------------------------------------------------- forward
template <typename T, int CT, int TH, bool DB>
struct FwdGeom {
  static constexpr int NT = 256, NW = 4;  // two workgroups per CU
  static constexpr int HW2 = TW + 2;
  static constexpr int NH = (TH + 2) * HW2;
  static constexpr int NHT = (NH + 15) / 16;  // 16-pixel tiles of tile + halo
  static constexpr int NHP = NHT * 16;
  static constexpr int XP = CT + FT<T>::PAD;  // xs / W1c row pitch
  static constexpr int WP = HC + FT<T>::PAD;  // W2c row pitch
  static constexpr int NB = DB ? 2 : 1;
  static constexpr size_t o_w1 = (size_t)NHP * XP * sizeof(T);
  static constexpr size_t W1B = (size_t)HC * XP * sizeof(T), W2B = (size_t)CT * WP * sizeof(T), PBB = PB * 4;
  static constexpr size_t o_w2 = o_w1 + NB * W1B;
  static constexpr size_t o_pb = o_w2 + NB * W2B;
  static constexpr size_t o_hs = o_pb + NB * PBB;
  static constexpr size_t lds = o_hs + (size_t)Planes<NHP>::FLOATS * 4;
};

template <typename T, int CT, int TH, bool DB>
__global__ __launch_bounds__(256) void convffn_fwd_kernel(FfnArgs a) {
  using G = FwdGeom<T, CT, TH, DB>;
  using F = FT<T>;
  using HP = Planes<G::NHP>;
  constexpr int NT = G::NT, NW = G::NW, XP = G::XP, WP = G::WP;
  constexpr int OT = CT / 16;           // fc2 output-channel tiles
  constexpr int PTW = 2;                // tile rows per wave (2 w, 2 w + 1)
  static_assert(TH == 2 * NW, "each wave owns two adjacent tile rows");
  constexpr int KC = CT / F::KS;        // fc1 k-steps
  constexpr int K2 = HC / F::KS;        // fc2 k-steps
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);
  float* hs = reinterpret_cast<float*>(smem + G::o_hs);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nt = a.B * a.tiles_y * a.tiles_x;
  const int tile = xcd_tile(blockIdx.x, nt);
  const int b = tile / (a.tiles_y * a.tiles_x);
  const int ty = (tile / a.tiles_x) % a.tiles_y, tx = tile % a.tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int C = a.C, hid = a.hid, H = a.H, W = a.W;
  const int px = lane & 15, kq = lane >> 4;

  ChunkPrefetch<T, CT, NT> pf;
  pf.load((const T*)a.w1, (const T*)a.w2, a.b1, a.bpos, a.wpos, C, hid, 0);
  stage_halo<T, CT, XP, NT>(xs, (const T*)a.xn, a.ldxn, G::NH, G::NHP, G::HW2, b, y0 - 1, x0 - 1, H, W, C);
  pf.template store<XP, WP>(reinterpret_cast<T*>(smem + G::o_w1), reinterpret_cast<T*>(smem + G::o_w2),
                                   reinterpret_cast<float*>(smem + G::o_pb));
  float4_t acc[PTW][OT];
#pragma unroll
  for (int i = 0; i < PTW; ++i)
#pragma unroll
    for (int o = 0; o < OT; ++o) acc[i][o] = float4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  const int nchunk = hid / HC;
  int buf = 0;
  for (int ci = 0; ci < nchunk; ++ci) {
    const T* w1s = reinterpret_cast<const T*>(smem + G::o_w1 + buf * G::W1B);
    const T* w2s = reinterpret_cast<const T*>(smem + G::o_w2 + buf * G::W2B);
    const float* pb = reinterpret_cast<const float*>(smem + G::o_pb + buf * G::PBB);
    const bool more = ci + 1 < nchunk;
    if (more) pf.load((const T*)a.w1, (const T*)a.w2, a.b1, a.bpos, a.wpos, C, hid, (ci + 1) * HC);
    // ---- [A] fc1 on tile + halo: h^T[hidden 16][pixel 16] = W1c xn^T, + b1, zero outside the image
    {
      typename F::frag aw[2][KC];
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int ks = 0; ks < KC; ++ks) aw[it][ks] = F::ld(w1s + (it * 16 + px) * XP, ks * F::KS, lane);
      float4 bb[2];
#pragma unroll
      for (int it = 0; it < 2; ++it) bb[it] = *reinterpret_cast<const float4*>(pb + it * 16 + 4 * kq);
      for (int jt = wid; jt < G::NHT; jt += NW) {
        float4_t h[2] = {float4_t{0.f, 0.f, 0.f, 0.f}, float4_t{0.f, 0.f, 0.f, 0.f}};
        const T* xrow = xs + (jt * 16 + px) * XP;
#pragma unroll
        for (int ks = 0; ks < KC; ++ks) {
          const typename F::frag xb = F::ld(xrow, ks * F::KS, lane);
#pragma unroll
          for (int it = 0; it < 2; ++it) h[it] = F::mma(aw[it][ks], xb, h[it]);
        }
        const int q = jt * 16 + px;
        const int yy = y0 - 1 + q / G::HW2, xx = x0 - 1 + q % G::HW2;
        const bool ok = q < G::NH && yy >= 0 && yy < H && xx >= 0 && xx < W;
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const float4 v = ok ? make_float4(h[it][0] + bb[it].x, h[it][1] + bb[it].y, h[it][2] + bb[it].z,
                                            h[it][3] + bb[it].w)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(hs + HP::at(q, it * 16 + 4 * kq)) = v;
        }
      }
    }
    lds_sync();  // hs complete
    // ---- [B] depthwise 3x3 (+ bias + identity) + GELU into the fc2 B fragments; out^T += W2c g^T.
    //          Wave w owns the adjacent tile rows 2w, 2w + 1: the 4 halo rows they touch are read once
    //          (12 tap positions for 2 output rows instead of 18); taps and bias sit in registers.
    {
      float wt[9][8], s0[8], s1[8];
      ld_lane8_par<T>(pb + HC, kq, s0);
#pragma unroll
      for (int t = 0; t < 9; ++t) ld_lane8_par<T>(pb + 2 * HC + t * HC, kq, wt[t]);
#pragma unroll
      for (int m = 0; m < 8; ++m) s1[m] = s0[m];
      typename F::frag a2[OT][K2];
#pragma unroll
      for (int o = 0; o < OT; ++o)
#pragma unroll
        for (int ks = 0; ks < K2; ++ks) a2[o][ks] = F::ld(w2s + (o * 16 + px) * WP, ks * F::KS, lane);
      const int pt0 = 2 * wid;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          float hv[8];
          ld_lane8<T, G::NHP>(hs, (pt0 + r) * G::HW2 + px + dx, kq, hv);
          if (r <= 2) {
#pragma unroll
            for (int m = 0; m < 8; ++m) s0[m] = fmaf(wt[r * 3 + dx][m], hv[m], s0[m]);
          }
          if (r >= 1) {
#pragma unroll
            for (int m = 0; m < 8; ++m) s1[m] = fmaf(wt[(r - 1) * 3 + dx][m], hv[m], s1[m]);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        s0[m] = gelu_f(s0[m]);
        s1[m] = gelu_f(s1[m]);
      }
#pragma unroll
      for (int ks = 0; ks < K2; ++ks) {
        const typename F::frag g0 = to_frag<T>(s0, ks), g1 = to_frag<T>(s1, ks);
#pragma unroll
        for (int o = 0; o < OT; ++o) {
          acc[0][o] = F::mma(a2[o][ks], g0, acc[0][o]);
          acc[1][o] = F::mma(a2[o][ks], g1, acc[1][o]);
        }
      }
    }
    // the next chunk's weights (requested at this chunk's start, landed under [A] / [B]) go to the
    // other buffer, which nobody has read since the previous chunk-end barrier
    if (DB && more)
      pf.template store<XP, WP>(reinterpret_cast<T*>(smem + G::o_w1 + (buf ^ 1) * G::W1B),
                                       reinterpret_cast<T*>(smem + G::o_w2 + (buf ^ 1) * G::W2B),
                                       reinterpret_cast<float*>(smem + G::o_pb + (buf ^ 1) * G::PBB));
    lds_sync();  // [B] done with hs, w2s, pb
    if (!DB && more) {
      pf.template store<XP, WP>(reinterpret_cast<T*>(smem + G::o_w1), reinterpret_cast<T*>(smem + G::o_w2),
                                       reinterpret_cast<float*>(smem + G::o_pb));
      lds_sync();
    }
    if (DB) buf ^= 1;
  }
  // ---- epilogue: lane holds out[pixel px of tile row pt][channels 16 o + 4 kq .. + 4]
  const float rs = a.rowscale ? a.rowscale[b] : 1.f;
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = 2 * wid + i;
    const int yy = y0 + pt, xx = x0 + px;
    if (yy >= H || xx >= W) continue;
    const long row = (long)(b * H + yy) * W + xx;
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      const int c = o * 16 + 4 * kq;
      if (c >= C) break;
      const float4 bb = *reinterpret_cast<const float4*>(a.b2 + c);
      const float4 ll = *reinterpret_cast<const float4*>(a.ls + c);
      const float fv[4] = {acc[i][o][0] + bb.x, acc[i][o][1] + bb.y, acc[i][o][2] + bb.z, acc[i][o][3] + bb.w};
      const float lv[4] = {ll.x, ll.y, ll.z, ll.w};
      float xv[4], ov[4];
      ld4<T>((const T*)a.x + row * a.ldx + c, xv);
#pragma unroll
      for (int r = 0; r < 4; ++r) ov[r] = xv[r] + lv[r] * rs * fv[r];
      st4g<T>((T*)a.f + row * a.ldf + c, fv);
      st4g<T>((T*)a.out + row * a.ldout + c, ov);
    }
  }
}

// ---------------------------------------------------------------- backward
struct FfnBwdArgs {
  int B, H, W, C, hid;
  int tiles_y, tiles_x;
  const void* xn;
  long ldxn;
  const void* df;
  long lddf;
  const void* w1;  // [hid][C]
  const float* b1;
  const float* wpos;
  const float* bpos;
  const void* w2;  // [C][hid]
  void* g;         // [P][ldg] GELU output
  long ldg;
  void* dh;        // [P][lddh] fc1-output gradient
  long lddh;
  void* dxn;       // [P][lddxn]
  long lddxn;
  float* part;     // [tiles][hid * 10] depthwise weight (9) + bias (1) gradient partials
  int skip;        // profiling only (DFM_FFN_SKIP): bit i skips phase [A], [B], [C], the reduction
  long long* stamp;  // profiling only (DFM_FFN_STAMP): s_memtime at the phase boundaries of workgroup 0
};

// ---- packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) for the per-channel-pair phase
typedef float f2v __attribute__((ext_vector_type(2)));
DFM_INLINE f2v f2fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
DFM_INLINE f2v f2s(float v) { return f2v{v, v}; }
// normal_cdf_pdf (common.h) on two values: the same operations in the same order (bitwise identical)
DFM_INLINE void normal_cdf_pdf2(f2v x, f2v& cdf, f2v& pdf) {
  const f2v u = x * f2s(0.70710678118654752f);
  const f2v au = f2v{fabsf(u.x), fabsf(u.y)};
  const f2v den = f2fma(f2s(0.3275911f), au, f2s(1.0f));
  const f2v t = f2v{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f2v p = f2fma(f2s(1.061405429f), t, f2s(-1.453152027f));
  p = f2fma(p, t, f2s(1.421413741f));
  p = f2fma(p, t, f2s(-0.284496736f));
  p = f2fma(p, t, f2s(0.254829592f));
  p = p * t;
  const f2v na = -au * au;
  const f2v e = f2v{__expf(na.x), __expf(na.y)};
  const f2v tail = f2s(0.5f) * p * e;
  const f2v one_m = f2s(1.0f) - tail;
  cdf = f2v{u.x < 0.0f ? tail.x : one_m.x, u.y < 0.0f ? tail.y : one_m.y};
  pdf = f2s(0.39894228040143268f) * e;
}

// XOR swizzle of the 16-byte chunks of row k of an unpadded [rows][R] 16-bit LDS image (as the GEMM's
// row-contiguous tiles): conflict-free for both the k-contiguous fragment reads (ds_read_b128) and
// the transposing reads (ds_read_b64_tr_b16) of the same image.
template <int R>
DFM_INLINE int tr_swz(int k) {
  if constexpr (R >= 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else if constexpr (R == 64) return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  else return 2 * ((k >> 3) & 1);
}
// v + v[lane ^ X] for X = 32 / 16 with the gfx950 row-swap permutes (VALU, no LDS round trip)
template <int X> DFM_INLINE float xor_sum(float v) {
  const unsigned u = __float_as_uint(v);
  if constexpr (X == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}

template <int R> DFM_INLINE int swz_at(int k, int r) { return k * R + ((((r >> 3) ^ tr_swz<R>(k)) << 3) | (r & 7)); }

// Weight images of one chunk in the backward kernel (16-bit: unpadded + swizzled; float32: padded):
//   w1s [HC][CT] = W1c, read as A[j][c] (h recompute) and transposed as A[c][j] (W1c^T, dxn)
//   w2s [CT][HC] = W2c, read transposed as A[j][c] (W2c^T, dg)
template <typename T, int CT> struct BwdW {
  static constexpr bool H16 = sizeof(T) == 2;
  static constexpr int P1 = H16 ? CT : CT + 4, P2 = H16 ? HC : HC + 4;  // row pitches
  static DFM_INLINE int at1(int j, int c) { return H16 ? swz_at<CT>(j, c) : j * P1 + c; }
  static DFM_INLINE int at2(int c, int j) { return H16 ? swz_at<HC>(c, j) : c * P2 + j; }
  // A fragment rows r0 .. r0 + 16 of the image [K][R] read transposed: A[r][k] = img[k][r]
  template <int R>
  static DFM_INLINE typename FT<T>::frag tr_frag(const T* img, int r0, int k0, int lane) {
    if constexpr (H16) {
      const int i = lane & 15, gq = lane >> 4, q = i >> 2, p = i & 3;
      typedef __attribute__((address_space(3))) short4_t lds_s4;
      const int k = k0 + 8 * gq + q, r = r0 + 4 * p;
      short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + swz_at<R>(k, r)));
      short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + swz_at<R>(k + 4, r)));
      typedef __attribute__((ext_vector_type(8))) short short8_t;
      short8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8_t, v);
    } else {
      return img[(k0 + (lane >> 4)) * (R + 4) + r0 + (lane & 15)];
    }
  }
  // A[j][c] = W1c[j][c] (k-contiguous rows of w1s)
  static DFM_INLINE typename FT<T>::frag w1_frag(const T* w1s, int j0, int k0, int lane) {
    const int j = j0 + (lane & 15);
    if constexpr (H16) {
      return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(w1s + at1(j, k0 + 8 * (lane >> 4))));
    } else {
      return w1s[at1(j, k0 + (lane >> 4))];
    }
  }
};

// register-staged prefetch of W1c / W2c / the chunk's parameters into the backward's swizzled images
template <typename T, int CT, int NT>
struct BwdPrefetch {
  using BW = BwdW<T, CT>;
  static constexpr int V = 16 / sizeof(T);
  static constexpr int N1 = HC * CT / V, N2 = CT * HC / V;
  static constexpr int R1 = (N1 + NT - 1) / NT, R2 = (N2 + NT - 1) / NT;
  static constexpr int RP = (PB + NT - 1) / NT;
  uint4 w1[R1], w2[R2];
  float par[RP];
  DFM_INLINE void load(const T* __restrict__ gw1, const T* __restrict__ gw2, const float* __restrict__ b1,
                       const float* __restrict__ bpos, const float* __restrict__ wpos, int C, int hid, int c0) {
#pragma unroll
    for (int i = 0; i < R1; ++i) {
      const int v = threadIdx.x + i * NT;
      const int j = v / (CT / V), c = (v % (CT / V)) * V;
      w1[i] = (v < N1 && c < C) ? *reinterpret_cast<const uint4*>(gw1 + (long)(c0 + j) * C + c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < R2; ++i) {
      const int v = threadIdx.x + i * NT;
      const int c = v / (HC / V), j = (v % (HC / V)) * V;
      w2[i] = (v < N2 && c < C) ? *reinterpret_cast<const uint4*>(gw2 + (long)c * hid + c0 + j) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int e = threadIdx.x + i * NT;
      float v = 0.f;
      if (e < HC) v = b1[c0 + e];
      else if (e < 2 * HC) v = bpos[c0 + e - HC];
      else if (e < PB) {
        const int t = (e - 2 * HC) / HC, ch = (e - 2 * HC) % HC;
        v = wpos[(long)(c0 + ch) * 9 + t] + (t == 4 ? 1.0f : 0.0f);
      }
      par[i] = v;
    }
  }
  DFM_INLINE void store(T* w1s, T* w2s, float* pb) const {
#pragma unroll
    for (int i = 0; i < R1; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= N1) break;
      const int j = v / (CT / V), c = (v % (CT / V)) * V;
      *reinterpret_cast<uint4*>(w1s + BW::at1(j, c)) = w1[i];
    }
#pragma unroll
    for (int i = 0; i < R2; ++i) {
      const int v = threadIdx.x + i * NT;
      if (v >= N2) break;
      const int c = v / (HC / V), j = (v % (HC / V)) * V;
      *reinterpret_cast<uint4*>(w2s + BW::at2(c, j)) = w2[i];
    }
#pragma unroll
    for (int i = 0; i < RP; ++i) {
      const int e = threadIdx.x + i * NT;
      if (e < PB) pb[e] = par[i];
    }
  }
};

template <typename T, int CT, int TH>
struct BwdGeom {
  static constexpr int NT = 512, NW = 8;
  static constexpr int HW2 = TW + 2, HW4 = TW + 4;
  static constexpr int NH1 = (TH + 2) * HW2, NT1 = (NH1 + 15) / 16, NH1P = NT1 * 16;  // tile + 1 halo
  static constexpr int NH2 = (TH + 4) * HW4, NT2 = (NH2 + 15) / 16, NH2P = NT2 * 16;  // tile + 2 halo
  static constexpr int TP = TH * TW;
  static constexpr int XP = CT + FT<T>::PAD;  // xs / dfs row pitch
  using BW = BwdW<T, CT>;
  using P1 = Planes<NH1P, 4>;   // dg -> dhpre: read in the MFMA operand layout ([C])
  using P2 = Planes<NH2P, 16>;  // h: read per channel pair ([B])
  static constexpr size_t o_df = (size_t)NH2P * XP * sizeof(T);
  static constexpr size_t o_w1 = o_df + (size_t)NH1P * XP * sizeof(T);
  static constexpr size_t o_w2 = o_w1 + (size_t)HC * BW::P1 * sizeof(T);
  static constexpr size_t o_pb = o_w2 + (size_t)CT * BW::P2 * sizeof(T);
  static constexpr size_t o_hs = o_pb + (size_t)PB * 4;
  static constexpr size_t o_ds = o_hs + (size_t)P2::FLOATS * 4;
  static constexpr size_t o_red = o_ds + (size_t)P1::FLOATS * 4;
  static constexpr size_t o_gs = o_red + (size_t)NW * (HC / 2) * 10 * 2 * 4;  // per-wave depthwise-gradient sums
  static constexpr int GP = HC + (sizeof(T) == 2 ? 8 : 4);  // g staging row pitch (elements)
  static constexpr size_t lds = o_gs + (size_t)TP * GP * sizeof(T);  // g of the tile, written out in [C]
};

template <typename T, int CT, int TH>
__global__ __launch_bounds__(512) void convffn_bwd_kernel(FfnBwdArgs a) {
  using G = BwdGeom<T, CT, TH>;
  using F = FT<T>;
  using P1 = typename G::P1;
  using P2 = typename G::P2;
  using BW = typename G::BW;
  constexpr int NT = G::NT, NW = G::NW, XP = G::XP;
  constexpr int OT = CT / 16;
  constexpr int KC = CT / F::KS;
  constexpr int K2 = HC / F::KS;
  constexpr int PTW = 1;                // [C]: waves 0 .. TH-1 own one tile row each
  static_assert(TH <= NW, "one tile row per wave in [C]");
  constexpr int NU = G::NT2 + G::NT1;  // [A] units: h tiles, then dg tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* xs = reinterpret_cast<T*>(smem);
  T* dfs = reinterpret_cast<T*>(smem + G::o_df);
  T* w1s = reinterpret_cast<T*>(smem + G::o_w1);
  T* w2s = reinterpret_cast<T*>(smem + G::o_w2);
  float* pb = reinterpret_cast<float*>(smem + G::o_pb);
  float* hs = reinterpret_cast<float*>(smem + G::o_hs);
  float* ds = reinterpret_cast<float*>(smem + G::o_ds);
  float* red = reinterpret_cast<float*>(smem + G::o_red);
  T* gs = reinterpret_cast<T*>(smem + G::o_gs);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nt = a.B * a.tiles_y * a.tiles_x;
  const int tile = xcd_tile(blockIdx.x, nt);
  const int b = tile / (a.tiles_y * a.tiles_x);
  const int ty = (tile / a.tiles_x) % a.tiles_y, tx = tile % a.tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int C = a.C, hid = a.hid, H = a.H, W = a.W;
  const int px = lane & 15, kq = lane >> 4;
  auto inside = [&](int yy, int xx) { return yy >= 0 && yy < H && xx >= 0 && xx < W; };
  auto pix = [&](int yy, int xx) { return (long)(b * H + yy) * W + xx; };

  BwdPrefetch<T, CT, NT> pf;
  pf.load((const T*)a.w1, (const T*)a.w2, a.b1, a.bpos, a.wpos, C, hid, 0);
  stage_halo<T, CT, XP, NT>(xs, (const T*)a.xn, a.ldxn, G::NH2, G::NH2P, G::HW4, b, y0 - 2, x0 - 2, H, W, C);
  stage_halo<T, CT, XP, NT>(dfs, (const T*)a.df, a.lddf, G::NH1, G::NH1P, G::HW2, b, y0 - 1, x0 - 1, H, W, C);
  pf.store(w1s, w2s, pb);
  float4_t acc[PTW][OT];  // dxn^T[c][pixel]
#pragma unroll
  for (int i = 0; i < PTW; ++i)
#pragma unroll
    for (int o = 0; o < OT; ++o) acc[i][o] = float4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  const int nchunk = hid / HC;
  const bool stamping = a.stamp != nullptr && blockIdx.x == 0 && tid == 0;
  auto stamp = [&](int i) {
    if (stamping) a.stamp[i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  for (int ci = 0; ci < nchunk; ++ci) {
    const int c0 = ci * HC;
    const bool more = ci + 1 < nchunk;
    stamp(1 + ci * 5);
    if (more) pf.load((const T*)a.w1, (const T*)a.w2, a.b1, a.bpos, a.wpos, C, hid, c0 + HC);
    // ---- [A] h^T = W1c xn^T on tile + 2 halo (+ b1, zero outside the image) -> hs; dg^T = W2c^T df^T
    //          on tile + 1 halo -> ds (df rows outside the image are zero, so is dg)
    {
      typename F::frag aw[2][2][KC];  // [W1c | W2c^T][hidden tile][k-step]
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int ks = 0; ks < KC; ++ks) {
          aw[0][it][ks] = BW::w1_frag(w1s, it * 16, ks * F::KS, lane);
          aw[1][it][ks] = BW::template tr_frag<HC>(w2s, it * 16, ks * F::KS, lane);
        }
      const int nu = (a.skip & 1) ? 0 : NU;
      for (int u = wid; u < nu; u += NW) {
        const bool isH = u < G::NT2;
        const T* brow = (isH ? xs + (u * 16 + px) * XP : dfs + ((u - G::NT2) * 16 + px) * XP);
        float4_t h[2] = {float4_t{0.f, 0.f, 0.f, 0.f}, float4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < KC; ++ks) {
          const typename F::frag xb = F::ld(brow, ks * F::KS, lane);
#pragma unroll
          for (int it = 0; it < 2; ++it) h[it] = F::mma(isH ? aw[0][it][ks] : aw[1][it][ks], xb, h[it]);
        }
        if (isH) {
          const int q = u * 16 + px;
          const int yy = y0 - 2 + q / G::HW4, xx = x0 - 2 + q % G::HW4;
          const bool ok = q < G::NH2 && inside(yy, xx);
#pragma unroll
          for (int it = 0; it < 2; ++it) {
            const float4 bb = *reinterpret_cast<const float4*>(pb + it * 16 + 4 * kq);
            const float4 o4 = ok ? make_float4(h[it][0] + bb.x, h[it][1] + bb.y, h[it][2] + bb.z, h[it][3] + bb.w)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(hs + P2::at(q, it * 16 + 4 * kq)) = o4;
          }
        } else {
          const int q = (u - G::NT2) * 16 + px;
#pragma unroll
          for (int it = 0; it < 2; ++it)
            *reinterpret_cast<float4*>(ds + P1::at(q, it * 16 + 4 * kq)) =
                make_float4(h[it][0], h[it][1], h[it][2], h[it][3]);
        }
      }
    }
    lds_sync();
    stamp(2 + ci * 5);
    // ---- [B] on tile + 1 halo, one channel pair per unit (fixed per thread, its taps in registers):
    //          hpre = DW3(h) + bpos + h; g = GELU(hpre) (tile pixels -> HBM); dhpre = dg GELU'(hpre)
    //          in place of dg. The depthwise weight / bias gradient of an interior pixel,
    //          sum_t dhpre[p] h[p + tap t], reuses the 9 h values just loaded for hpre[p]: per-thread
    //          sums, then a fixed-order reduction (lanes l ^ 16, l ^ 32, then the 8 waves via LDS).
    {
      const int cp = tid & 15, ch = 2 * cp;  // channels ch, ch + 1 of the chunk
      f2v wt[9];
      const f2v bias2 = *reinterpret_cast<const f2v*>(pb + HC + ch);
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t] = *reinterpret_cast<const f2v*>(pb + 2 * HC + t * HC + ch);
      f2v dw[10];
#pragma unroll
      for (int t = 0; t < 10; ++t) dw[t] = f2s(0.f);
      const int nq = (a.skip & 2) ? 0 : G::NH1;
      for (int q = tid >> 4; q < nq; q += NT / 16) {
        const int qy = q / G::HW2, qx = q % G::HW2;
        f2v hv[9];
#pragma unroll
        for (int t = 0; t < 9; ++t)
          hv[t] = *reinterpret_cast<const f2v*>(hs + P2::at((qy + t / 3) * G::HW4 + qx + t % 3, ch));
        f2v* dp = reinterpret_cast<f2v*>(ds + P1::at(q, ch));
        f2v dv = *dp;
        f2v sv = bias2;
#pragma unroll
        for (int t = 0; t < 9; ++t) sv = f2fma(wt[t], hv[t], sv);
        f2v cdf, pdf;
        normal_cdf_pdf2(sv, cdf, pdf);
        dv = dv * f2fma(sv, pdf, cdf);
        *dp = dv;
        const int yy = y0 - 1 + qy, xx = x0 - 1 + qx;
        if (qy >= 1 && qy <= TH && qx >= 1 && qx <= TW && inside(yy, xx)) {
          // g of the interior pixels -> the LDS tile; [C] writes it out with one 16-byte store per lane
          T* gp = gs + ((qy - 1) * TW + qx - 1) * G::GP + ch;
          const f2v gv = sv * cdf;
          if constexpr (sizeof(T) == 2) {
            const T e2[2] = {Num<T>::from_f(gv.x), Num<T>::from_f(gv.y)};
            *reinterpret_cast<uint32_t*>(gp) = *reinterpret_cast<const uint32_t*>(e2);
          } else {
            *reinterpret_cast<float2*>(gp) = make_float2(gv.x, gv.y);
          }
#pragma unroll
          for (int t = 0; t < 9; ++t) dw[t] = f2fma(dv, hv[t], dw[t]);
          dw[9] += dv;
        }
      }
#pragma unroll
      for (int t = 0; t < 10; ++t) {  // + lane ^ 32, then + lane ^ 16 (v_permlane{32,16}_swap)
        dw[t].x = xor_sum<32>(dw[t].x);
        dw[t].y = xor_sum<32>(dw[t].y);
        dw[t].x = xor_sum<16>(dw[t].x);
        dw[t].y = xor_sum<16>(dw[t].y);
      }
      if (lane < 16) {
#pragma unroll
        for (int t = 0; t < 10; ++t) *reinterpret_cast<f2v*>(red + ((wid * 16 + cp) * 10 + t) * 2) = dw[t];
      }
    }
    lds_sync();
    stamp(3 + ci * 5);
    // ---- [C] dh = DW3^T(dhpre) + dhpre on the tile rows of this wave, straight into the B fragments
    //          of dxn^T += W1c^T dh^T; dh -> HBM
    {
      typename F::frag a1[OT][K2];
#pragma unroll
      for (int o = 0; o < OT; ++o)
#pragma unroll
        for (int ks = 0; ks < K2; ++ks) a1[o][ks] = BW::template tr_frag<CT>(w1s, o * 16, ks * F::KS, lane);
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        const int pt = wid + i * NW;
        if (pt >= TH || (a.skip & 4)) break;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {  // tap t reads dhpre at p - (t / 3 - 1, t % 3 - 1)
          float dv[8], wv[8];
          ld_lane8<T, G::NH1P>(ds, (pt + 2 - t / 3) * G::HW2 + px + 2 - t % 3, kq, dv);
          ld_lane8_par<T>(pb + 2 * HC + t * HC, kq, wv);
#pragma unroll
          for (int m = 0; m < 8; ++m) s[m] = fmaf(wv[m], dv[m], s[m]);
        }
#pragma unroll
        for (int ks = 0; ks < K2; ++ks) {
          const typename F::frag db = to_frag<T>(s, ks);
#pragma unroll
          for (int o = 0; o < OT; ++o) acc[i][o] = F::mma(a1[o][ks], db, acc[i][o]);
        }
        const int yy = y0 + pt, xx = x0 + px;
        if (inside(yy, xx)) {
          T* dp = (T*)a.dh + pix(yy, xx) * a.lddh + c0;
          T* gp = (T*)a.g + pix(yy, xx) * a.ldg + c0;
          const T* gl = gs + (pt * TW + px) * G::GP;
          if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4*>(dp + 8 * kq) = __builtin_bit_cast(uint4, pack16x8<T>(s));
            *reinterpret_cast<uint4*>(gp + 8 * kq) = *reinterpret_cast<const uint4*>(gl + 8 * kq);
          } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) dp[lane_ch<T>(kq, m)] = s[m];
            *reinterpret_cast<float4*>(gp + 8 * kq) = *reinterpret_cast<const float4*>(gl + 8 * kq);
            *reinterpret_cast<float4*>(gp + 8 * kq + 4) = *reinterpret_cast<const float4*>(gl + 8 * kq + 4);
          }
        }
      }
    }
    // the depthwise-gradient partials of the NW waves, summed in a fixed order: by the waves without a
    // tile row in [C] when there are enough of them, else after the chunk-end barrier
    constexpr int R0 = TH * 64 + HC * 10 <= NT ? TH * 64 : 0;
    auto reduce_red = [&]() {
      if (tid >= R0 && tid - R0 < HC * 10 && !(a.skip & 8)) {
        const int r = tid - R0, chn = r / 10, t = r % 10;
        const int cp = chn >> 1, e = chn & 1;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[((w * 16 + cp) * 10 + t) * 2 + e];
        a.part[(long)tile * hid * 10 + (long)(c0 + chn) * 10 + t] = v;
      }
    };
    if (R0 > 0) reduce_red();
    lds_sync();  // chunk done: hs / ds / weights / pb free
    stamp(4 + ci * 5);
    if (R0 == 0) reduce_red();  // red is rewritten only after the next chunk's [A] barrier
    if (more) {
      pf.store(w1s, w2s, pb);
      lds_sync();
    }
    stamp(5 + ci * 5);
  }
  // ---- dxn: lane holds dxn[pixel px of tile row pt][channels 16 o + 4 kq .. + 4]
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = wid + i * NW;
    if (PTW * NW > TH && pt >= TH) break;
    const int yy = y0 + pt, xx = x0 + px;
    if (!inside(yy, xx)) continue;
    T* dp = (T*)a.dxn + pix(yy, xx) * a.lddxn;
#pragma unroll
    for (int o = 0; o < OT; ++o) {
      const int c = o * 16 + 4 * kq;
      if (c >= C) break;
      const float v[4] = {acc[i][o][0], acc[i][o][1], acc[i][o][2], acc[i][o][3]};
      st4g<T>(dp + c, v);
    }
  }
}

// ---------------------------------------------------------------- launch configurations
// forward: 16-bit C <= 64 tiles 8 x 16 with double-buffered weights (two workgroups per CU); C = 128
// tiles 4 x 16, single-buffered; float32 (the parity path) single-buffered.
template <typename T, int CT> struct FwdCfg { static constexpr int TH = CT <= 64 ? 8 : 4; static constexpr bool DB = sizeof(T) == 2 && CT <= 64; };
// backward: one 512-thread workgroup per CU; float32 halves the tile
template <typename T, int CT> struct BwdCfg { static constexpr int TH = sizeof(T) == 2 ? 8 : 4; };

template <typename T, int CT>
int launch_fwd(FfnArgs& a, hipStream_t s) {
  using Cf = FwdCfg<T, CT>;
  using G = FwdGeom<T, CT, Cf::TH, Cf::DB>;
  static_assert(G::lds <= 160 * 1024, "LDS");
  auto kern = convffn_fwd_kernel<T, CT, Cf::TH, Cf::DB>;
  a.tiles_y = cdiv(a.H, Cf::TH);
  a.tiles_x = cdiv(a.W, TW);
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  DFM_LAUNCH(kern, dim3((unsigned)nblk), dim3(G::NT), G::lds, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, int CT>
int launch_bwd(FfnBwdArgs& a, hipStream_t s) {
  using Cf = BwdCfg<T, CT>;
  using G = BwdGeom<T, CT, Cf::TH>;
  static_assert(G::lds <= 160 * 1024, "LDS");
  auto kern = convffn_bwd_kernel<T, CT, Cf::TH>;
  a.tiles_y = cdiv(a.H, Cf::TH);
  a.tiles_x = cdiv(a.W, TW);
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  DFM_LAUNCH(kern, dim3((unsigned)nblk), dim3(G::NT), G::lds, s, a);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T>
long bwd_nblk(int B, int H, int W) {
  return (long)B * cdiv(H, BwdCfg<T, 64>::TH) * cdiv(W, TW);
}

template <typename T>
int fwd_dispatch(FfnArgs& a, hipStream_t s) {
  if (a.C <= 32) return launch_fwd<T, 32>(a, s);
  return launch_fwd<T, 64>(a, s);
}

template <typename T>
int bwd_dispatch(FfnBwdArgs& a, hipStream_t s) {
  if (a.C <= 32) return launch_bwd<T, 32>(a, s);
  return launch_bwd<T, 64>(a, s);
}

bool al16p(const void* p, long ld, int es) { return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0); }

}  // namespace

// The fused kernels cover the channel widths whose forward and backward tiles fit the LDS together
// (C <= 64, a multiple of 16: DFormer's stage-0 / stage-1 depth-branch ConvFFNs and Tiny / Large's
// narrow ones); wider ConvFFNs run on the separate GEMM / depthwise kernels.
extern "C" int dfm_convffn_supported(int dtype, int C, int hid) {
  if (dtype != DFM_BF16 && dtype != DFM_F16 && dtype != DFM_F32) return 0;
  return C >= 16 && C <= 64 && C % 16 == 0 && hid > 0 && hid % HC == 0;
}

extern "C" int dfm_convffn_fwd(int dtype, int B, int H, int W, int C, int hid, const void* xn, long ldxn,
                               const void* x, long ldx, const void* w1, const float* b1, const float* wpos,
                               const float* bpos, const void* w2, const float* b2, const float* ls,
                               const float* rowscale, void* out, long ldout, void* f, long ldf, dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, C, hid), "dfm_convffn_fwd: unsupported C=%d hid=%d dtype=%d", C, hid,
                dtype);
  DFM_CHECK_ARG(xn && x && w1 && b1 && wpos && bpos && w2 && b2 && ls && out && f, "dfm_convffn_fwd: null argument");
  const int es = dtype == DFM_F32 ? 4 : 2;
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
  if (dtype == DFM_F16) return fwd_dispatch<f16_t>(a, s);
  return fwd_dispatch<float>(a, s);
}

extern "C" size_t dfm_convffn_bwd_workspace(int dtype, int B, int H, int W, int C, int hid) {
  (void)C;
  const long nblk = dtype == DFM_F32 ? bwd_nblk<float>(B, H, W) : bwd_nblk<bf16_t>(B, H, W);
  return (size_t)nblk * hid * 10 * sizeof(float);
}

extern "C" int dfm_convffn_bwd(int dtype, int B, int H, int W, int C, int hid, const void* xn, long ldxn,
                               const void* df, long lddf, const void* w1, const float* b1, const float* wpos,
                               const float* bpos, const void* w2, void* g, long ldg, void* dh, long lddh, void* dxn,
                               long lddxn, float* dwpos, float* dbpos, void* workspace, dfm_stream_t stream) {
  DFM_CHECK_ARG(dfm_convffn_supported(dtype, C, hid), "dfm_convffn_bwd: unsupported C=%d hid=%d dtype=%d", C, hid,
                dtype);
  DFM_CHECK_ARG(xn && df && w1 && b1 && wpos && bpos && w2 && g && dh && dxn && dwpos && dbpos && workspace,
                "dfm_convffn_bwd: null argument");
  const int es = dtype == DFM_F32 ? 4 : 2;
  DFM_CHECK_ARG(al16p(xn, ldxn, es) && al16p(df, lddf, es) && al16p(g, ldg, es) && al16p(dh, lddh, es) &&
                    al16p(dxn, lddxn, es) && al16p(w1, C, es) && al16p(w2, hid, es) && al16p(b1, 0, 4) &&
                    al16p(bpos, 0, 4) && al16p(wpos, 0, 4),
                "dfm_convffn_bwd: rows must be 16-byte aligned");
  if ((long)B * H * W == 0) return DFM_OK;
  FfnBwdArgs a{};
  a.B = B; a.H = H; a.W = W; a.C = C; a.hid = hid;
  a.xn = xn; a.ldxn = ldxn; a.df = df; a.lddf = lddf;
  a.w1 = w1; a.b1 = b1; a.wpos = wpos; a.bpos = bpos; a.w2 = w2;
  a.g = g; a.ldg = ldg; a.dh = dh; a.lddh = lddh; a.dxn = dxn; a.lddxn = lddxn;
  a.part = (float*)workspace;
  static const int skip_env = [] {
    const char* e = getenv("DFM_FFN_SKIP");
    return e ? atoi(e) : 0;
  }();
  a.skip = skip_env;
  static long long* stamp_buf = [] {
    long long* p = nullptr;
    if (getenv("DFM_FFN_STAMP")) (void)hipMalloc(&p, 4096 * sizeof(long long));
    return p;
  }();
  a.stamp = stamp_buf;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if (dtype == DFM_BF16) rc = bwd_dispatch<bf16_t>(a, s);
  else if (dtype == DFM_F16) rc = bwd_dispatch<f16_t>(a, s);
  else rc = bwd_dispatch<float>(a, s);
  if (rc != DFM_OK) return rc;
  const long nblk = (long)a.B * a.tiles_y * a.tiles_x;
  DFM_LAUNCH(partial_sum_kernel<2>, dim3(cdiv((long)hid * 10, 64)), dim3(1024), 0, s, (int)nblk, (long)hid * 10,
             (const float*)workspace, dwpos, dbpos, 10L, 0);
  DFM_LAUNCH_CHECK();
  if (stamp_buf) {  // profiling only: print the phase cycles of workgroup 0 (averaged over the chunks)
    long long h[4096];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h, stamp_buf, sizeof(h), hipMemcpyDeviceToHost);
    const int nc = hid / HC;
    double ph[4] = {0, 0, 0, 0};
    for (int c = 0; c < nc; ++c)
      for (int k = 0; k < 4; ++k) ph[k] += (double)(h[2 + c * 5 + k] - h[1 + c * 5 + k]) / nc;
    fprintf(stderr, "convffn_bwd stamps (s_memtime ticks / chunk): prologue %lld  A %.0f  B %.0f  C %.0f  "
            "red+store %.0f  total %lld\n", h[1] - h[0], ph[0], ph[1], ph[2], ph[3], h[nc * 5] - h[0]);
  }
  return DFM_OK;
}
