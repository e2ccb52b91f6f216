// Depthwise k x k convolution over NHWC (DFormer.py:80-81 7x7 conv/e_conv, DFormer.py:54,62 3x3
// pos + identity): forward (+ fused identity / GELU second output), input gradient (the forward
// with flipped taps) and weight + bias gradient.
//
// HBM-bound. Both kernels stage an output tile's input window (tile + k-1 halo, zero-padded) in
// LDS once with coalesced 16-byte channel vectors (8 bf16 / 4 fp32 per lane), then every thread
// slides a register window along one LDS row for TWS consecutive outputs of one channel group.
// The weight gradient keeps per-thread tap accumulators across all tiles a block visits and writes
// one partial per block; a fixed-order second pass sums them (deterministic, no float atomics).
#include <algorithm>
#include <cstdlib>

#include <type_traits>

#include "common.h"

namespace {
template <typename T> struct DwCfg { static constexpr int CPT = 16 / sizeof(T); };

typedef float f2v __attribute__((ext_vector_type(2)));

// GELU(v) and GELU'(v) of N (even) channels, a channel pair per packed evaluation
template <int N>
DFM_INLINE void gelu_pairs(const float* v, float* g, float* d) {
#pragma unroll
  for (int e = 0; e < N; e += 2) {
    const f2v x = f2v{v[e], v[e + 1]};
    f2v cdf, pdf;
    normal_cdf_pdf2(x, cdf, pdf);
    const f2v gg = x * cdf, dd = __builtin_elementwise_fma(x, pdf, cdf);
    g[e] = gg.x; g[e + 1] = gg.y;
    d[e] = dd.x; d[e + 1] = dd.y;
  }
}

// one 16-byte vector -> CPT/2 channel pairs (packed-FMA operands; bf16 / f16 widen exactly)
template <typename T>
DFM_INLINE void unpack_pairs(uint4 q, f2v* v) {
  const uint32_t u[4] = {q.x, q.y, q.z, q.w};
  if constexpr (std::is_same<T, bf16_t>::value) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = f2v{__uint_as_float(u[k] << 16), __uint_as_float(u[k] & 0xffff0000u)};
  } else if constexpr (std::is_same<T, f16_t>::value) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = f2v{h2f((uint16_t)(u[k] & 0xffffu)), h2f((uint16_t)(u[k] >> 16))};
  } else {
    v[0] = f2v{__uint_as_float(u[0]), __uint_as_float(u[1])};
    v[1] = f2v{__uint_as_float(u[2]), __uint_as_float(u[3])};
  }
}


template <typename T>
DFM_INLINE void ldv(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    ld8<T>(p, v);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}
template <typename T>
DFM_INLINE void stv(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    st8<T>(p, v);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// ---------------------------------------------------------------- LDS-tiled forward (v3)
// A block owns an output tile of TH rows x TWT columns of one image and NG channel groups
// (NG * CPT channels). The (TH+K-1) x (TWT+K-1) input tile (zero-padded at the image border) is
// staged once into LDS as 16-byte vectors [row][col][group]; the block's K*K weights as fp32
// [tap][channel]. Each thread then produces TWS consecutive outputs of one row for one channel
// group, sliding a (TWS+K-1)-vector window along the LDS row for each of the K kernel rows.
// Global traffic is the tile plus its halo (read once, coalesced along channels); the identity
// term comes from the staged tile centre for free.
// XCD-aware block order. Blocks are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one L2), so block b is given logical index remap(b): XCD k owns one contiguous run of the
// logical order. Logical indices run channel-group fastest, then tile in raster order, so the
// blocks that read the two halves of one 128-byte line, and the vertically adjacent tiles that
// share K-1 halo rows, run on the same XCD close together in time (their re-reads hit its L2).
DFM_INLINE long xcd_remap(long b, long n) {
  const long per = n / 8, rem = n % 8, k = b % 8, i = b / 8;
  return k * per + (k < rem ? k : rem) + i;
}

template <typename T, int K>
struct DwTile;
template <typename T> struct DwTile<T, 3> { static constexpr int TWS = 4, STRIPS = 8; };
template <typename T> struct DwTile<T, 7> { static constexpr int TWS = 4, STRIPS = 4; };

// forward tile shape: VAR 0 = DwTile; VAR 1 (7x7) = 8 outputs per thread along the row (the window
// and the tap weights each read once per kernel row serve twice the FMAs of TWS = 4)
template <typename T, int K, int VAR>
struct DwFwdTile {
  static constexpr int TWS = VAR == 1 ? 8 : DwTile<T, K>::TWS, STRIPS = VAR == 1 ? 2 : DwTile<T, K>::STRIPS;
};

template <typename T, int K, bool FLIP, int NG, int VAR = 0>
__global__ __launch_bounds__(256) void dw_tile_fwd_kernel(int B, int H, int W, int C, int tiles_h, int tiles_w,
                                                          const T* __restrict__ x, long ldx,
                                                          const float* __restrict__ w, const float* __restrict__ bias,
                                                          int add_identity, T* __restrict__ y, long ldy,
                                                          int accumulate, T* __restrict__ gout, long ldg) {
  constexpr int CPT = DwCfg<T>::CPT, R = K / 2;
  constexpr int TWS = DwFwdTile<T, K, VAR>::TWS, STRIPS = DwFwdTile<T, K, VAR>::STRIPS;
  constexpr int TH = 256 / (NG * STRIPS), TWT = TWS * STRIPS;
  constexpr int IH = TH + K - 1, IW = TWT + K - 1, CW = NG * CPT;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  uint4* xs = reinterpret_cast<uint4*>(dsm);                    // [IH][IW][NG]
  float* wl = reinterpret_cast<float*>(dsm + IH * IW * NG * 16);  // [K*K][CW]

  const int ncg = (C / CPT + NG - 1) / NG;
  const long l = xcd_remap(blockIdx.x, (long)gridDim.x);
  const int tile = (int)(l / ncg);
  const int tw = tile % tiles_w, th = (tile / tiles_w) % tiles_h, b = tile / (tiles_w * tiles_h);
  const int h0 = th * TH, w0 = tw * TWT;
  const int cbase = (int)(l % ncg) * CW;
  const long img = (long)b * H * W;

  for (int e = threadIdx.x; e < K * K * CW; e += 256) {
    const int tap = e / CW, c = cbase + e % CW;
    wl[e] = c < C ? w[(long)c * K * K + (FLIP ? K * K - 1 - tap : tap)] : 0.f;
  }
  {  // all of a thread's tile loads in flight together, then one LDS write pass
    constexpr int NV = IH * IW * NG, NL = (NV + 255) / 256;
    uint4 buf[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int v = threadIdx.x + l * 256;
      const int g = v % NG, col = (v / NG) % IW, row = v / (NG * IW);
      const int hh = h0 + row - R, ww = w0 + col - R, c = cbase + g * CPT;
      buf[l] = make_uint4(0, 0, 0, 0);
      if (v < NV && hh >= 0 && hh < H && ww >= 0 && ww < W && c < C)
        buf[l] = *reinterpret_cast<const uint4*>(x + (img + (long)hh * W + ww) * ldx + c);
    }
#pragma unroll
    for (int l = 0; l < NL; ++l)
      if (threadIdx.x + l * 256 < NV) xs[threadIdx.x + l * 256] = buf[l];
  }
  __syncthreads();

  const int g = threadIdx.x % NG, strip = (threadIdx.x / NG) % STRIPS, row = threadIdx.x / (NG * STRIPS);
  const int c0 = cbase + g * CPT;
  const int oh = h0 + row, ow0 = w0 + strip * TWS;
  if (c0 >= C || oh >= H || ow0 >= W) return;
  // channel pairs on packed FMA (v_pk_fma_f32): the same per-element FMA sequence, half the instructions
  constexpr int CP = CPT / 2;
  f2v accp[TWS][CP];
#pragma unroll
  for (int e = 0; e < CP; ++e) {
    const f2v bv = bias ? f2v{bias[c0 + 2 * e], bias[c0 + 2 * e + 1]} : f2v{0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TWS; ++t) accp[t][e] = bv;
  }
#pragma unroll 1
  for (int i = 0; i < K; ++i) {
    f2v win[TWS + K - 1][CP];
    const uint4* xr = xs + ((row + i) * IW + strip * TWS) * NG + g;
#pragma unroll
    for (int u = 0; u < TWS + K - 1; ++u) unpack_pairs<T>(xr[u * NG], win[u]);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      f2v wv[CP];
      const float4* wp = reinterpret_cast<const float4*>(wl + (i * K + j) * CW + g * CPT);
#pragma unroll
      for (int q4 = 0; q4 < CPT / 4; ++q4) {
        const float4 f = wp[q4];
        wv[2 * q4] = f2v{f.x, f.y};
        wv[2 * q4 + 1] = f2v{f.z, f.w};
      }
#pragma unroll
      for (int t = 0; t < TWS; ++t)
#pragma unroll
        for (int e = 0; e < CP; ++e) accp[t][e] = __builtin_elementwise_fma(wv[e], win[t + j][e], accp[t][e]);
    }
  }
  float acc[TWS][CPT];
#pragma unroll
  for (int t = 0; t < TWS; ++t)
#pragma unroll
    for (int e = 0; e < CP; ++e) {
      acc[t][2 * e] = accp[t][e].x;
      acc[t][2 * e + 1] = accp[t][e].y;
    }
#pragma unroll
  for (int t = 0; t < TWS; ++t) {
    const int ow = ow0 + t;
    if (ow >= W) break;
    const long p = img + (long)oh * W + ow;
    if (add_identity & 1) {
      const uint4 q = xs[((row + R) * IW + strip * TWS + t + R) * NG + g];
      float xi[CPT];
      if constexpr (sizeof(T) == 2) {
        Raw8<T> r8;
        r8.w[0] = q;
        unpack8(r8, xi);
      } else {
        xi[0] = __uint_as_float(q.x); xi[1] = __uint_as_float(q.y);
        xi[2] = __uint_as_float(q.z); xi[3] = __uint_as_float(q.w);
      }
#pragma unroll
      for (int e = 0; e < CPT; ++e) acc[t][e] += xi[e];
    }
    T* yp = y + p * ldy + c0;
    if (accumulate) {
      float o[CPT];
      ldv<T>(yp, o);
#pragma unroll
      for (int e = 0; e < CPT; ++e) acc[t][e] += o[e];
    }
    if (gout) {  // GELU output; y holds the pre-activation or (flag 2) its GELU derivative
      float gv[CPT], dv[CPT];
      gelu_pairs<CPT>(acc[t], gv, dv);
      stv<T>(yp, (add_identity & 2) ? dv : acc[t]);
      stv<T>(gout + p * ldg + c0, gv);
    } else {
      stv<T>(yp, acc[t]);
    }
  }
}

// ---------------------------------------------------------------- row-streaming 3x3 weight gradient
// The tiled kernel above reduces one LDS tile per block visit; on the small-spatial, wide-channel
// stages (30x40 / 15x20 with 1024-2048 hidden channels) a block sees a single tile and the
// staging, the strip-major LDS reads (bank conflicts) and the per-block reduction dominate. Here a
// lane owns one 8-byte channel vector (4 bf16 / 2 fp32 channels: the register window + 10 tap
// accumulators fit in ~160 VGPRs, 3 waves per SIMD) and a TW-column strip and walks down a chunk of RC rows,
// keeping the three input rows its taps touch in registers (one new input row and one dy row per
// output row, loaded one row ahead so the next loads are in flight during the FMAs). A wave's
// lanes cover consecutive channel vectors of one pixel (512 contiguous bytes per load), so every
// load is coalesced and each element of x and dy is fetched once from HBM (the two halo columns
// and halo rows between neighbouring strips / chunks come from L2). The 9 taps + bias of all the
// units a block visits stay in registers; one LDS reduction per block writes the block's partial
// [blockIdx.x][C][10]; partial_sum_kernel sums them in fixed order (deterministic).
constexpr int W3_TW = 4;

struct W3Geom {
  int LPU, UPW, slices, nstrips, nchunks, RC;
  long units, nsb;
};

__host__ __device__ inline long w3_units(int B, int nstrips, int nchunks) { return (long)B * nstrips * nchunks; }

template <typename T> struct W3Cfg { static constexpr int EPL = 8 / sizeof(T); };

// Row chunking of the streaming 3x3 kernels. A unit is one TW-column strip x RC rows of one image
// for one wave's channel vectors; every wave takes one unit. The backward and forward kernels hold
// 2 waves per SIMD (VGPR-bound), so a launch runs in rounds of 2048 waves on the 256 CUs: the chunk
// count minimises rounds x (RC + 2 halo rows), chunks of at least 5 rows. Measured over the
// DFormer-B ConvFFN shapes (tools/dw3_geom_sweep.py, profiles/r04_dw3_geom_sweep.txt): a wave count
// just past a round boundary cost up to 40 % (30x40x1024 backward 58 vs 42 us at 3200 vs 1920
// waves); a fixed 3072 / 8192-wave target sat past one on five of the eight shapes.
inline W3Geom w3_geom_cpl(int B, int H, int W, int C, int CPT, int waves_per_simd) {
  W3Geom g;
  const int G = C / CPT;
  g.LPU = std::min(64, G);
  g.UPW = 64 / g.LPU;
  g.slices = (G + g.LPU - 1) / g.LPU;
  g.nstrips = (W + W3_TW - 1) / W3_TW;
  const long slots = 256L * 4 * waves_per_simd;
  const int max_chunks = std::max(1, H / 5);
  long best = -1;
  for (int n = 1; n <= max_chunks; ++n) {
    const int rc = (H + n - 1) / n;
    if (n > 1 && (H + rc - 1) / rc != n) continue;  // same row chunk as a smaller count
    const long waves = (w3_units(B, g.nstrips, n) + g.UPW - 1) / g.UPW * g.slices;
    const long cost = (waves + slots - 1) / slots * (rc + 2);
    if (best < 0 || cost < best) {
      best = cost;
      g.RC = rc;
    }
  }
  g.nchunks = (H + g.RC - 1) / g.RC;
  g.units = w3_units(B, g.nstrips, g.nchunks);
  const long waves = (g.units + g.UPW - 1) / g.UPW;
  g.nsb = std::max(1L, (waves + 3) / 4);
  return g;
}
template <typename T>
W3Geom w3_geom(int B, int H, int W, int C, int waves_per_simd = 2) {
  return w3_geom_cpl(B, H, W, C, W3Cfg<T>::EPL, waves_per_simd);
}

// Out-of-image taps: every row load is issued unconditionally from an in-image address (the unit's
// own first row h0 / first column w0, already in cache) and the out-of-image vectors are zeroed at
// their first use through a per-row column bitmask. A load under `ok ? load : 0` sits in a divergent
// branch and hipcc waits for it (vmcnt(0)) at the merge right after issue, so the next row's
// prefetch never overlapped the current row's FMAs; the mask is applied one loop iteration after the
// load, where the wait is needed anyway.
template <typename T>
DFM_INLINE uint2 w3_ld(const T* base, long ld, long img, int W, int h, int ww, int c0) {
  return *reinterpret_cast<const uint2*>(base + (img + (long)h * W + ww) * ld + c0);
}

// The streaming forward's input through a raw buffer resource (tensors of < 2 GiB, the host checks): a
// load's 32-bit byte offset is a running row offset (one add per row) plus a wave-uniform column step (one
// add per load), instead of a 64-bit multiply per load. Rows / columns outside the tensor (negative offsets
// wrap past the extent) read as zero through the resource's range check (num_records = the operand's
// extent; the whole offset is in the VGPR operand, which is what the check covers) and are masked at
// first use anyway, so no address needs clamping. Isolated (tools/ffn_kernels_bench.py): stage 1 / 2
// forwards 137.7 -> 120.8, 61.4 -> 53.2, 32.0 -> 30.5 us, stage 0 unchanged; the same change in the fused
// backward (2 operands) was slower (242.9 -> 248.5 us at stage 0, 39.1 -> 45.9 at stage 2) and is not used:
// at 2 waves per SIMD that kernel is latency-bound, not bound by its quarter-rate address instructions.
template <typename T>
DFM_INLINE __amdgpu_buffer_rsrc_t w3_rsrc(const T* p, long rows, long ld, int C) {
  const long ext = ((rows - 1) * ld + C) * (long)sizeof(T);  // (unused past 2 GiB: the pointer path runs)
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)min(ext, 0x7fffffffL), 0x00020000);
}
DFM_INLINE uint2 w3_bld(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
}
// the buffer path addresses every operand byte with a 32-bit offset
template <typename T>
bool w3_buf_ok(long rows, long ld, int C) {
  return ((rows - 1) * ld + C) * (long)sizeof(T) < (1L << 31) - (1L << 20);
}

template <int N>
DFM_INLINE void w3_keep(uint2* r, unsigned m) {  // zero the vectors whose bit in m is clear
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const bool k = (m >> q) & 1u;
    r[q].x = k ? r[q].x : 0u;
    r[q].y = k ? r[q].y : 0u;
  }
}

template <typename T>
DFM_INLINE void w3_unpack(uint2 q, float* v) {
  if constexpr (std::is_same<T, f16_t>::value) {
    v[0] = h2f((uint16_t)(q.x & 0xffffu)); v[1] = h2f((uint16_t)(q.x >> 16));
    v[2] = h2f((uint16_t)(q.y & 0xffffu)); v[3] = h2f((uint16_t)(q.y >> 16));
  } else if constexpr (sizeof(T) == 2) {
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  } else {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y);
  }
}

template <typename T>
DFM_INLINE void w3_pairs(uint2 q, f2v* v) {
  if constexpr (std::is_same<T, f16_t>::value) {
    v[0] = f2v{h2f((uint16_t)(q.x & 0xffffu)), h2f((uint16_t)(q.x >> 16))};
    v[1] = f2v{h2f((uint16_t)(q.y & 0xffffu)), h2f((uint16_t)(q.y >> 16))};
  } else if constexpr (sizeof(T) == 2) {
    v[0] = f2v{__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u)};
    v[1] = f2v{__uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u)};
  } else {
    v[0] = f2v{__uint_as_float(q.x), __uint_as_float(q.y)};
  }
}

template <typename T>
DFM_INLINE void w3_store(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    uint2 q;
    q.x = (uint32_t)bits16<T>(v[0]) | ((uint32_t)bits16<T>(v[1]) << 16);
    q.y = (uint32_t)bits16<T>(v[2]) | ((uint32_t)bits16<T>(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = q;
  } else {
    *reinterpret_cast<uint2*>(p) = make_uint2(__float_as_uint(v[0]), __float_as_uint(v[1]));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dw3_stream_wgrad_kernel(int B, int H, int W, int C, int RC, int nstrips,
                                                               int nchunks, int LPU, int UPW,
                                                               const T* __restrict__ x, long ldx,
                                                               const T* __restrict__ dy, long lddy,
                                                               float* __restrict__ part) {
  constexpr int CPT = W3Cfg<T>::EPL, TW = W3_TW, NX = TW + 2, NV = 10 * CPT, VCH = 20;
  __shared__ float red[4][VCH][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lg = lane % LPU, usub = lane / LPU;
  const int G = C / CPT, cg = blockIdx.y * LPU + lg;
  const bool valid = usub < UPW && cg < G;
  const int c0 = cg * CPT;
  const long units = w3_units(B, nstrips, nchunks);

  float acc[10][CPT];
#pragma unroll
  for (int a = 0; a < 10; ++a)
#pragma unroll
    for (int e = 0; e < CPT; ++e) acc[a][e] = 0.f;

  const long stride = (long)gridDim.x * 4 * UPW;
  for (long u = ((long)blockIdx.x * 4 + wave) * UPW + usub; valid && u < units; u += stride) {
    const int strip = (int)(u % nstrips), chunk = (int)((u / nstrips) % nchunks);
    const long b = u / ((long)nstrips * nchunks);
    const int w0 = strip * TW, h0 = chunk * RC, h1 = min(h0 + RC, H);
    const long img = b * H * W;
    unsigned cmx = 0, cmd = 0;  // in-image columns of the x window / the dy strip
#pragma unroll
    for (int q = 0; q < NX; ++q) cmx |= (unsigned)(w0 - 1 + q >= 0 && w0 - 1 + q < W) << q;
#pragma unroll
    for (int t = 0; t < TW; ++t) cmd |= (unsigned)(w0 + t < W) << t;
    auto load_x = [&](int h, uint2* r) -> unsigned {  // returns the row's keep mask
      const bool hok = h >= 0 && h < H;
      const int hc = hok ? h : h0;
#pragma unroll
      for (int q = 0; q < NX; ++q) r[q] = w3_ld<T>(x, ldx, img, W, hc, ((cmx >> q) & 1u) ? w0 - 1 + q : w0, c0);
      return hok ? cmx : 0u;
    };
    auto load_dy = [&](int h, uint2* r) -> unsigned {
      const bool hok = h < h1;
      const int hc = hok ? h : h0;
#pragma unroll
      for (int t = 0; t < TW; ++t) r[t] = w3_ld<T>(dy, lddy, img, W, hc, ((cmd >> t) & 1u) ? w0 + t : w0, c0);
      return hok ? cmd : 0u;
    };
    uint2 x0[NX], x1[NX], x2[NX], dc[TW];
    w3_keep<NX>(x0, load_x(h0 - 1, x0));
    w3_keep<NX>(x1, load_x(h0, x1));
    unsigned m2 = load_x(h0 + 1, x2);
    unsigned md = load_dy(h0, dc);
    for (int h = h0; h < h1; ++h) {
      w3_keep<NX>(x2, m2);  // the rows loaded one iteration ago
      w3_keep<TW>(dc, md);
      uint2 xn[NX], dn[TW];
      m2 = load_x(h + 1 < h1 ? h + 2 : H, xn);  // row H (and any row past the chunk) reads as zeros
      md = load_dy(h + 1, dn);
      float gv[TW][CPT];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        w3_unpack<T>(dc[t], gv[t]);
#pragma unroll
        for (int e = 0; e < CPT; ++e) acc[9][e] += gv[t][e];
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const uint2* xr = a == 0 ? x0 : (a == 1 ? x1 : x2);
#pragma unroll
        for (int q = 0; q < NX; ++q) {
          float xv[CPT];
          w3_unpack<T>(xr[q], xv);
          // input column q feeds output column t with tap j = q - t
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const int j = q - t;
            if (j < 0 || j >= 3) continue;
#pragma unroll
            for (int e = 0; e < CPT; ++e) acc[a * 3 + j][e] = fmaf(gv[t][e], xv[e], acc[a * 3 + j][e]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) {
        x0[q] = x1[q];
        x1[q] = x2[q];
        x2[q] = xn[q];
      }
#pragma unroll
      for (int t = 0; t < TW; ++t) dc[t] = dn[t];
    }
  }

  // block reduction over the 4 waves and the UPW units of a wave that share a channel vector
  const long pbase = (long)blockIdx.x * C * 10;
#pragma unroll
  for (int vc = 0; vc < NV; vc += VCH) {
    if (vc) __syncthreads();
#pragma unroll
    for (int v = 0; v < VCH; ++v)
      if (vc + v < NV) red[wave][v][lane] = acc[(vc + v) / CPT][(vc + v) % CPT];
    __syncthreads();
    for (int idx = threadIdx.x; idx < VCH * LPU; idx += 256) {
      const int v = idx / LPU, l = idx % LPU, V = vc + v;
      const int c = (blockIdx.y * LPU + l) * CPT + V % CPT;
      if (V >= NV || c >= C) continue;
      float sum = 0.f;
      for (int w = 0; w < 4; ++w)
        for (int us = 0; us < UPW; ++us) sum += red[w][v][us * LPU + l];
      const int tap = V / CPT;  // 0..8 = kernel row * 3 + col, 9 = bias
      part[pbase + (long)c * 10 + tap] = sum;
    }
  }
}

template <typename T>
long w3_launch(int B, int H, int W, int C, const void* x, long ldx, const void* dy, long lddy, float* part,
               hipStream_t s) {
  const W3Geom g = w3_geom<T>(B, H, W, C, 3);
  DFM_LAUNCH(dw3_stream_wgrad_kernel<T>, dim3((unsigned)g.nsb, (unsigned)g.slices), dim3(256), 0, s, B, H,
                     W, C, g.RC, g.nstrips, g.nchunks, g.LPU, g.UPW, (const T*)x, ldx, (const T*)dy, lddy, part);
  return g.nsb;
}

// ---------------------------------------------------------------- LDS-tiled 7x7 weight gradient (v4)
// The streaming kernel above re-reads every input row once per kernel row (7 blocks) and every
// input column 2.5x (halo of a 4-wide strip), ~17x the input through L2 per pass. Here a block owns
// NG channel vectors (CPT channels each) and walks spatial tiles of TH x TW output pixels; per tile
// the dy tile [TH][TW][NG] and its zero-padded input window [TH+6][TW+6][NG] are staged in LDS once
// (1.9x the input, 1x dy, from HBM/L2), then thread (g, i, part) accumulates kernel row i of
// channel vector g — 7 taps x CPT channels — over pixel rows part, part + NP, ...: per pixel one dy
// vector and one new input vector (the 7-vector window slides along the row in registers) feed
// 7 * CPT FMAs, so the kernel runs at the VALU rate, not the L2 rate. The input window's row pitch
// is padded so NG * pitch = 4 (mod 8) vectors: the lanes of one 8-lane LDS phase — NG channel
// vectors x 2 kernel rows — fall on 8 distinct 16-byte bank groups (dy reads of one pixel are
// broadcast). At the end the NP parts of a (g, i) meet in LDS in a fixed order and the block writes
// its partial [blockIdx.x][C][50]; partial_sum_kernel<2> sums the spatial lanes (deterministic).
constexpr int W7L_NG = 4, W7L_TH = 16, W7L_TW = 14, W7L_NP = 8;   // TW: a multiple of 7 (register ring)
constexpr int W7L_IH = W7L_TH + 6, W7L_IW = W7L_TW + 7;  // +7: pitch 21 -> NG * pitch = 84 = 4 (mod 8)
static_assert((W7L_NG * W7L_IW) % 8 == 4, "LDS pitch");

template <typename T>
__global__ __launch_bounds__(256) void dw7_lds_wgrad_kernel(int B, int H, int W, int C, int tiles_h, int tiles_w,
                                                            int nsb, int slabs, const T* __restrict__ x, long ldx,
                                                            const T* __restrict__ dy, long lddy,
                                                            float* __restrict__ part) {
  constexpr int CPT = DwCfg<T>::CPT, CP = CPT / 2, NG = W7L_NG, TH = W7L_TH, TW = W7L_TW, NP = W7L_NP;
  constexpr int IH = W7L_IH, IW = W7L_IW, NX = IH * (TW + 6) * NG, ND = TH * TW * NG;
  constexpr int NL = (NX + ND + 255) / 256, NACT = NG * 7 * NP, BQ = 256 / NG;
  __shared__ uint4 xs[IH * IW * NG];
  __shared__ uint4 ds[ND];
  const int ncv = C / CPT;
  // (spatial lane sb, channel slab): slabs fastest in an order dealt to the XCDs in contiguous runs, so
  // the slabs that read the 64-byte halves of one 128-byte pixel line, and the spatial lanes that share
  // tile halos, run on one XCD at the same time (their re-reads hit its L2)
  const int lid = (int)xcd_remap(blockIdx.x, (long)nsb * slabs);
  const int sb = lid / slabs;
  const int cv0 = (lid % slabs) * NG;  // first channel vector of the slab
  const long ntiles = (long)B * tiles_h * tiles_w;
  const int t = threadIdx.x;
  const int g = t % NG, i = (t / NG) % 7, prt = t / (NG * 7);
  const bool active = t < NACT;
  f2v acc[7][CP], bs[CP];
#pragma unroll
  for (int j = 0; j < 7; ++j)
#pragma unroll
    for (int e = 0; e < CP; ++e) acc[j][e] = f2v{0.f, 0.f};
#pragma unroll
  for (int e = 0; e < CP; ++e) bs[e] = f2v{0.f, 0.f};

  for (long tile = sb; tile < ntiles; tile += nsb) {
    const int tw = (int)(tile % tiles_w), th = (int)((tile / tiles_w) % tiles_h);
    const long b = tile / ((long)tiles_w * tiles_h);
    const int h0 = th * TH, w0 = tw * TW;
    const long img = b * H * W;
    uint4 buf[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int v = t + l * 256;
      buf[l] = make_uint4(0, 0, 0, 0);
      if (v < NX) {
        const int gg = v % NG, col = (v / NG) % (TW + 6), row = v / (NG * (TW + 6));
        const int hh = h0 + row - 3, ww = w0 + col - 3, cv = cv0 + gg;
        if (hh >= 0 && hh < H && ww >= 0 && ww < W && cv < ncv)
          buf[l] = *reinterpret_cast<const uint4*>(x + (img + (long)hh * W + ww) * ldx + cv * CPT);
      } else if (v < NX + ND) {
        const int u = v - NX;
        const int gg = u % NG, col = (u / NG) % TW, row = u / (NG * TW);
        const int hh = h0 + row, ww = w0 + col, cv = cv0 + gg;
        if (hh < H && ww < W && cv < ncv)
          buf[l] = *reinterpret_cast<const uint4*>(dy + (img + (long)hh * W + ww) * lddy + cv * CPT);
      }
    }
    __syncthreads();  // the previous tile's reads are done
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int v = t + l * 256;
      if (v < NX) {
        const int gg = v % NG, col = (v / NG) % (TW + 6), row = v / (NG * (TW + 6));
        xs[(row * IW + col) * NG + gg] = buf[l];
      } else if (v < NX + ND) {
        ds[v - NX] = buf[l];
      }
    }
    __syncthreads();
    {  // bias gradient: thread (g, q) sums the tile's pixels q, q + BQ, ... of channel vector g
      for (int pix = t / NG; pix < TH * TW; pix += BQ) {
        f2v d[CP];
        unpack_pairs<T>(ds[pix * NG + g], d);
#pragma unroll
        for (int e = 0; e < CP; ++e) bs[e] += d[e];
      }
    }
    if (active) {
#pragma unroll 1
      for (int r = prt; r < TH; r += NP) {
        const uint4* xr = xs + ((r + i) * IW) * NG + g;
        const uint4* dr = ds + (r * TW) * NG + g;
        f2v xw[7][CP];  // ring: input column q of the row in slot q % 7
#pragma unroll
        for (int u = 0; u < 6; ++u) unpack_pairs<T>(xr[u * NG], xw[u]);
#pragma unroll 1
        for (int cb = 0; cb < TW; cb += 7) {
#pragma unroll
          for (int s7 = 0; s7 < 7; ++s7) {
            const int c = cb + s7;
            unpack_pairs<T>(xr[(c + 6) * NG], xw[(s7 + 6) % 7]);
            f2v d[CP];
            unpack_pairs<T>(dr[c * NG], d);
#pragma unroll
            for (int j = 0; j < 7; ++j)
#pragma unroll
              for (int e = 0; e < CP; ++e) acc[j][e] = __builtin_elementwise_fma(d[e], xw[(s7 + j) % 7][e], acc[j][e]);
          }
        }
      }
    }
  }
  // the NP parts of each (g, i) meet in LDS in part order, then part 0 writes the block's partial;
  // the bias partials of the BQ pixel lanes of each g likewise (lane order)
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);
  constexpr int RS = 7 * CPT + 1;
  for (int q = 1; q < NP; ++q) {
    if (active && prt == q) {
      float* o = red + (g * 7 + i) * RS;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int e = 0; e < CP; ++e) {
          o[j * CPT + 2 * e] = acc[j][e].x;
          o[j * CPT + 2 * e + 1] = acc[j][e].y;
        }
    }
    __syncthreads();
    if (active && prt == 0) {
      const float* o = red + (g * 7 + i) * RS;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int e = 0; e < CP; ++e) acc[j][e] += f2v{o[j * CPT + 2 * e], o[j * CPT + 2 * e + 1]};
    }
    __syncthreads();
  }
  float* bred = red + NG * 7 * RS;  // [BQ][NG][CPT]
#pragma unroll
  for (int e = 0; e < CP; ++e) {
    bred[t * CPT + 2 * e] = bs[e].x;
    bred[t * CPT + 2 * e + 1] = bs[e].y;
  }
  __syncthreads();
  const long pbase = (long)sb * C * 50;
  if (active && prt == 0 && cv0 + g < ncv) {
#pragma unroll
    for (int e = 0; e < CP; ++e) {
      const int c = (cv0 + g) * CPT + 2 * e;
      float* o = part + pbase + (long)c * 50;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        o[i * 7 + j] = acc[j][e].x;
        o[50 + i * 7 + j] = acc[j][e].y;
      }
    }
  }
  if (t < NG * CPT) {  // bias: thread (g, e) sums the BQ lanes in order
    const int gg = t / CPT, e = t % CPT;
    if (cv0 + gg < ncv) {
      float sum = 0.f;
      for (int q = 0; q < BQ; ++q) sum += bred[(q * NG + gg) * CPT + e];
      part[pbase + (long)((cv0 + gg) * CPT + e) * 50 + 49] = sum;
    }
  }
}

// ---------------------------------------------------------------- one-pass 7x7 backward (data + weight)
// The attention's 7x7 depthwise backward (DFormer.py:80-81, 115, 133; conv and e_conv) in ONE launch over
// dy: a block (spatial lane, channel slab of NG vectors, as dw7_lds_wgrad_kernel) stages per TH x TW tile
// the zero-padded input window and the dy window (tile + 3-pixel halo) in LDS once; the tile's input
// gradient (the dy window against the flipped taps, 7 outputs of one row x half a channel vector per
// thread) and the weight / bias partials (the dy tile against the input window, thread (g, kernel row i,
// part) as the weight-gradient kernel) both read that staging. The separate kernels read dy twice from
// HBM (the input gradient's window, the weight gradient's tile) in two launches.
template <typename T>
__global__ __launch_bounds__(256) void dw7_bwd_fused_kernel(int B, int H, int W, int C, int tiles_h, int tiles_w,
                                                            int nsb, int slabs, const T* __restrict__ x, long ldx,
                                                            const T* __restrict__ dy, long lddy,
                                                            const float* __restrict__ w, T* __restrict__ dx, long lddx,
                                                            int accumulate, float* __restrict__ part) {
  constexpr int CPT = DwCfg<T>::CPT, CP = CPT / 2, NG = W7L_NG, TH = W7L_TH, TW = W7L_TW, NP = W7L_NP;
  constexpr int IH = W7L_IH, IW = W7L_IW, NXW = IH * (TW + 6) * NG;  // vectors of one staged window
  constexpr int NL = (2 * NXW + 255) / 256, NACT = NG * 7 * NP, BQ = 256 / NG;
  constexpr int HCP = sizeof(T) == 2 ? 2 : 1;  // channel pairs in half a vector (one 8-byte load)
  static_assert(NG * 2 * 2 * TH == 256, "input-gradient thread map");
  static_assert(TW == 14, "two 7-column strips per tile row");
  __shared__ uint4 xs[IH * IW * NG];
  __shared__ uint4 ds[IH * IW * NG];
  __shared__ float wl[49 * NG * CPT];  // the slab's taps, flipped (input gradient)
  const int ncv = C / CPT;
  const int lid = (int)xcd_remap(blockIdx.x, (long)nsb * slabs);
  const int sb = lid / slabs;
  const int cv0 = (lid % slabs) * NG;
  const long ntiles = (long)B * tiles_h * tiles_w;
  const int t = threadIdx.x;
  // weight gradient map (as dw7_lds_wgrad_kernel)
  const int g = t % NG, i = (t / NG) % 7, prt = t / (NG * 7);
  const bool active = t < NACT;
  // input gradient map: channel vector dg, half hf, 7-column strip st, tile row dr
  const int dg = t & 3, hf = (t >> 2) & 1, st = (t >> 3) & 1, dr = t >> 4;
  for (int e = t; e < 49 * NG * CPT; e += 256) {
    const int tap = e / (NG * CPT), c = cv0 * CPT + e % (NG * CPT);
    wl[e] = c < C ? w[(long)c * 49 + 48 - tap] : 0.f;
  }
  f2v acc[7][CP], bs[CP];
#pragma unroll
  for (int j = 0; j < 7; ++j)
#pragma unroll
    for (int e = 0; e < CP; ++e) acc[j][e] = f2v{0.f, 0.f};
#pragma unroll
  for (int e = 0; e < CP; ++e) bs[e] = f2v{0.f, 0.f};

  for (long tile = sb; tile < ntiles; tile += nsb) {
    const int tw = (int)(tile % tiles_w), th = (int)((tile / tiles_w) % tiles_h);
    const long b = tile / ((long)tiles_w * tiles_h);
    const int h0 = th * TH, w0 = tw * TW;
    const long img = b * H * W;
    uint4 buf[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int v = t + l * 256;
      buf[l] = make_uint4(0, 0, 0, 0);
      if (v < 2 * NXW) {
        const bool isx = v < NXW;
        const int u = isx ? v : v - NXW;
        const int gg = u % NG, col = (u / NG) % (TW + 6), row = u / (NG * (TW + 6));
        const int hh = h0 + row - 3, ww = w0 + col - 3, cv = cv0 + gg;
        if (hh >= 0 && hh < H && ww >= 0 && ww < W && cv < ncv) {
          const long pix = img + (long)hh * W + ww;
          buf[l] = isx ? *reinterpret_cast<const uint4*>(x + pix * ldx + cv * CPT)
                       : *reinterpret_cast<const uint4*>(dy + pix * lddy + cv * CPT);
        }
      }
    }
    __syncthreads();  // the previous tile's reads are done
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int v = t + l * 256;
      if (v < 2 * NXW) {
        const bool isx = v < NXW;
        const int u = isx ? v : v - NXW;
        const int gg = u % NG, col = (u / NG) % (TW + 6), row = u / (NG * (TW + 6));
        (isx ? xs : ds)[(row * IW + col) * NG + gg] = buf[l];
      }
    }
    __syncthreads();
    {  // bias gradient: thread (g, q) sums the tile's pixels q, q + BQ, ... of channel vector g
      for (int pix = t / NG; pix < TH * TW; pix += BQ) {
        f2v d[CP];
        unpack_pairs<T>(ds[((pix / TW + 3) * IW + pix % TW + 3) * NG + g], d);
#pragma unroll
        for (int e = 0; e < CP; ++e) bs[e] += d[e];
      }
    }
    {  // input gradient of output row h0 + dr, columns w0 + 7 st .. + 6, channels of half hf of vector dg
      f2v o[7][HCP];
#pragma unroll
      for (int q = 0; q < 7; ++q)
#pragma unroll
        for (int e = 0; e < HCP; ++e) o[q][e] = f2v{0.f, 0.f};
#pragma unroll 1
      for (int ki = 0; ki < 7; ++ki) {
        const uint2* dw_ = reinterpret_cast<const uint2*>(ds + ((dr + ki) * IW + 7 * st) * NG + dg) + hf;
        f2v win[13][HCP];
#pragma unroll
        for (int u = 0; u < 13; ++u) w3_pairs<T>(dw_[u * NG * 2], win[u]);
#pragma unroll
        for (int kj = 0; kj < 7; ++kj) {
          const float* wp = wl + (ki * 7 + kj) * NG * CPT + dg * CPT + hf * (CPT / 2);
          f2v wv[HCP];
#pragma unroll
          for (int e = 0; e < HCP; ++e) wv[e] = f2v{wp[2 * e], wp[2 * e + 1]};
#pragma unroll
          for (int q = 0; q < 7; ++q)
#pragma unroll
            for (int e = 0; e < HCP; ++e) o[q][e] = __builtin_elementwise_fma(wv[e], win[q + kj][e], o[q][e]);
        }
      }
      const int hh = h0 + dr;
      if (hh < H && cv0 + dg < ncv) {
        T* drow = dx + (img + (long)hh * W + w0 + 7 * st) * lddx + (cv0 + dg) * CPT + hf * (CPT / 2);
#pragma unroll
        for (int q = 0; q < 7; ++q) {
          if (w0 + 7 * st + q >= W) break;
          T* dp = drow + q * lddx;
          float ov[2 * HCP];
#pragma unroll
          for (int e = 0; e < HCP; ++e) {
            ov[2 * e] = o[q][e].x;
            ov[2 * e + 1] = o[q][e].y;
          }
          if (accumulate) {
            float pv[4];
            w3_unpack<T>(*reinterpret_cast<const uint2*>(dp), pv);
#pragma unroll
            for (int e = 0; e < 2 * HCP; ++e) ov[e] += pv[e];
          }
          w3_store<T>(dp, ov);
        }
      }
    }
    if (active) {  // weight gradient: kernel row i of channel vector g over tile rows prt, prt + NP
#pragma unroll 1
      for (int r = prt; r < TH; r += NP) {
        const uint4* xr = xs + ((r + i) * IW) * NG + g;
        const uint4* drr = ds + ((r + 3) * IW + 3) * NG + g;
        f2v xw[7][CP];  // ring: input column q of the row in slot q % 7
#pragma unroll
        for (int u = 0; u < 6; ++u) unpack_pairs<T>(xr[u * NG], xw[u]);
#pragma unroll 1
        for (int cb = 0; cb < TW; cb += 7) {
#pragma unroll
          for (int s7 = 0; s7 < 7; ++s7) {
            const int c = cb + s7;
            unpack_pairs<T>(xr[(c + 6) * NG], xw[(s7 + 6) % 7]);
            f2v d[CP];
            unpack_pairs<T>(drr[c * NG], d);
#pragma unroll
            for (int j = 0; j < 7; ++j)
#pragma unroll
              for (int e = 0; e < CP; ++e) acc[j][e] = __builtin_elementwise_fma(d[e], xw[(s7 + j) % 7][e], acc[j][e]);
          }
        }
      }
    }
  }
  // the NP parts of each (g, i) meet in LDS in part order, then part 0 writes the block's partial;
  // the bias partials of the BQ pixel lanes of each g likewise (lane order)
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);
  constexpr int RS = 7 * CPT + 1;
  for (int q = 1; q < NP; ++q) {
    if (active && prt == q) {
      float* o = red + (g * 7 + i) * RS;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int e = 0; e < CP; ++e) {
          o[j * CPT + 2 * e] = acc[j][e].x;
          o[j * CPT + 2 * e + 1] = acc[j][e].y;
        }
    }
    __syncthreads();
    if (active && prt == 0) {
      const float* o = red + (g * 7 + i) * RS;
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int e = 0; e < CP; ++e) acc[j][e] += f2v{o[j * CPT + 2 * e], o[j * CPT + 2 * e + 1]};
    }
    __syncthreads();
  }
  float* bred = red + NG * 7 * RS;  // [BQ][NG][CPT]
#pragma unroll
  for (int e = 0; e < CP; ++e) {
    bred[t * CPT + 2 * e] = bs[e].x;
    bred[t * CPT + 2 * e + 1] = bs[e].y;
  }
  __syncthreads();
  const long pbase = (long)sb * C * 50;
  if (active && prt == 0 && cv0 + g < ncv) {
#pragma unroll
    for (int e = 0; e < CP; ++e) {
      const int c = (cv0 + g) * CPT + 2 * e;
      float* o = part + pbase + (long)c * 50;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        o[i * 7 + j] = acc[j][e].x;
        o[50 + i * 7 + j] = acc[j][e].y;
      }
    }
  }
  if (t < NG * CPT) {  // bias: thread (g, e) sums the BQ lanes in order
    const int gg = t / CPT, e = t % CPT;
    if (cv0 + gg < ncv) {
      float sum = 0.f;
      for (int q = 0; q < BQ; ++q) sum += bred[(q * NG + gg) * CPT + e];
      part[pbase + (long)((cv0 + gg) * CPT + e) * 50 + 49] = sum;
    }
  }
}

template <typename T>
long w7l_nsb(int B, int H, int W, int C) {
  const long ntiles = (long)B * cdiv(H, W7L_TH) * cdiv(W, W7L_TW);
  const long slabs = cdiv(C / DwCfg<T>::CPT, W7L_NG);
  // one round of blocks: the kernel holds 2 blocks per CU (196 VGPRs), 512 on the chip (768 ran
  // 1.5 rounds: 459.8-460.7 vs 461.1-461.4 images/s)
  return std::max(1L, std::min(ntiles, (512 + slabs - 1) / slabs));
}

template <typename T>
long w7l_launch(int B, int H, int W, int C, const void* x, long ldx, const void* dy, long lddy, float* part,
                hipStream_t s) {
  const long nsb = w7l_nsb<T>(B, H, W, C);
  const unsigned slabs = cdiv(C / DwCfg<T>::CPT, W7L_NG);
  DFM_LAUNCH(dw7_lds_wgrad_kernel<T>, dim3((unsigned)(nsb * slabs)), dim3(256), 0, s, B, H, W, C, cdiv(H, W7L_TH),
             cdiv(W, W7L_TW), (int)nsb, (int)slabs, (const T*)x, ldx, (const T*)dy, lddy, part);
  return nsb;
}

template <typename T>
long b7_launch(int B, int H, int W, int C, const void* x, long ldx, const void* dy, long lddy, const float* w,
               void* dx, long lddx, int acc, float* part, hipStream_t s) {
  const long nsb = w7l_nsb<T>(B, H, W, C);
  const unsigned slabs = cdiv(C / DwCfg<T>::CPT, W7L_NG);
  DFM_LAUNCH(dw7_bwd_fused_kernel<T>, dim3((unsigned)(nsb * slabs)), dim3(256), 0, s, B, H, W, C, cdiv(H, W7L_TH),
             cdiv(W, W7L_TW), (int)nsb, (int)slabs, (const T*)x, ldx, (const T*)dy, lddy, w, (T*)dx, lddx, acc, part);
  return nsb;
}

// ---------------------------------------------------------------- row-streaming 3x3 forward / input gradient
// The forward counterpart of the streaming weight gradient: a lane owns one 8-byte channel vector
// and a TW-column strip, keeps its 9 taps + bias and the three input rows of the current output
// row in registers (the next input row is loaded one row ahead), and writes TW outputs per row
// (+ the fused identity, accumulate and GELU second output). No LDS, no block synchronisation.
template <typename T>
W3Geom f3_geom(int B, int H, int W, int C) {
  return w3_geom<T>(B, H, W, C, 2);
}


template <typename T, bool FLIP, bool BUF>
__global__ __launch_bounds__(256) void dw3_stream_fwd_kernel(int B, int H, int W, int C, int RC, int nstrips,
                                                             int nchunks, int LPU, int UPW,
                                                             const T* __restrict__ x, long ldx,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias, int add_identity,
                                                             T* __restrict__ y, long ldy, int accumulate,
                                                             T* __restrict__ gout, long ldg) {
  constexpr int CPT = W3Cfg<T>::EPL, CP = CPT / 2, TW = W3_TW, NX = TW + 2;
  constexpr unsigned ES = sizeof(T);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lg = lane % LPU, usub = lane / LPU;
  const int G = C / CPT, cg = blockIdx.y * LPU + lg;
  if (usub >= UPW || cg >= G) return;
  const int c0 = cg * CPT;
  const long units = w3_units(B, nstrips, nchunks);
  f2v wv[9][CP], bv[CP];  // channel pairs (packed FMA)
#pragma unroll
  for (int e = 0; e < CP; ++e) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      wv[tap][e] = f2v{w[(long)(c0 + 2 * e) * 9 + (FLIP ? 8 - tap : tap)], w[(long)(c0 + 2 * e + 1) * 9 + (FLIP ? 8 - tap : tap)]};
    bv[e] = bias ? f2v{bias[c0 + 2 * e], bias[c0 + 2 * e + 1]} : f2v{0.f, 0.f};
  }
  const long stride = (long)gridDim.x * 4 * UPW;
  const __amdgpu_buffer_rsrc_t xr_ = w3_rsrc(x, (long)B * H * W, ldx, C);
  const unsigned rstep = (unsigned)(W * ldx) * ES, cstep = (unsigned)ldx * ES;  // wave-uniform byte steps
  for (long u = ((long)blockIdx.x * 4 + wave) * UPW + usub; u < units; u += stride) {
    const int strip = (int)(u % nstrips), chunk = (int)((u / nstrips) % nchunks);
    const long b = u / ((long)nstrips * nchunks);
    const int w0 = strip * TW, h0 = chunk * RC, h1 = min(h0 + RC, H);
    const long img = b * H * W;
    unsigned cm = 0;  // in-image columns of the window
#pragma unroll
    for (int q = 0; q < NX; ++q) cm |= (unsigned)(w0 - 1 + q >= 0 && w0 - 1 + q < W) << q;
    // BUF: byte offset of (row h0 - 1, column w0 - 1); negative offsets wrap out of range and read zero
    unsigned xoff = (unsigned)(((img + (long)(h0 - 1) * W + w0 - 1) * ldx + c0) * (long)ES);
    auto load_x = [&](int h, uint2* r) -> unsigned {  // returns the row's keep mask
      const bool hok = h >= 0 && h < H;
      if constexpr (BUF) {
#pragma unroll
        for (int q = 0; q < NX; ++q) r[q] = w3_bld(xr_, xoff + q * cstep, 0u);
        xoff += rstep;
      } else {
        const int hc = hok ? h : h0;
#pragma unroll
        for (int q = 0; q < NX; ++q) r[q] = w3_ld<T>(x, ldx, img, W, hc, ((cm >> q) & 1u) ? w0 - 1 + q : w0, c0);
      }
      return hok ? cm : 0u;
    };
    uint2 x0[NX], x1[NX], x2[NX];
    w3_keep<NX>(x0, load_x(h0 - 1, x0));
    w3_keep<NX>(x1, load_x(h0, x1));
    unsigned m2 = load_x(h0 + 1, x2);
    T* yrow = y + (img + (long)h0 * W + w0) * ldy + c0;
    T* grow = gout ? gout + (img + (long)h0 * W + w0) * ldg + c0 : nullptr;
    for (int h = h0; h < h1; ++h, yrow += W * ldy, grow += gout ? W * ldg : 0) {
      w3_keep<NX>(x2, m2);  // the row loaded one iteration ago
      uint2 xn[NX];
      // the next row (its loads in flight during this row's FMAs); past the chunk it is not used
      m2 = load_x(BUF ? h + 2 : (h + 1 < h1 ? h + 2 : H), xn);
      f2v accp[TW][CP];
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int e = 0; e < CP; ++e) accp[t][e] = bv[e];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const uint2* xr = a == 0 ? x0 : (a == 1 ? x1 : x2);
#pragma unroll
        for (int q = 0; q < NX; ++q) {
          f2v xv[CP];
          w3_pairs<T>(xr[q], xv);
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const int j = q - t;
            if (j < 0 || j >= 3) continue;
#pragma unroll
            for (int e = 0; e < CP; ++e) accp[t][e] = __builtin_elementwise_fma(wv[a * 3 + j][e], xv[e], accp[t][e]);
          }
          if (q >= 1 && q <= TW && (add_identity & 1)) {
            if (a == 1) {
#pragma unroll
              for (int e = 0; e < CP; ++e) accp[q - 1][e] += xv[e];
            }
          }
        }
      }
      float acc[TW][CPT];
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int e = 0; e < CP; ++e) {
          acc[t][2 * e] = accp[t][e].x;
          acc[t][2 * e + 1] = accp[t][e].y;
        }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int ww = w0 + t;
        if (ww >= W) break;
        T* yp = yrow + t * ldy;
        if (accumulate) {
          float o[CPT];
          w3_unpack<T>(*reinterpret_cast<const uint2*>(yp), o);
#pragma unroll
          for (int e = 0; e < CPT; ++e) acc[t][e] += o[e];
        }
        if (gout) {  // GELU output; y holds the pre-activation or (flag 2) its GELU derivative
          float gv[CPT], dv[CPT];
          gelu_pairs<CPT>(acc[t], gv, dv);
          w3_store<T>(yp, (add_identity & 2) ? dv : acc[t]);
          w3_store<T>(grow + t * ldg, gv);
        } else {
          w3_store<T>(yp, acc[t]);
        }
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) {
        x0[q] = x1[q];
        x1[q] = x2[q];
        x2[q] = xn[q];
      }
    }
  }
}

template <typename T, bool FLIP>
int f3_launch(int B, int H, int W, int C, const void* x, long ldx, const float* w, const float* bias, int id,
              void* y, long ldy, int acc, void* gout, long ldg, hipStream_t s) {
  const W3Geom g = f3_geom<T>(B, H, W, C);
  auto kern = w3_buf_ok<T>((long)B * H * W, ldx, C) ? dw3_stream_fwd_kernel<T, FLIP, true>
                                                    : dw3_stream_fwd_kernel<T, FLIP, false>;
  DFM_LAUNCH(kern, dim3((unsigned)g.nsb, (unsigned)g.slices), dim3(256), 0, s, B, H, W, C, g.RC, g.nstrips,
             g.nchunks, g.LPU, g.UPW, (const T*)x, ldx, w, bias, id, (T*)y, ldy, acc, (T*)gout, ldg);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ---------------------------------------------------------------- fused 3x3 backward (data + weight)
// The ConvFFN's depthwise 3x3 + identity backward (DFormer.py:54,62) in ONE pass over dy and x:
//   dx[h][w] (+)= sum_taps w[2-a][2-j] dy[h+a-1][w+j-1] + dy[h][w]     (identity)
//   dw[a][j] += dy[h][w] x[h+a-1][w+j-1],  db += dy[h][w]              (per-block partials)
// The separate kernels read dy twice (input gradient, weight gradient) and x once; here each lane
// (one 8-byte channel vector, a TW-column strip walking a chunk of RC rows as in the streaming
// weight gradient) keeps the three dy rows and the three x rows around output row h in registers,
// loading the next row of each one ahead. dy is read once from HBM (its halo rows / columns from
// L2), x once, dx written once. All FMAs are packed (v_pk_fma_f32 over channel pairs).
template <typename T>
__global__ __launch_bounds__(256) void dw3_stream_bwd_kernel(int B, int H, int W, int C, int RC, int nstrips,
                                                             int nchunks, int LPU, int UPW,
                                                             const T* __restrict__ x, long ldx,
                                                             const T* __restrict__ dy, long lddy,
                                                             const float* __restrict__ w, int add_identity,
                                                             T* __restrict__ dx, long lddx, int accumulate,
                                                             float* __restrict__ part) {
  constexpr int CPT = W3Cfg<T>::EPL, CP = CPT / 2, TW = W3_TW, NX = TW + 2, NV = 10 * CPT, VCH = 20;
  __shared__ float red[4][VCH][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lg = lane % LPU, usub = lane / LPU;
  const int G = C / CPT, cg = blockIdx.y * LPU + lg;
  const bool valid = usub < UPW && cg < G;
  const int c0 = cg * CPT;
  const long units = w3_units(B, nstrips, nchunks);

  f2v wf[9][CP];  // flipped taps (input gradient), centre tap + 1 when add_identity
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int e = 0; e < CP; ++e) {
      const float idt = (tap == 4 && add_identity) ? 1.0f : 0.0f;
      wf[tap][e] = valid ? f2v{w[(long)(c0 + 2 * e) * 9 + 8 - tap] + idt, w[(long)(c0 + 2 * e + 1) * 9 + 8 - tap] + idt}
                         : f2v{0.f, 0.f};
    }
  f2v acc[10][CP];
#pragma unroll
  for (int a = 0; a < 10; ++a)
#pragma unroll
    for (int e = 0; e < CP; ++e) acc[a][e] = f2v{0.f, 0.f};

  const long stride = (long)gridDim.x * 4 * UPW;
  for (long u = ((long)blockIdx.x * 4 + wave) * UPW + usub; valid && u < units; u += stride) {
    const int strip = (int)(u % nstrips), chunk = (int)((u / nstrips) % nchunks);
    const long b = u / ((long)nstrips * nchunks);
    const int w0 = strip * TW, h0 = chunk * RC, h1 = min(h0 + RC, H);
    const long img = b * H * W;
    unsigned cm = 0;  // in-image columns of the window
#pragma unroll
    for (int q = 0; q < NX; ++q) cm |= (unsigned)(w0 - 1 + q >= 0 && w0 - 1 + q < W) << q;
    // columns w0-1 .. w0+TW of row h; returns the row's keep mask (zero outside the image)
    auto load_row = [&](const T* src, long ld, int h, uint2* r) -> unsigned {
      const bool hok = h >= 0 && h < H;
      const int hc = hok ? h : h0;
#pragma unroll
      for (int q = 0; q < NX; ++q) r[q] = w3_ld<T>(src, ld, img, W, hc, ((cm >> q) & 1u) ? w0 - 1 + q : w0, c0);
      return hok ? cm : 0u;
    };
    uint2 x0[NX], x1[NX], x2[NX], d0[NX], d1[NX], d2[NX];
    w3_keep<NX>(x0, load_row(x, ldx, h0 - 1, x0));
    w3_keep<NX>(x1, load_row(x, ldx, h0, x1));
    unsigned m2 = load_row(x, ldx, h0 + 1, x2);
    w3_keep<NX>(d0, load_row(dy, lddy, h0 - 1, d0));
    w3_keep<NX>(d1, load_row(dy, lddy, h0, d1));
    unsigned m2d = load_row(dy, lddy, h0 + 1, d2);
    for (int h = h0; h < h1; ++h) {
      w3_keep<NX>(x2, m2);  // the rows loaded one iteration ago
      w3_keep<NX>(d2, m2d);
      uint2 xn[NX], dn[NX];
      const int hn = h + 1 < h1 ? h + 2 : H;  // row H (and any row past the chunk) reads as zeros
      m2 = load_row(x, ldx, hn, xn);
      m2d = load_row(dy, lddy, hn, dn);
      f2v o[TW][CP];
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int e = 0; e < CP; ++e) o[t][e] = f2v{0.f, 0.f};
      // weight gradient: the centre dy row against the three x rows
      f2v gc[TW][CP];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        w3_pairs<T>(d1[t + 1], gc[t]);
#pragma unroll
        for (int e = 0; e < CP; ++e) acc[9][e] += gc[t][e];
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const uint2* xr = a == 0 ? x0 : (a == 1 ? x1 : x2);
        const uint2* dr = a == 0 ? d0 : (a == 1 ? d1 : d2);
#pragma unroll
        for (int q = 0; q < NX; ++q) {
          f2v xv[CP], dv[CP];
          w3_pairs<T>(xr[q], xv);
          w3_pairs<T>(dr[q], dv);
          // input column q feeds output column t with tap j = q - t
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const int j = q - t;
            if (j < 0 || j >= 3) continue;
#pragma unroll
            for (int e = 0; e < CP; ++e) {
              acc[a * 3 + j][e] = __builtin_elementwise_fma(gc[t][e], xv[e], acc[a * 3 + j][e]);
              o[t][e] = __builtin_elementwise_fma(wf[a * 3 + j][e], dv[e], o[t][e]);
            }
          }
        }
      }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int ww = w0 + t;
        if (ww >= W) break;
        T* dp = dx + (img + (long)h * W + ww) * lddx + c0;
        float ov[CPT];
#pragma unroll
        for (int e = 0; e < CP; ++e) {
          ov[2 * e] = o[t][e].x;
          ov[2 * e + 1] = o[t][e].y;
        }
        if (accumulate) {
          float pv[CPT];
          w3_unpack<T>(*reinterpret_cast<const uint2*>(dp), pv);
#pragma unroll
          for (int e = 0; e < CPT; ++e) ov[e] += pv[e];
        }
        w3_store<T>(dp, ov);
      }
#pragma unroll
      for (int q = 0; q < NX; ++q) {
        x0[q] = x1[q];
        x1[q] = x2[q];
        x2[q] = xn[q];
        d0[q] = d1[q];
        d1[q] = d2[q];
        d2[q] = dn[q];
      }
    }
  }

  // block reduction over the 4 waves and the UPW units of a wave that share a channel vector
  const long pbase = (long)blockIdx.x * C * 10;
#pragma unroll
  for (int vc = 0; vc < NV; vc += VCH) {
    if (vc) __syncthreads();
#pragma unroll
    for (int v = 0; v < VCH; ++v)
      if (vc + v < NV) {
        const int V = vc + v, e = V % CPT;
        const f2v pr = acc[V / CPT][e / 2];
        red[wave][v][lane] = (e & 1) ? pr.y : pr.x;
      }
    __syncthreads();
    for (int idx = threadIdx.x; idx < VCH * LPU; idx += 256) {
      const int v = idx / LPU, l = idx % LPU, V = vc + v;
      const int c = (blockIdx.y * LPU + l) * CPT + V % CPT;
      if (V >= NV || c >= C) continue;
      float sum = 0.f;
      for (int wv = 0; wv < 4; ++wv)
        for (int us = 0; us < UPW; ++us) sum += red[wv][v][us * LPU + l];
      part[pbase + (long)c * 10 + V / CPT] = sum;
    }
  }
}

// ---------------------------------------------------------------- fused 3x3 backward, row scatter
// The same sums as dw3_stream_bwd_kernel with every input row unpacked ONCE: a lane owns one channel
// pair (4 bytes of bf16 / f16) and walks the input rows r = h0-1 .. h1+1 of its unit. dy row r is
// scattered into the three pending input-gradient rows it feeds (r-1 completes and is stored, r + 1
// starts); x row r-1 meets the unpacked centre columns of dy rows r-2 .. r (kept from their own
// steps) for the weight gradient. The gather form above re-unpacks its three-row windows for every
// output row (3x the unpack work, ~1.3 unpack / address instructions per packed FMA); here a step is
// 72 packed FMAs against 12 loads and 12 unpacks. Pending rows rotate with period 3; the loop is
// unrolled by 3 so the rotation is register renaming, not moves. 135 VGPRs (the 8-byte-lane kernel:
// 250), so 3 waves per SIMD. Units are wave-uniform (whole 64-lane channel slices), so the row / column
// bookkeeping is scalar. Isolated (tools/ffn_kernels_bench.py, DFormer-B bs 16): s0 234 vs 244 us, s1
// 135 vs 138, s2 34.2 vs 39.2, s3 25.9 vs 30.2 (mlp; mlp_e2 alike); step 480.4 / 482.0 vs 476.5 / 477.1.
template <typename T> struct W3Pair { using type = uint32_t; };
template <> struct W3Pair<float> { using type = uint2; };

template <typename T>
DFM_INLINE f2v w3p_unpack(typename W3Pair<T>::type q) {
  if constexpr (std::is_same<T, f16_t>::value) return f2v{h2f((uint16_t)(q & 0xffffu)), h2f((uint16_t)(q >> 16))};
  else if constexpr (sizeof(T) == 2) return f2v{__uint_as_float(q << 16), __uint_as_float(q & 0xffff0000u)};
  else return f2v{__uint_as_float(q.x), __uint_as_float(q.y)};
}
template <typename T>
DFM_INLINE typename W3Pair<T>::type w3p_pack(f2v v) {
  if constexpr (sizeof(T) == 2) return (uint32_t)bits16<T>(v.x) | ((uint32_t)bits16<T>(v.y) << 16);
  else return make_uint2(__float_as_uint(v.x), __float_as_uint(v.y));
}
template <typename P>
DFM_INLINE P w3p_zero() {
  if constexpr (sizeof(P) == 4) return 0u;
  else return make_uint2(0u, 0u);
}

template <typename T>
__global__ __launch_bounds__(256, 3) void dw3_rows_bwd_kernel(int B, int H, int W, int C, int RC, int nstrips,
                                                           int nchunks, const T* __restrict__ x, long ldx,
                                                           const T* __restrict__ dy, long lddy,
                                                           const float* __restrict__ w, int add_identity,
                                                           T* __restrict__ dx, long lddx, int accumulate,
                                                           float* __restrict__ part) {
  using P = typename W3Pair<T>::type;
  constexpr int TW = W3_TW, NX = TW + 2, NV = 20;
  constexpr long ES = sizeof(T);
  __shared__ float red[4][NV][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // every lane owns a channel pair; lanes past C (a partial last slice) read the last pair and store nothing
  const int cq = (blockIdx.y * 64 + lane) * 2;
  const bool cvalid = cq < C;
  const int c0 = cvalid ? cq : C - 2;
  const long units = w3_units(B, nstrips, nchunks);

  f2v wf[9];  // flipped taps (input gradient), centre tap + 1 when add_identity
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const float idt = (tap == 4 && add_identity) ? 1.0f : 0.0f;
    wf[tap] = f2v{w[(long)c0 * 9 + 8 - tap] + idt, w[(long)(c0 + 1) * 9 + 8 - tap] + idt};
  }
  f2v acc[10];
#pragma unroll
  for (int a = 0; a < 10; ++a) acc[a] = f2v{0.f, 0.f};
  const unsigned c0b = (unsigned)(c0 * ES);  // the lane's byte offset in a pixel; the rest of every address is scalar

  // units are wave-uniform: row / column bookkeeping and the row and column base addresses are scalar,
  // so a load is one scalar address plus the lane's channel offset (global_load saddr + voffset)
  for (long u = (long)blockIdx.x * 4 + wave; u < units; u += (long)gridDim.x * 4) {
    const int strip = (int)(u % nstrips), chunk = (int)((u / nstrips) % nchunks);
    const long b = u / ((long)nstrips * nchunks);
    const int w0 = strip * TW, h0 = chunk * RC, h1 = min(h0 + RC, H);
    unsigned cm = 0;  // in-image window columns (out-of-image ones read column w0 and are zeroed)
    long xcol[NX], ycol[NX];
#pragma unroll
    for (int q = 0; q < NX; ++q) {
      const bool in = w0 - 1 + q >= 0 && w0 - 1 + q < W;
      cm |= (unsigned)in << q;
      const long cc = in ? w0 - 1 + q : w0;
      xcol[q] = cc * ldx * ES;
      ycol[q] = cc * lddy * ES;
    }
    const bool edge = cm != (1u << NX) - 1;
    const char* xim = reinterpret_cast<const char*>(x + b * H * W * ldx);
    const char* yim = reinterpret_cast<const char*>(dy + b * H * W * lddy);
    auto fetch = [&](const char* im, long ld, const long* col, int h, P* r) -> bool {
      const bool ok = h >= 0 && h < H;
      const char* rp = im + (long)(ok ? h : h0) * W * ld * ES;
#pragma unroll
      for (int q = 0; q < NX; ++q) r[q] = *reinterpret_cast<const P*>(rp + col[q] + c0b);
      return ok;
    };
    auto unpack_row = [&](const P* r, bool ok, f2v* v) {
      if (ok && !edge) {
#pragma unroll
        for (int q = 0; q < NX; ++q) v[q] = w3p_unpack<T>(r[q]);
      } else {
#pragma unroll
        for (int q = 0; q < NX; ++q) v[q] = (ok && ((cm >> q) & 1u)) ? w3p_unpack<T>(r[q]) : f2v{0.f, 0.f};
      }
    };
    // one packed row buffer per operand: a step unpacks the row fetched by the previous step, then
    // fetches the next one into the same registers (its latency hides under this step's FMAs)
    P D[NX], X[NX];
    bool dok, xok = false;
    f2v O[3][TW], Cc[3][TW];  // pending input-gradient rows; unpacked dy centre columns (chunk rows only)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int t = 0; t < TW; ++t) O[i][t] = Cc[i][t] = f2v{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NX; ++q) X[q] = w3p_zero<P>();
    dok = fetch(yim, lddy, ycol, h0 - 1, D);
    int r = h0 - 1;
    // step r (k = (r - h0 + 1) % 3): D holds dy row r, X x row r - 1; fetches dy row r + 1 and x row r.
    // Rows past h1 + 1 / h1 are never used for anything that is kept.
    auto step = [&](auto kc) {
      constexpr int k = decltype(kc)::value, k1 = (k + 1) % 3, k2 = (k + 2) % 3;
      f2v dv[NX], xv[NX];
      unpack_row(D, dok, dv);
      dok = fetch(yim, lddy, ycol, r + 1, D);
      unpack_row(X, xok, xv);
      xok = fetch(xim, ldx, xcol, r, X);
      // dy row r feeds input-gradient rows r - 1 (taps a = 2), r (a = 1), r + 1 (a = 0, the row's first)
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        O[k1][t] = wf[0] * dv[t];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          O[k2][t] = __builtin_elementwise_fma(wf[6 + j], dv[t + j], O[k2][t]);
          O[k][t] = __builtin_elementwise_fma(wf[3 + j], dv[t + j], O[k][t]);
          if (j) O[k1][t] = __builtin_elementwise_fma(wf[j], dv[t + j], O[k1][t]);
        }
      }
      if (r >= h0 && r < h1) {  // dy rows of this chunk carry the weight gradient
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          Cc[k][t] = dv[t + 1];
          acc[9] += dv[t + 1];
        }
      } else {
#pragma unroll
        for (int t = 0; t < TW; ++t) Cc[k][t] = f2v{0.f, 0.f};
      }
      // x row r - 1 against dy rows r (a = 0), r - 1 (a = 1), r - 2 (a = 2)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int cr = a == 0 ? k : (a == 1 ? k2 : k1);
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int t = 0; t < TW; ++t) acc[a * 3 + j] = __builtin_elementwise_fma(Cc[cr][t], xv[t + j], acc[a * 3 + j]);
      }
      // input-gradient row r - 1 is complete
      if (r - 1 >= h0 && r - 1 < h1 && cvalid) {
        char* dp = reinterpret_cast<char*>(dx + ((b * H + r - 1) * W + w0) * lddx);
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          if (w0 + t >= W) break;
          P* op = reinterpret_cast<P*>(dp + t * lddx * ES + c0b);
          f2v v = O[k2][t];
          if (accumulate) v += w3p_unpack<T>(*op);
          *op = w3p_pack<T>(v);
        }
      }
    };
    for (;;) {
      step(std::integral_constant<int, 0>{});
      if (++r > h1 + 1) break;
      step(std::integral_constant<int, 1>{});
      if (++r > h1 + 1) break;
      step(std::integral_constant<int, 2>{});
      if (++r > h1 + 1) break;
    }
  }

  // block reduction over the 4 waves
  const long pbase = (long)blockIdx.x * C * 10;
#pragma unroll
  for (int v = 0; v < NV; ++v) red[wave][v][lane] = (v & 1) ? acc[v >> 1].y : acc[v >> 1].x;
  __syncthreads();
  for (int idx = threadIdx.x; idx < NV * 64; idx += 256) {
    const int v = idx / 64, l = idx % 64;
    const int c = (blockIdx.y * 64 + l) * 2 + (v & 1);
    if (c < C) part[pbase + (long)c * 10 + (v >> 1)] = red[0][v][l] + red[1][v][l] + red[2][v][l] + red[3][v][l];
  }
}

// waves per SIMD of dw3_rows_bwd_kernel (135 VGPRs; its geometry's round size). Capped at 4 (128 VGPRs)
// it spills and is 10-22 % slower (s0 286 vs 234 us; step 470.2 vs 480.8 images/s)
constexpr int W3R_WPS = 3;

// the row-scatter kernel: 64-lane channel slices (wave-uniform units; a partial last slice only from 384
// channels, where it idles at most a sixth of the lanes: DFormer-Large's 576), 32-bit byte offsets in a row
inline bool w3r_ok(int W, int C, long ldx, long lddy, long lddx, long es) {
  return (C % 128 == 0 || (C % 2 == 0 && C >= 384)) && (long)W * std::max({ldx, lddy, lddx}) * es < (1L << 31);
}

template <typename T>
long b3_launch(int B, int H, int W, int C, const void* x, long ldx, const void* dy, long lddy, const float* w,
               int id, void* dx, long lddx, int acc, float* part, hipStream_t s) {
  if (w3r_ok(W, C, ldx, lddy, lddx, sizeof(T))) {
    const W3Geom g = w3_geom_cpl(B, H, W, C, 2, W3R_WPS);
    DFM_LAUNCH((dw3_rows_bwd_kernel<T>), dim3((unsigned)g.nsb, (unsigned)g.slices), dim3(256), 0, s, B, H, W, C,
               g.RC, g.nstrips, g.nchunks, (const T*)x, ldx, (const T*)dy, lddy, w, id, (T*)dx, lddx, acc, part);
    return g.nsb;
  }
  const W3Geom g = w3_geom<T>(B, H, W, C);
  DFM_LAUNCH((dw3_stream_bwd_kernel<T>), dim3((unsigned)g.nsb, (unsigned)g.slices), dim3(256), 0, s, B, H, W, C,
                     g.RC, g.nstrips, g.nchunks, g.LPU, g.UPW, (const T*)x, ldx, (const T*)dy, lddy, w, id,
                     (T*)dx, lddx, acc, part);
  return g.nsb;
}

template <typename T>
bool dw_aligned(int C, const void* p, long ld) {
  constexpr int CPT = DwCfg<T>::CPT;
  return C % CPT == 0 && ld % CPT == 0 && ((uintptr_t)p % 16) == 0;
}

template <typename T, int K, bool FLIP, int NG, int VAR = 0>
int dw_tile_launch(int B, int H, int W, int C, const void* x, long ldx, const float* w, const float* bias, int id,
                   void* y, long ldy, int acc, void* gout, long ldg, hipStream_t s) {
  constexpr int CPT = DwCfg<T>::CPT, TWS = DwFwdTile<T, K, VAR>::TWS, STRIPS = DwFwdTile<T, K, VAR>::STRIPS;
  constexpr int TH = 256 / (NG * STRIPS), TWT = TWS * STRIPS;
  const int tiles_h = (H + TH - 1) / TH, tiles_w = (W + TWT - 1) / TWT;
  const int G = C / CPT;
  dim3 grid((unsigned)((long)B * tiles_h * tiles_w * cdiv(G, NG)));
  const size_t lds = (size_t)(TH + K - 1) * (TWT + K - 1) * NG * 16 + (size_t)K * K * NG * CPT * sizeof(float);
  if (lds > 64 * 1024) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)dw_tile_fwd_kernel<T, K, FLIP, NG, VAR>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
  }
  DFM_LAUNCH((dw_tile_fwd_kernel<T, K, FLIP, NG, VAR>), grid, dim3(256), lds, s, B, H, W, C, tiles_h, tiles_w,
                     (const T*)x, ldx, w, bias, id, (T*)y, ldy, acc, (T*)gout, ldg);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, bool FLIP>
int dw_fwd(int B, int H, int W, int C, int k, const void* x, long ldx, const float* w, const float* bias, int id,
           void* y, long ldy, int acc, void* gout, long ldg, hipStream_t s) {
  DFM_CHECK_ARG(dw_aligned<T>(C, x, ldx) && dw_aligned<T>(C, y, ldy) && (!gout || dw_aligned<T>(C, gout, ldg)),
                "dwconv: C, row strides and pointers must be 16-byte vector aligned");
  DFM_CHECK_ARG(k == 3 || k == 7, "dwconv: k=%d unsupported", k);
  // streaming 3x3 up to 65,536-pixel planes: with its buffer-addressed loads (round 6) it also wins on
  // DFormer-Large's 133x183 stage-0 planes (config 5: 274.1 / 275.7 -> 276.6 / 279.5 images/s; DFormer-B
  // and -Tiny, whose stage-0 ConvFFN forward is the fused kernel, within noise). Round 4 had the LDS-tiled
  // kernel ahead on 120x160 (302 vs 328 us at 512 channels, profiles/r04_dw3_geom_sweep.txt).
  const long plane = (long)H * W;
  if (k == 3 && plane <= 65536) return f3_launch<T, FLIP>(B, H, W, C, x, ldx, w, bias, id, y, ldy, acc, gout, ldg, s);
  const int G = C / DwCfg<T>::CPT;
  // channel groups per block: as many as the tile geometry allows without idling lanes
#define GO(KK, NGV) return dw_tile_launch<T, KK, FLIP, NGV>(B, H, W, C, x, ldx, w, bias, id, y, ldy, acc, gout, ldg, s)
  if (k == 3) {
    // 64-channel groups (whole 128-byte lines per pixel) on the 120x160 planes: 297-300 vs 307 us at
    // 512 channels, 128-129 vs 138 at 256 (4 x 32 tiles; 16 x 16 tiles with 8 outputs per thread
    // hold 169 VGPRs and lose, profiles/r04_dw3_geom_sweep.txt)
    if (G >= 8) GO(3, 8);
    if (G >= 4) GO(3, 4);
    if (G >= 2) GO(3, 2);
    GO(3, 1);
  }
  // (8 outputs per thread along the row, VAR 1: 467.1 / 465.9 vs 468.3 / 468.7 images/s)
  if (G >= 8) GO(7, 8);
  if (G >= 4) GO(7, 4);
  if (G >= 2) GO(7, 2);
  GO(7, 1);
#undef GO
}

}  // namespace

extern "C" int dfm_dwconv_fwd(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx, const float* w,
                              const float* bias, int add_identity, void* y, long ldy, void* gout, long ldg,
                              dfm_stream_t stream) {
  DFM_CHECK_ARG(x && w && y && B > 0 && H > 0 && W > 0 && C > 0, "dfm_dwconv_fwd: bad argument");
  if (dtype == DFM_BF16) return dw_fwd<bf16_t, false>(B, H, W, C, k, x, ldx, w, bias, add_identity, y, ldy, 0, gout, ldg, (hipStream_t)stream);
  else if (dtype == DFM_F16) return dw_fwd<f16_t, false>(B, H, W, C, k, x, ldx, w, bias, add_identity, y, ldy, 0, gout, ldg, (hipStream_t)stream);
  if (dtype == DFM_F32) return dw_fwd<float, false>(B, H, W, C, k, x, ldx, w, bias, add_identity, y, ldy, 0, gout, ldg, (hipStream_t)stream);
  dfm_set_error("dfm_dwconv_fwd: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_dwconv_bwd_data(int dtype, int B, int H, int W, int C, int k, const void* dy, long lddy,
                                   const float* w, int add_identity, void* dx, long lddx, int accumulate,
                                   dfm_stream_t stream) {
  DFM_CHECK_ARG(dy && w && dx && B > 0 && H > 0 && W > 0 && C > 0, "dfm_dwconv_bwd_data: bad argument");
  if (dtype == DFM_BF16)
    return dw_fwd<bf16_t, true>(B, H, W, C, k, dy, lddy, w, nullptr, add_identity, dx, lddx, accumulate, nullptr, 0,
                                (hipStream_t)stream);
  else if (dtype == DFM_F16)
    return dw_fwd<f16_t, true>(B, H, W, C, k, dy, lddy, w, nullptr, add_identity, dx, lddx, accumulate, nullptr, 0,
                                (hipStream_t)stream);
  if (dtype == DFM_F32)
    return dw_fwd<float, true>(B, H, W, C, k, dy, lddy, w, nullptr, add_identity, dx, lddx, accumulate, nullptr, 0,
                               (hipStream_t)stream);
  dfm_set_error("dfm_dwconv_bwd_data: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" size_t dfm_dwconv_bwd_weight_workspace(int B, int H, int W, int C, int k) {
  long nsb = 1;
  if (k == 3)
    for (int occ = 2; occ <= 3; ++occ)  // fused backward (2 waves / SIMD), weight gradient alone (3)
      nsb = std::max({nsb, w3_geom<float>(B, H, W, C, occ).nsb, w3_geom<bf16_t>(B, H, W, C, occ).nsb,
                      w3_geom_cpl(B, H, W, C, 2, W3R_WPS).nsb});  // (row-scatter fused backward)
  else if (k == 7)
    nsb = std::max(w7l_nsb<float>(B, H, W, C), w7l_nsb<bf16_t>(B, H, W, C));
  return (size_t)nsb * C * (k * k + 1) * sizeof(float);
}

extern "C" int dfm_dwconv_bwd(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx,
                              const void* dy, long lddy, const float* w, int add_identity, void* dx, long lddx,
                              int accumulate, float* dw, float* db, void* workspace, DfmPartialSum* defer,
                              dfm_stream_t stream) {
  if (defer) *defer = DfmPartialSum{};
  DFM_CHECK_ARG(x && dy && w && dx && dw && workspace, "dfm_dwconv_bwd: null argument");
  DFM_CHECK_ARG(k == 3 || (k == 7 && !add_identity), "dfm_dwconv_bwd: k=%d%s unsupported", k,
                add_identity ? " with identity" : "");
  DFM_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0, "dfm_dwconv_bwd: bad shape");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  long nsb;
  if (k == 7) {  // one pass over dy for the input and the weight gradient (dw7_bwd_fused_kernel)
    if (dtype == DFM_BF16) {
      DFM_CHECK_ARG(dw_aligned<bf16_t>(C, x, ldx) && dw_aligned<bf16_t>(C, dy, lddy) && dw_aligned<bf16_t>(C, dx, lddx),
                    "dfm_dwconv_bwd: alignment");
      nsb = b7_launch<bf16_t>(B, H, W, C, x, ldx, dy, lddy, w, dx, lddx, accumulate, part, s);
    } else if (dtype == DFM_F16) {
      DFM_CHECK_ARG(dw_aligned<f16_t>(C, x, ldx) && dw_aligned<f16_t>(C, dy, lddy) && dw_aligned<f16_t>(C, dx, lddx),
                    "dfm_dwconv_bwd: alignment");
      nsb = b7_launch<f16_t>(B, H, W, C, x, ldx, dy, lddy, w, dx, lddx, accumulate, part, s);
    } else if (dtype == DFM_F32) {
      DFM_CHECK_ARG(dw_aligned<float>(C, x, ldx) && dw_aligned<float>(C, dy, lddy) && dw_aligned<float>(C, dx, lddx),
                    "dfm_dwconv_bwd: alignment");
      nsb = b7_launch<float>(B, H, W, C, x, ldx, dy, lddy, w, dx, lddx, accumulate, part, s);
    } else {
      dfm_set_error("dfm_dwconv_bwd: bad dtype");
      return DFM_ERR_DTYPE;
    }
    DFM_LAUNCH_CHECK();
    return second_stage(2, (int)nsb, (long)C * 50, part, dw, db, 50L, 0, defer, s);
  }
  if (dtype == DFM_BF16) {
    DFM_CHECK_ARG(dw_aligned<bf16_t>(C, x, ldx) && dw_aligned<bf16_t>(C, dy, lddy) && dw_aligned<bf16_t>(C, dx, lddx),
                  "dfm_dwconv_bwd: alignment");
    nsb = b3_launch<bf16_t>(B, H, W, C, x, ldx, dy, lddy, w, add_identity, dx, lddx, accumulate, part, s);
  } else if (dtype == DFM_F16) {
    DFM_CHECK_ARG(dw_aligned<f16_t>(C, x, ldx) && dw_aligned<f16_t>(C, dy, lddy) && dw_aligned<f16_t>(C, dx, lddx),
                  "dfm_dwconv_bwd: alignment");
    nsb = b3_launch<f16_t>(B, H, W, C, x, ldx, dy, lddy, w, add_identity, dx, lddx, accumulate, part, s);
  } else if (dtype == DFM_F32) {
    DFM_CHECK_ARG(dw_aligned<float>(C, x, ldx) && dw_aligned<float>(C, dy, lddy) && dw_aligned<float>(C, dx, lddx),
                  "dfm_dwconv_bwd: alignment");
    nsb = b3_launch<float>(B, H, W, C, x, ldx, dy, lddy, w, add_identity, dx, lddx, accumulate, part, s);
  } else {
    dfm_set_error("dfm_dwconv_bwd: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return second_stage(2, (int)nsb, (long)C * 10, part, dw, db, 10L, 0, defer, s);
}

extern "C" int dfm_dwconv_bwd_weight(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx,
                                     const void* dy, long lddy, float* dw, float* db, void* workspace,
                                     DfmPartialSum* defer, dfm_stream_t stream) {
  if (defer) *defer = DfmPartialSum{};
  DFM_CHECK_ARG(x && dy && dw && workspace, "dfm_dwconv_bwd_weight: null argument");
  DFM_CHECK_ARG(k == 3 || k == 7, "dfm_dwconv_bwd_weight: k=%d unsupported", k);
  DFM_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0, "dfm_dwconv_bwd_weight: bad shape");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  long nsb;
  if (dtype == DFM_BF16) {
    DFM_CHECK_ARG(dw_aligned<bf16_t>(C, x, ldx) && dw_aligned<bf16_t>(C, dy, lddy), "dwconv wgrad: alignment");
    nsb = k == 7 ? w7l_launch<bf16_t>(B, H, W, C, x, ldx, dy, lddy, part, s)
                 : w3_launch<bf16_t>(B, H, W, C, x, ldx, dy, lddy, part, s);
  }
  else if (dtype == DFM_F16) {
    DFM_CHECK_ARG(dw_aligned<f16_t>(C, x, ldx) && dw_aligned<f16_t>(C, dy, lddy), "dwconv wgrad: alignment");
    nsb = k == 7 ? w7l_launch<f16_t>(B, H, W, C, x, ldx, dy, lddy, part, s)
                 : w3_launch<f16_t>(B, H, W, C, x, ldx, dy, lddy, part, s);
  } else if (dtype == DFM_F32) {
    DFM_CHECK_ARG(dw_aligned<float>(C, x, ldx) && dw_aligned<float>(C, dy, lddy), "dwconv wgrad: alignment");
    nsb = k == 7 ? w7l_launch<float>(B, H, W, C, x, ldx, dy, lddy, part, s)
                 : w3_launch<float>(B, H, W, C, x, ldx, dy, lddy, part, s);
  } else {
    dfm_set_error("dfm_dwconv_bwd_weight: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return second_stage(2, (int)nsb, (long)C * (k * k + 1), part, dw, db, (long)(k * k + 1), 0, defer, s);
}
