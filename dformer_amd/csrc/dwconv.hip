// Depthwise k x k convolution over NHWC (DFormer.py:80-81 7x7 conv/e_conv, DFormer.py:54,62 3x3
// pos + identity), forward / input-gradient / weight-gradient.
//
// HBM-bound. Every thread owns CPT consecutive channels (one 16-byte vector: 8 bf16 or 4 fp32)
// of a TW-pixel strip of one output row; input rows are streamed as 16-byte vectors through a
// register sliding window (neighbouring strips share their halo through L1/L2, so HBM sees each
// byte about once). A block covers GPB channel groups x SPB strips; the block's k*k weights live
// in LDS transposed to [k*k][channels] so each tap is one vector LDS read.
// The weight gradient accumulates per thread over many strips, reduces across the block's strip
// lanes in LDS, writes per-block partials [block][C][k*k+1] (last column: bias grad) and sums
// them in a fixed order (deterministic, no float atomics).
#include "common.h"

namespace {
constexpr int TW = 4;

template <typename T> struct DwCfg { static constexpr int CPT = 16 / sizeof(T); };

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

struct DwGeom {
  int G;       // channel groups (C / CPT)
  int GPB;     // groups per block
  int SPB;     // strip lanes per block
  int nstrip;  // strips per row
  long strips; // B * H * nstrip
};

template <typename T>
DwGeom dw_geom(int B, int H, int W, int C) {
  constexpr int CPT = DwCfg<T>::CPT;
  DwGeom g;
  g.G = C / CPT;
  g.GPB = g.G < 32 ? g.G : 32;
  g.SPB = 256 / g.GPB;
  g.nstrip = (W + TW - 1) / TW;
  g.strips = (long)B * H * g.nstrip;
  return g;
}

template <typename T, int K, bool FLIP>
__global__ __launch_bounds__(256) void dw_fwd_kernel(int B, int H, int W, int C, DwGeom gm, const T* __restrict__ x,
                                                     long ldx, const float* __restrict__ w,
                                                     const float* __restrict__ bias, int add_identity,
                                                     T* __restrict__ y, long ldy, int accumulate, T* __restrict__ gout,
                                                     long ldg) {
  constexpr int CPT = DwCfg<T>::CPT, R = K / 2, WIN = TW + K - 1;
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [K*K][GPB*CPT]
  const int CW = gm.GPB * CPT;
  const int cbase = blockIdx.y * CW;
  for (int e = threadIdx.x; e < K * K * CW; e += 256) {
    const int tap = e / CW, cl = e % CW, c = cbase + cl;
    wl[e] = c < C ? w[(long)c * K * K + (FLIP ? K * K - 1 - tap : tap)] : 0.f;
  }
  __syncthreads();
  const int cg = threadIdx.x % gm.GPB, lane = threadIdx.x / gm.GPB;
  if (lane >= gm.SPB) return;
  const int c0 = cbase + cg * CPT;
  if (c0 >= C) return;
  float bv[CPT];
#pragma unroll
  for (int e = 0; e < CPT; ++e) bv[e] = bias ? bias[c0 + e] : 0.f;
  for (long s = (long)blockIdx.x * gm.SPB + lane; s < gm.strips; s += (long)gridDim.x * gm.SPB) {
    const int ws = s % gm.nstrip;
    const long bh = s / gm.nstrip;
    const int h = bh % H;
    const long img_row0 = (bh - h) * W;  // b * H * W
    const int w0 = ws * TW;
    float acc[TW][CPT];
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int e = 0; e < CPT; ++e) acc[t][e] = bv[e];
    constexpr int UI = K == 7 ? 1 : K;  // keep the 7x7 window's live range to one input row
#pragma unroll UI
    for (int i = 0; i < K; ++i) {
      const int hh = h + i - R;
      if (hh < 0 || hh >= H) continue;
      const T* row = x + (img_row0 + (long)hh * W) * ldx + c0;
      float win[WIN][CPT];
#pragma unroll
      for (int u = 0; u < WIN; ++u) {
        const int ww = w0 + u - R;
        if (ww >= 0 && ww < W) ldv<T>(row + (long)ww * ldx, win[u]);
        else {
#pragma unroll
          for (int e = 0; e < CPT; ++e) win[u][e] = 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < K; ++j) {
        float wv[CPT];
#pragma unroll
        for (int e = 0; e < CPT; ++e) wv[e] = wl[(i * K + j) * CW + cg * CPT + e];
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int e = 0; e < CPT; ++e) acc[t][e] += wv[e] * win[t + j][e];
      }
    }
    const long orow = img_row0 + (long)h * W;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int ww = w0 + t;
      if (ww >= W) break;
      if (add_identity) {
        float xi[CPT];
        ldv<T>(x + (orow + ww) * ldx + c0, xi);
#pragma unroll
        for (int e = 0; e < CPT; ++e) acc[t][e] += xi[e];
      }
      T* yp = y + (orow + ww) * ldy + c0;
      if (accumulate) {
        float o[CPT];
        ldv<T>(yp, o);
#pragma unroll
        for (int e = 0; e < CPT; ++e) acc[t][e] += o[e];
      }
      stv<T>(yp, acc[t]);
      if (gout) {
        float gv[CPT];
#pragma unroll
        for (int e = 0; e < CPT; ++e) gv[e] = gelu_f(acc[t][e]);
        stv<T>(gout + (orow + ww) * ldg + c0, gv);
      }
    }
  }
}

// dW partials: block (strip block bx, channel chunk by, kernel-row group bz); each thread accumulates
// KI kernel rows x K columns x CPT channels over its strips.
template <typename T, int K, int KI>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(int B, int H, int W, int C, DwGeom gm, const T* __restrict__ x,
                                                       long ldx, const T* __restrict__ dy, long lddy,
                                                       float* __restrict__ part) {
  constexpr int CPT = DwCfg<T>::CPT, R = K / 2, WIN = TW + K - 1, KK1 = K * K + 1;
  __shared__ float red[256][CPT + 1];
  const int CW = gm.GPB * CPT;
  const int cbase = blockIdx.y * CW;
  const int cg = threadIdx.x % gm.GPB, lane = threadIdx.x / gm.GPB;
  const int c0 = cbase + cg * CPT;
  const bool active = lane < gm.SPB && c0 < C;
  const int i0 = blockIdx.z * KI;
  float acc[KI][K][CPT];
  float dbs[CPT];
#pragma unroll
  for (int e = 0; e < CPT; ++e) dbs[e] = 0.f;
#pragma unroll
  for (int a = 0; a < KI; ++a)
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int e = 0; e < CPT; ++e) acc[a][j][e] = 0.f;
  if (active) {
    for (long s = (long)blockIdx.x * gm.SPB + lane; s < gm.strips; s += (long)gridDim.x * gm.SPB) {
      const int ws = s % gm.nstrip;
      const long bh = s / gm.nstrip;
      const int h = bh % H;
      const long img_row0 = (bh - h) * W;
      const int w0 = ws * TW;
      float g[TW][CPT];
      const long orow = img_row0 + (long)h * W;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        if (w0 + t < W) ldv<T>(dy + (orow + w0 + t) * lddy + c0, g[t]);
        else {
#pragma unroll
          for (int e = 0; e < CPT; ++e) g[t][e] = 0.f;
        }
      }
      if (i0 == 0) {
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int e = 0; e < CPT; ++e) dbs[e] += g[t][e];
      }
#pragma unroll
      for (int a = 0; a < KI; ++a) {
        const int hh = h + i0 + a - R;
        if (hh < 0 || hh >= H) continue;
        const T* row = x + (img_row0 + (long)hh * W) * ldx + c0;
        float win[WIN][CPT];
#pragma unroll
        for (int u = 0; u < WIN; ++u) {
          const int ww = w0 + u - R;
          if (ww >= 0 && ww < W) ldv<T>(row + (long)ww * ldx, win[u]);
          else {
#pragma unroll
            for (int e = 0; e < CPT; ++e) win[u][e] = 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int t = 0; t < TW; ++t)
#pragma unroll
            for (int e = 0; e < CPT; ++e) acc[a][j][e] += g[t][e] * win[t + j][e];
      }
    }
  }
  // reduce across the strip lanes of each channel group, one (a, j) tap at a time
  const long pbase = (long)blockIdx.x * C * KK1;
#pragma unroll
  for (int tap = 0; tap <= KI * K; ++tap) {
    if (tap == KI * K && i0 != 0) break;
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      float v = 0.f;
      if (active) v = tap < KI * K ? acc[tap / K][tap % K][e] : dbs[e];
      red[threadIdx.x][e] = v;
    }
    __syncthreads();
    if (threadIdx.x < gm.GPB * CPT) {
      const int g2 = threadIdx.x / CPT, e = threadIdx.x % CPT;
      const int c = cbase + g2 * CPT + e;
      if (c < C) {
        float s = 0.f;
        for (int l = 0; l < gm.SPB; ++l) s += red[l * gm.GPB + g2][e];
        const int col = tap < KI * K ? (i0 + tap / K) * K + tap % K : K * K;
        part[pbase + (long)c * KK1 + col] = s;
      }
    }
    __syncthreads();
  }
}

template <typename T>
bool dw_aligned(int C, const void* p, long ld) {
  constexpr int CPT = DwCfg<T>::CPT;
  return C % CPT == 0 && ld % CPT == 0 && ((uintptr_t)p % 16) == 0;
}

template <typename T, bool FLIP>
int dw_fwd(int B, int H, int W, int C, int k, const void* x, long ldx, const float* w, const float* bias, int id,
           void* y, long ldy, int acc, void* gout, long ldg, hipStream_t s) {
  DFM_CHECK_ARG(dw_aligned<T>(C, x, ldx) && dw_aligned<T>(C, y, ldy) && (!gout || dw_aligned<T>(C, gout, ldg)),
                "dwconv: C, row strides and pointers must be 16-byte vector aligned");
  const DwGeom gm = dw_geom<T>(B, H, W, C);
  const unsigned chunks = cdiv(gm.G, gm.GPB);
  const long want = (long)min(cdiv(gm.strips, gm.SPB), 8192u);
  dim3 grid((unsigned)want, chunks);
  const size_t lds = (size_t)k * k * gm.GPB * DwCfg<T>::CPT * sizeof(float);
#define GO(KK)                                                                                                   \
  hipLaunchKernelGGL((dw_fwd_kernel<T, KK, FLIP>), grid, dim3(256), lds, s, B, H, W, C, gm, (const T*)x, ldx, w, \
                     bias, id, (T*)y, ldy, acc, (T*)gout, ldg)
  if (k == 7) GO(7);
  else if (k == 3) GO(3);
  else {
    dfm_set_error("dwconv: k=%d unsupported", k);
    return DFM_ERR_ARG;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T>
int wgrad_grid(int B, int H, int W, int C, int k, DwGeom& gm, dim3& grid) {
  gm = dw_geom<T>(B, H, W, C);
  const int KI = k == 3 ? 3 : 1;
  const unsigned chunks = cdiv(gm.G, gm.GPB);
  const unsigned zdim = k / KI;
  long nsb = (1024 + (long)chunks * zdim - 1) / ((long)chunks * zdim);
  nsb = max(1L, min(nsb, (long)cdiv(gm.strips, gm.SPB)));
  grid = dim3((unsigned)nsb, chunks, zdim);
  return (int)nsb;
}
}  // namespace

extern "C" int dfm_dwconv_fwd(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx, const float* w,
                              const float* bias, int add_identity, void* y, long ldy, void* gout, long ldg,
                              dfm_stream_t stream) {
  DFM_CHECK_ARG(x && w && y && B > 0 && H > 0 && W > 0 && C > 0, "dfm_dwconv_fwd: bad argument");
  if (dtype == DFM_BF16) return dw_fwd<bf16_t, false>(B, H, W, C, k, x, ldx, w, bias, add_identity, y, ldy, 0, gout, ldg, (hipStream_t)stream);
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
  if (dtype == DFM_F32)
    return dw_fwd<float, true>(B, H, W, C, k, dy, lddy, w, nullptr, add_identity, dx, lddx, accumulate, nullptr, 0,
                               (hipStream_t)stream);
  dfm_set_error("dfm_dwconv_bwd_data: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" size_t dfm_dwconv_bwd_weight_workspace(int B, int H, int W, int C, int k) {
  DwGeom gm;
  dim3 grid;
  const int nsb = wgrad_grid<float>(B, H, W, C, k, gm, grid);  // fp32 geometry has the most strip blocks
  DwGeom gm2;
  dim3 grid2;
  const int nsb2 = wgrad_grid<bf16_t>(B, H, W, C, k, gm2, grid2);
  return (size_t)max(nsb, nsb2) * C * (k * k + 1) * sizeof(float);
}

extern "C" int dfm_dwconv_bwd_weight(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx,
                                     const void* dy, long lddy, float* dw, float* db, void* workspace,
                                     dfm_stream_t stream) {
  DFM_CHECK_ARG(x && dy && dw && workspace, "dfm_dwconv_bwd_weight: null argument");
  DFM_CHECK_ARG(k == 3 || k == 7, "dfm_dwconv_bwd_weight: k=%d unsupported", k);
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  DwGeom gm;
  dim3 grid;
  int nsb;
  if (dtype == DFM_BF16) {
    DFM_CHECK_ARG(dw_aligned<bf16_t>(C, x, ldx) && dw_aligned<bf16_t>(C, dy, lddy), "dwconv wgrad: alignment");
    nsb = wgrad_grid<bf16_t>(B, H, W, C, k, gm, grid);
    if (k == 7) hipLaunchKernelGGL((dw_wgrad_kernel<bf16_t, 7, 1>), grid, dim3(256), 0, s, B, H, W, C, gm, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, part);
    else hipLaunchKernelGGL((dw_wgrad_kernel<bf16_t, 3, 3>), grid, dim3(256), 0, s, B, H, W, C, gm, (const bf16_t*)x, ldx, (const bf16_t*)dy, lddy, part);
  } else if (dtype == DFM_F32) {
    DFM_CHECK_ARG(dw_aligned<float>(C, x, ldx) && dw_aligned<float>(C, dy, lddy), "dwconv wgrad: alignment");
    nsb = wgrad_grid<float>(B, H, W, C, k, gm, grid);
    if (k == 7) hipLaunchKernelGGL((dw_wgrad_kernel<float, 7, 1>), grid, dim3(256), 0, s, B, H, W, C, gm, (const float*)x, ldx, (const float*)dy, lddy, part);
    else hipLaunchKernelGGL((dw_wgrad_kernel<float, 3, 3>), grid, dim3(256), 0, s, B, H, W, C, gm, (const float*)x, ldx, (const float*)dy, lddy, part);
  } else {
    dfm_set_error("dfm_dwconv_bwd_weight: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  hipLaunchKernelGGL(partial_sum_kernel<2>, dim3(cdiv((long)C * (k * k + 1), 64)), dim3(1024), 0, s, nsb,
                     (long)C * (k * k + 1), (const float*)part, dw, db, (long)(k * k + 1), 0);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
