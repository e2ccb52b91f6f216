// LayerNorm over the channel dim of NHWC rows (DFormer.py:21-45, channels_last, eps 1e-6).
// A group of G lanes owns one row; the row lives in registers (E <= 16 elements per lane), so
// the statistics are exact two-pass values with one read of x. Backward recomputes xhat from
// the saved mean/rstd and reduces dgamma/dbeta deterministically (per-block partials + sum).
#include "common.h"

namespace {
constexpr int MAXE = 16;

template <int G> DFM_INLINE float gsum(float v) { return group_sum<G>(v); }

template <typename T, int G>
__global__ __launch_bounds__(256) void ln_fwd_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, T* __restrict__ y, long ldy, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lg = threadIdx.x % G;
  const long row = (long)blockIdx.x * (256 / G) + threadIdx.x / G;
  if (row >= rows) return;
  const T* xr = x + row * ldx;
  float v[MAXE];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int c = j * G + lg;
    v[j] = c < C ? ldf(xr + c) : 0.f;
    s += v[j];
  }
  const float mu = gsum<G>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int c = j * G + lg;
    const float d = c < C ? v[j] - mu : 0.f;
    q += d * d;
  }
  const float rs = rsqrtf(gsum<G>(q) / C + eps);
  T* yr = y + row * ldy;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    const int c = j * G + lg;
    if (c < C) stf(yr + c, (v[j] - mu) * rs * gamma[c] + beta[c]);
  }
  if (lg == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// Each block: grid-stride over row groups; dx per row; per-lane column partials for dgamma/dbeta,
// reduced across the block's groups through LDS into part[block][2][C].
template <typename T, int G>
__global__ __launch_bounds__(256) void ln_bwd_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                     const T* __restrict__ dy, long lddy, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const T* __restrict__ dres, long lddres,
                                                     T* __restrict__ dx, long lddx, int accumulate,
                                                     float* __restrict__ part) {
  constexpr int RPB = 256 / G;
  const int lg = threadIdx.x % G, grp = threadIdx.x / G;
  float pg[MAXE], pb[MAXE];
#pragma unroll
  for (int j = 0; j < MAXE; ++j) pg[j] = pb[j] = 0.f;
  for (long row = (long)blockIdx.x * RPB + grp; row < rows; row += (long)gridDim.x * RPB) {
    const T* xr = x + row * ldx;
    const T* gr = dy + row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXE], g[MAXE];
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      const int c = j * G + lg;
      if (c < C) {
        xh[j] = (ldf(xr + c) - mu) * rs;
        const float d = ldf(gr + c);
        pg[j] += d * xh[j];
        pb[j] += d;
        g[j] = d * gamma[c];
      } else {
        xh[j] = g[j] = 0.f;
      }
      sa += g[j];
      sb += g[j] * xh[j];
    }
    sa = gsum<G>(sa) / C;
    sb = gsum<G>(sb) / C;
    T* dr = dx + row * lddx;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      const int c = j * G + lg;
      if (c < C) {
        float v = rs * (g[j] - sa - xh[j] * sb);
        if (dres) v += ldf(dres + row * lddres + c);
        if (accumulate) v += ldf(dr + c);
        stf(dr + c, v);
      }
    }
  }
  // block reduce of the column partials: groups of a wave by shuffles, then the 4 waves via LDS
  __shared__ float red[4][2][1024];
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < MAXE; ++j) {
    float a = pg[j], bsum = pb[j];
#pragma unroll
    for (int o = G; o < 64; o <<= 1) {
      a += __shfl_xor(a, o, 64);
      bsum += __shfl_xor(bsum, o, 64);
    }
    const int c = j * G + lg;
    if ((threadIdx.x & 63) < G && c < C) {
      red[wave][0][c] = a;
      red[wave][1][c] = bsum;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(long)blockIdx.x * 2 * C + c] = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    part[(long)blockIdx.x * 2 * C + C + c] = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
  }
}

__global__ void ln_partial_sum_kernel(int nblk, int C, const float* __restrict__ part, float* __restrict__ dg,
                                      float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * C) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(long)b * 2 * C + c];
  if (c < C) dg[c] = s;
  else db[c - C] = s;
}


// ---- vectorized path: 16-byte vectors (8 bf16 / 4 fp32 channels) per lane, G lanes per row,
// NV vectors per lane (lane lg owns vectors lg, lg + G, ...). A wave reads 64/G whole rows with
// consecutive lanes on consecutive 16-byte chunks, so every load and store is fully coalesced.
template <typename T> struct LnVec { static constexpr int V = 16 / sizeof(T); };

template <typename T>
DFM_INLINE void ln_ldv(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    ld8<T>(p, v);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}
template <typename T>
DFM_INLINE void ln_stv(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    st8<T>(p, v);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}
DFM_INLINE void ln_ldw(const float* p, float* v, int n) {  // n = 4 or 8 fp32 params
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  if (n == 8) {
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

template <typename T, int G, int NV>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps,
                                                         T* __restrict__ y, long ldy, float* __restrict__ mean,
                                                         float* __restrict__ rstd) {
  constexpr int V = LnVec<T>::V;
  const int lg = threadIdx.x % G;
  const long row = (long)blockIdx.x * (256 / G) + threadIdx.x / G;
  const int nvec = C / V;
  const bool live = row < rows;
  const T* xr = x + (live ? row : 0) * ldx;
  float v[NV][V];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int vi = j * G + lg;
    if (live && vi < nvec) {
      ln_ldv<T>(xr + vi * V, v[j]);
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) v[j][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < V; ++e) s += v[j][e];
  }
  const float mu = group_sum<G>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const bool ok = j * G + lg < nvec;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float d = ok ? v[j][e] - mu : 0.f;
      q += d * d;
    }
  }
  const float rs = rsqrtf(group_sum<G>(q) / C + eps);
  if (!live) return;
  T* yr = y + row * ldy;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int vi = j * G + lg;
    if (vi >= nvec) continue;
    float gw[V], bw[V], o[V];
    ln_ldw(gamma + vi * V, gw, V);
    ln_ldw(beta + vi * V, bw, V);
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = (v[j][e] - mu) * rs * gw[e] + bw[e];
    ln_stv<T>(yr + vi * V, o);
  }
  if (lg == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

template <typename T, int G, int NV>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                         const T* __restrict__ dy, long lddy,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, const T* __restrict__ dres,
                                                         long lddres, T* __restrict__ dx, long lddx, int accumulate,
                                                         float* __restrict__ part) {
  constexpr int V = LnVec<T>::V;
  constexpr int RPB = 256 / G;
  const int lg = threadIdx.x % G, grp = threadIdx.x / G;
  const int nvec = C / V;
  float pg[NV][V], pb[NV][V], gw[NV][V];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int vi = j * G + lg;
#pragma unroll
    for (int e = 0; e < V; ++e) pg[j][e] = pb[j][e] = gw[j][e] = 0.f;
    if (vi < nvec) ln_ldw(gamma + vi * V, gw[j], V);
  }
  for (long row = (long)blockIdx.x * RPB + grp; row < rows; row += (long)gridDim.x * RPB) {
    const T* xr = x + row * ldx;
    const T* gr = dy + row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float xh[NV][V], g[NV][V], rv[NV][V];
#pragma unroll
    for (int j = 0; j < NV; ++j) {  // all loads of the row first
      const int vi = j * G + lg;
      if (vi < nvec) {
        ln_ldv<T>(xr + vi * V, xh[j]);
        ln_ldv<T>(gr + vi * V, g[j]);
        if (dres) ln_ldv<T>(dres + row * lddres + vi * V, rv[j]);
        if (accumulate) {
          float o[V];
          ln_ldv<T>(dx + row * lddx + vi * V, o);
#pragma unroll
          for (int e = 0; e < V; ++e) rv[j][e] = (dres ? rv[j][e] : 0.f) + o[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) xh[j][e] = g[j][e] = rv[j][e] = 0.f;
      }
    }
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const bool ok = j * G + lg < nvec;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        xh[j][e] = ok ? (xh[j][e] - mu) * rs : 0.f;
        pg[j][e] += g[j][e] * xh[j][e];
        pb[j][e] += g[j][e];
        g[j][e] *= gw[j][e];
        sa += g[j][e];
        sb += g[j][e] * xh[j][e];
      }
    }
    sa = group_sum<G>(sa) / C;
    sb = group_sum<G>(sb) / C;
    T* dr = dx + row * lddx;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int vi = j * G + lg;
      if (vi >= nvec) continue;
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = rs * (g[j][e] - sa - xh[j][e] * sb);
        if (dres || accumulate) o[e] += rv[j][e];
      }
      ln_stv<T>(dr + vi * V, o);
    }
  }
  // column partials: lanes with the same lg (one per row group of the wave) by shuffles, then the
  // 4 waves through LDS, in a fixed order
  __shared__ float red[4][2][1024];
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int vi = j * G + lg;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float a = pg[j][e], bsum = pb[j][e];
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        a += __shfl_xor(a, o, 64);
        bsum += __shfl_xor(bsum, o, 64);
      }
      if ((threadIdx.x & 63) < G && vi < nvec) {
        red[wave][0][vi * V + e] = a;
        red[wave][1][vi * V + e] = bsum;
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    part[(long)blockIdx.x * 2 * C + c] = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    part[(long)blockIdx.x * 2 * C + C + c] = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
  }
}

// lanes per row / vectors per lane of the vector path; false if the row layout does not allow it
template <typename T>
bool ln_vec_geom(int C, int& G, int& NV) {
  constexpr int V = LnVec<T>::V;
  if (C % V != 0) return false;
  const int nvec = C / V;
  if (nvec < 4) return false;
  G = 4;
  while (G < 64 && G < nvec) G *= 2;
  NV = (nvec + G - 1) / G;
  return NV == 1 || NV == 2 || NV == 4;
}
template <typename T>
bool ln_al(const void* p, long ld) {
  return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % LnVec<T>::V == 0);
}

int pick_g(int C) {
  int g = 8;
  while (g < 64 && g * MAXE / 2 < C) g *= 2;  // keep E <= 8 where possible
  while (g < 64 && g * MAXE < C) g *= 2;
  return g;
}

constexpr int LN_BWD_BLOCKS = 512;

template <typename T>
int ln_fwd(long rows, int C, const void* x, long ldx, const float* gamma, const float* beta, float eps, void* y,
           long ldy, float* mean, float* rstd, hipStream_t s) {
  int VG, VNV;
  if (ln_vec_geom<T>(C, VG, VNV) && ln_al<T>(x, ldx) && ln_al<T>(y, ldy) && (uintptr_t)gamma % 16 == 0 &&
      (uintptr_t)beta % 16 == 0) {
    const unsigned vgrid = cdiv(rows, 256 / VG);
#define GOV(GG, NN)                                                                                          \
  if (VG == GG && VNV == NN) {                                                                                \
    DFM_LAUNCH((ln_fwd_vec_kernel<T, GG, NN>), dim3(vgrid), dim3(256), 0, s, rows, C, (const T*)x, ldx, \
                       gamma, beta, eps, (T*)y, ldy, mean, rstd);                                             \
    DFM_LAUNCH_CHECK();                                                                                      \
    return DFM_OK;                                                                                           \
  }
    GOV(4, 1) GOV(8, 1) GOV(16, 1) GOV(32, 1) GOV(64, 1) GOV(64, 2) GOV(64, 4)
#undef GOV
  }
  const int G = pick_g(C);
  const unsigned grid = cdiv(rows, 256 / G);
#define GO(GG)                                                                                            \
  DFM_LAUNCH((ln_fwd_kernel<T, GG>), dim3(grid), dim3(256), 0, s, rows, C, (const T*)x, ldx, gamma, \
                     beta, eps, (T*)y, ldy, mean, rstd)
  switch (G) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    default: GO(64); break;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T>
int ln_bwd(long rows, int C, const void* x, long ldx, const void* dy, long lddy, const float* gamma,
           const float* mean, const float* rstd, const void* dres, long lddres, void* dx, long lddx, int acc,
           float* dg, float* db, void* ws, DfmPartialSum* defer,
           hipStream_t s) {
  float* part = (float*)ws;
  int VG, VNV;
  if (ln_vec_geom<T>(C, VG, VNV) && ln_al<T>(x, ldx) && ln_al<T>(dy, lddy) && ln_al<T>(dres, lddres) &&
      ln_al<T>(dx, lddx) && (uintptr_t)gamma % 16 == 0) {
    const unsigned vgrid = min((unsigned)LN_BWD_BLOCKS, cdiv(rows, 256 / VG));
    bool launched = false;
#define GOV(GG, NN)                                                                                            \
  if (!launched && VG == GG && VNV == NN) {                                                                     \
    DFM_LAUNCH((ln_bwd_vec_kernel<T, GG, NN>), dim3(vgrid), dim3(256), 0, s, rows, C, (const T*)x, ldx,   \
                       (const T*)dy, lddy, gamma, mean, rstd, (const T*)dres, lddres, (T*)dx, lddx, acc, part); \
    launched = true;                                                                                           \
  }
    GOV(4, 1) GOV(8, 1) GOV(16, 1) GOV(32, 1) GOV(64, 1) GOV(64, 2) GOV(64, 4)
#undef GOV
    if (launched) {
      DFM_LAUNCH_CHECK();
      return second_stage(1, (int)vgrid, 2L * C, part, dg, db, (long)C, 0, defer, s);
    }
  }
  const int G = pick_g(C);
  const unsigned grid = min((unsigned)LN_BWD_BLOCKS, cdiv(rows, 256 / G));
#define GO(GG)                                                                                             \
  DFM_LAUNCH((ln_bwd_kernel<T, GG>), dim3(grid), dim3(256), 0, s, rows, C, (const T*)x, ldx,         \
                     (const T*)dy, lddy, gamma, mean, rstd, (const T*)dres, lddres, (T*)dx, lddx, acc, part)
  switch (G) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    default: GO(64); break;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  return second_stage(1, (int)grid, 2L * C, part, dg, db, (long)C, 0, defer, s);
}
}  // namespace

extern "C" int dfm_layernorm_fwd(int dtype, long rows, int C, const void* x, long ldx, const float* gamma,
                                 const float* beta, float eps, void* y, long ldy, float* mean, float* rstd,
                                 dfm_stream_t stream) {
  DFM_CHECK_ARG(C > 0 && C <= 64 * MAXE, "dfm_layernorm_fwd: C=%d unsupported (max %d)", C, 64 * MAXE);
  DFM_CHECK_ARG(x && y && gamma && beta && mean && rstd, "dfm_layernorm_fwd: null argument");
  if (rows == 0) return DFM_OK;
  if (dtype == DFM_BF16) return ln_fwd<bf16_t>(rows, C, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, (hipStream_t)stream);
  else if (dtype == DFM_F16) return ln_fwd<f16_t>(rows, C, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, (hipStream_t)stream);
  if (dtype == DFM_F32) return ln_fwd<float>(rows, C, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, (hipStream_t)stream);
  dfm_set_error("dfm_layernorm_fwd: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" size_t dfm_layernorm_bwd_workspace(long rows, int C) {
  (void)rows;
  return (size_t)LN_BWD_BLOCKS * 2 * C * sizeof(float);
}

extern "C" int dfm_layernorm_bwd(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                                 const float* gamma, const float* mean, const float* rstd, const void* dres,
                                 long lddres, void* dx, long lddx, int accumulate, float* dgamma, float* dbeta,
                                 void* workspace, DfmPartialSum* defer, dfm_stream_t stream) {
  if (defer) *defer = DfmPartialSum{};  // n = 0: nothing to sum unless the first stage runs
  DFM_CHECK_ARG(C > 0 && C <= 1024, "dfm_layernorm_bwd: C=%d unsupported", C);
  DFM_CHECK_ARG(x && dy && dx && gamma && mean && rstd && dgamma && dbeta && workspace,
                "dfm_layernorm_bwd: null argument");
  if (rows == 0) return DFM_OK;
  if (dtype == DFM_BF16)
    return ln_bwd<bf16_t>(rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dres, lddres, dx, lddx, accumulate, dgamma, dbeta,
                          workspace, defer, (hipStream_t)stream);
  else if (dtype == DFM_F16)
    return ln_bwd<f16_t>(rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dres, lddres, dx, lddx, accumulate, dgamma, dbeta,
                          workspace, defer, (hipStream_t)stream);
  if (dtype == DFM_F32)
    return ln_bwd<float>(rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dres, lddres, dx, lddx, accumulate, dgamma, dbeta,
                         workspace, defer, (hipStream_t)stream);
  dfm_set_error("dfm_layernorm_bwd: bad dtype");
  return DFM_ERR_DTYPE;
}
