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
  const int G = pick_g(C);
  const unsigned grid = cdiv(rows, 256 / G);
#define GO(GG)                                                                                            \
  hipLaunchKernelGGL((ln_fwd_kernel<T, GG>), dim3(grid), dim3(256), 0, s, rows, C, (const T*)x, ldx, gamma, \
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
           float* dg, float* db, void* ws,
           hipStream_t s) {
  const int G = pick_g(C);
  const unsigned grid = min((unsigned)LN_BWD_BLOCKS, cdiv(rows, 256 / G));
  float* part = (float*)ws;
#define GO(GG)                                                                                             \
  hipLaunchKernelGGL((ln_bwd_kernel<T, GG>), dim3(grid), dim3(256), 0, s, rows, C, (const T*)x, ldx,         \
                     (const T*)dy, lddy, gamma, mean, rstd, (const T*)dres, lddres, (T*)dx, lddx, acc, part)
  switch (G) {
    case 8: GO(8); break;
    case 16: GO(16); break;
    case 32: GO(32); break;
    default: GO(64); break;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  hipLaunchKernelGGL(partial_sum_kernel<1>, dim3(cdiv(2L * C, 64)), dim3(1024), 0, s, (int)grid, 2L * C,
                     (const float*)part, dg, db, (long)C, 0);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
}  // namespace

extern "C" int dfm_layernorm_fwd(int dtype, long rows, int C, const void* x, long ldx, const float* gamma,
                                 const float* beta, float eps, void* y, long ldy, float* mean, float* rstd,
                                 dfm_stream_t stream) {
  DFM_CHECK_ARG(C > 0 && C <= 64 * MAXE, "dfm_layernorm_fwd: C=%d unsupported (max %d)", C, 64 * MAXE);
  DFM_CHECK_ARG(x && y && gamma && beta && mean && rstd, "dfm_layernorm_fwd: null argument");
  if (rows == 0) return DFM_OK;
  if (dtype == DFM_BF16) return ln_fwd<bf16_t>(rows, C, x, ldx, gamma, beta, eps, y, ldy, mean, rstd, (hipStream_t)stream);
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
                                 void* workspace, dfm_stream_t stream) {
  DFM_CHECK_ARG(C > 0 && C <= 1024, "dfm_layernorm_bwd: C=%d unsupported", C);
  DFM_CHECK_ARG(x && dy && dx && gamma && mean && rstd && dgamma && dbeta && workspace,
                "dfm_layernorm_bwd: null argument");
  if (rows == 0) return DFM_OK;
  if (dtype == DFM_BF16)
    return ln_bwd<bf16_t>(rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dres, lddres, dx, lddx, accumulate, dgamma, dbeta,
                          workspace, (hipStream_t)stream);
  if (dtype == DFM_F32)
    return ln_bwd<float>(rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dres, lddres, dx, lddx, accumulate, dgamma, dbeta,
                         workspace, (hipStream_t)stream);
  dfm_set_error("dfm_layernorm_bwd: bad dtype");
  return DFM_ERR_DTYPE;
}
