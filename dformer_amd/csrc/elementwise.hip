// Bandwidth-bound helpers: column reductions (bias / layer-scale grads, BatchNorm statistics),
// activation backward, residual chain rule, dtype casts, NMF multiplicative updates and AdamW.
// All reductions are two-stage with fixed order (deterministic, no float atomics).
#include <cstdlib>

#include <algorithm>

#include "common.h"

namespace {
constexpr int COLS = 64;       // columns per block in column reductions
// column-reduction geometry: at most DFM_RED_BLOCKS blocks of at least DFM_RED_MIN_ROWS rows (compile-time
// knobs so a variant build can be A/B'd; dfm_build_tag reports them)
#ifndef DFM_RED_MIN_ROWS
#define DFM_RED_MIN_ROWS 256
#endif
#ifndef DFM_RED_BLOCKS
#define DFM_RED_BLOCKS 512
#endif
constexpr int RED_BLOCKS = DFM_RED_BLOCKS, RED_MIN_ROWS = DFM_RED_MIN_ROWS;

// part[blk][k][c] for k < NOUT: sum over this block's rows of f_k(row, c)
template <typename T, int MODE>
__global__ __launch_bounds__(256) void colred_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                     const T* __restrict__ y, long ldy, const float* __restrict__ p0,
                                                     const float* __restrict__ p1, long rps, float* __restrict__ part,
                                                     int nblk, float* __restrict__ aux) {
  // MODE 0: sum x * (y?) * rowscale(p1?)           -> 1 output
  // MODE 1: BN stats, shifted by K = x[row 0]: sum (x-K), sum (x-K)^2 -> 2 outputs (+ K into aux)
  // MODE 2: BN bwd:  sum y, sum y * (x - p0[c]) * p1[c]   -> 2 outputs (y = dy, p0 mean, p1 rstd)
  constexpr int NOUT = MODE == 0 ? 1 : 2;
  const int cl = threadIdx.x % COLS, rl = threadIdx.x / COLS;  // 4 row lanes
  const int c = blockIdx.y * COLS + cl;
  const long per = (rows + nblk - 1) / nblk;
  const long r0 = (long)blockIdx.x * per, r1 = min(rows, r0 + per);
  float s0 = 0.f, s1 = 0.f;
  const float k0 = (MODE == 1 && c < C) ? ldf(x + c) : 0.f;
  if (MODE == 1 && blockIdx.x == 0 && rl == 0 && c < C) aux[c] = k0;
  if (c < C) {
    for (long r = r0 + rl; r < r1; r += 4) {
      const float xv = ldf(x + r * ldx + c) - k0;
      if (MODE == 0) {
        float v = xv;
        if (y) v *= ldf(y + r * ldy + c);
        if (p1) v *= p1[r / rps];
        s0 += v;
      } else if (MODE == 1) {
        s0 += xv;
        s1 += xv * xv;
      } else {
        const float g = ldf(y + r * ldy + c);
        s0 += g;
        s1 += g * (xv - p0[c]) * p1[c];
      }
    }
  }
  __shared__ float red[NOUT][4][COLS];
  red[0][rl][cl] = s0;
  if (NOUT == 2) red[NOUT - 1][rl][cl] = s1;
  __syncthreads();
  if (rl == 0 && c < C) {
    part[((long)blockIdx.x * NOUT + 0) * C + c] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    if (NOUT == 2)
      part[((long)blockIdx.x * NOUT + 1) * C + c] =
          red[NOUT - 1][0][cl] + red[NOUT - 1][1][cl] + red[NOUT - 1][2][cl] + red[NOUT - 1][3][cl];
  }
}

// Narrow-row variant (C/V lanes per row, V = one 16-byte vector of channels per lane, 256/(C/V)
// rows per pass): the scalar kernel above idles most of its 64 column lanes and issues 2-byte
// loads when C is 16..64 (the stem BatchNorms: 1.2M rows x 16/32 channels). Same partial layout.
template <typename T>
DFM_INLINE void ldvec(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    ld8<T>(p, v);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}

// YP: y present (a compile-time flag: a load under a runtime `if (y)` was waited on right where it was
// issued, which serialized the four rows in flight)
template <typename T, int MODE, bool YP>
__global__ __launch_bounds__(256) void colred_vec_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                         const T* __restrict__ y, long ldy,
                                                         const float* __restrict__ p0, const float* __restrict__ p1,
                                                         long rps, float* __restrict__ part, int nblk,
                                                         float* __restrict__ aux) {
  constexpr int NOUT = MODE == 0 ? 1 : 2, V = 16 / sizeof(T);
  __shared__ float red[NOUT][256][V + 1];
  // RL rows per pass; when G does not divide 256 the last 256 - RL * G lanes sit out (C = 96 / 288 / 576:
  // DFormer-Large's BatchNorms ran the scalar kernel's 2-byte loads before)
  const int G = C / V, RL = 256 / G;
  const int g = threadIdx.x % G, rl = threadIdx.x / G, c0 = g * V;
  const long per = (rows + nblk - 1) / nblk;
  const long r0 = (long)blockIdx.x * per, r1 = rl < RL ? min(rows, r0 + per) : r0;
  float s0[V], s1[V], mu[V], rs[V], k0[V];
  if (MODE == 1) ldvec<T>(x + c0, k0);  // BN stats shift: row 0
#pragma unroll
  for (int e = 0; e < V; ++e) {
    s0[e] = 0.f;
    s1[e] = 0.f;
    mu[e] = MODE == 2 ? p0[c0 + e] : 0.f;
    rs[e] = MODE == 2 ? p1[c0 + e] : 0.f;
    if (MODE != 1) k0[e] = 0.f;
  }
  if (MODE == 1 && blockIdx.x == 0 && rl == 0) {
#pragma unroll
    for (int e = 0; e < V; ++e) aux[c0 + e] = k0[e];
  }
  // one row's contribution; rows are added in order, four rows' loads in flight at a time
  auto add_row = [&](long r, float* xv, const float* yv) {
    if (MODE == 1) {
#pragma unroll
      for (int e = 0; e < V; ++e) xv[e] -= k0[e];
    }
    if (MODE == 0) {
      const float sc = p1 ? p1[r / rps] : 1.f;
#pragma unroll
      for (int e = 0; e < V; ++e) s0[e] += (YP ? xv[e] * yv[e] : xv[e]) * sc;
    } else if (MODE == 1) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        s0[e] += xv[e];
        s1[e] += xv[e] * xv[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        s0[e] += yv[e];
        s1[e] += yv[e] * (xv[e] - mu[e]) * rs[e];
      }
    }
  };
  constexpr bool HAS_Y = MODE != 1 && YP;
  long r = r0 + rl;
  for (; r + 3 * RL < r1; r += 4 * RL) {
    float xv[4][V], yv[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ldvec<T>(x + (r + u * RL) * ldx + c0, xv[u]);
      if (HAS_Y) ldvec<T>(y + (r + u * RL) * ldy + c0, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) add_row(r + u * RL, xv[u], yv[u]);
  }
  for (; r < r1; r += RL) {
    float xv[V], yv[V];
    ldvec<T>(x + r * ldx + c0, xv);
    if (HAS_Y) ldvec<T>(y + r * ldy + c0, yv);
    add_row(r, xv, yv);
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    red[0][threadIdx.x][e] = s0[e];
    if (NOUT == 2) red[NOUT - 1][threadIdx.x][e] = s1[e];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < NOUT * C; idx += 256) {
    const int k = idx / C, c = idx % C, gg = c / V, e = c % V;
    float v = 0.f;
    for (int q = 0; q < RL; ++q) v += red[k][q * G + gg][e];
    part[((long)blockIdx.x * NOUT + k) * C + c] = v;
  }
}

__global__ void colred_sum_kernel(int nblk, int n, const float* __restrict__ part, float* __restrict__ out,
                                  int accumulate) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(long)b * n + e];
  out[e] = accumulate ? out[e] + s : s;
}

int red_blocks(long rows) { return (int)min((long)RED_BLOCKS, max(1L, (rows + RED_MIN_ROWS - 1) / RED_MIN_ROWS)); }

template <typename T, int MODE>
int colred(long rows, int C, const void* x, long ldx, const void* y, long ldy, const float* p0, const float* p1,
           long rps, float* out, int accumulate, void* ws, hipStream_t s, float* aux = nullptr) {
  constexpr int NOUT = MODE == 0 ? 1 : 2;
  const int nblk = red_blocks(rows);
  constexpr int V = 16 / sizeof(T);
  const int G = C / V;
  // The vectorized narrow-row reduction wherever the row layout allows it. BN statistics are sums
  // shifted by the first row, so the variance does not cancel (E[x²] - E[x]² moved the fp32
  // input-gradient golden past 1e-3 in round 1).
  const bool vec = C % V == 0 && G <= 256 && ldx % V == 0 && ((uintptr_t)x & 15) == 0 &&
                   (!y || (ldy % V == 0 && ((uintptr_t)y & 15) == 0));
  if (vec && y)
    DFM_LAUNCH((colred_vec_kernel<T, MODE, true>), dim3(nblk), dim3(256), 0, s, rows, C, (const T*)x, ldx,
               (const T*)y, ldy, p0, p1, rps > 0 ? rps : 1, (float*)ws, nblk, aux);
  else if (vec)
    DFM_LAUNCH((colred_vec_kernel<T, MODE, false>), dim3(nblk), dim3(256), 0, s, rows, C, (const T*)x, ldx,
               (const T*)y, ldy, p0, p1, rps > 0 ? rps : 1, (float*)ws, nblk, aux);
  else
    DFM_LAUNCH((colred_kernel<T, MODE>), dim3(nblk, cdiv(C, COLS)), dim3(256), 0, s, rows, C, (const T*)x,
                       ldx, (const T*)y, ldy, p0, p1, rps > 0 ? rps : 1, (float*)ws, nblk, aux);
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(partial_sum_kernel<0>, dim3(cdiv((long)NOUT * C, 64)), dim3(1024), 0, s, nblk, (long)NOUT * C,
                     (const float*)ws, out, (float*)nullptr, 0L, accumulate);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ---- elementwise over [rows, C] with strides
template <typename T, int OP>
__global__ void ew2d_kernel(long rows, int C, const T* __restrict__ a, long lda, const T* __restrict__ b, long ldb,
                            const float* __restrict__ colscale, const float* __restrict__ rowscale, long rps,
                            float alpha, T* __restrict__ d, long ldd, int accumulate) {
  const long n = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = i % C;
    const float av = ldf(a + r * lda + c);
    float v;
    if (OP == 0) {  // scale_mul
      v = alpha * av;
      if (b) v *= ldf(b + r * ldb + c);
      if (colscale) v *= colscale[c];
      if (rowscale) v *= rowscale[r / rps];
    } else if (OP == 1) {  // gelu bwd: a = dy, b = pre
      v = av * gelu_grad_f(ldf(b + r * ldb + c));
    } else {  // relu bwd: a = dy, b = relu output
      v = ldf(b + r * ldb + c) > 0.f ? av : 0.f;
    }
    T* dp = d + r * ldd + c;
    if (accumulate) v += ldf(dp);
    stf(dp, v);
  }
}


// 8-column vector form of ew2d_kernel (rows 16-byte aligned, C % 8 == 0)
template <typename T, int OP>
__global__ void ew2d_vec_kernel(long rows, int C, const T* __restrict__ a, long lda, const T* __restrict__ b, long ldb,
                                const float* __restrict__ colscale, const float* __restrict__ rowscale, long rps,
                                float alpha, T* __restrict__ d, long ldd, int accumulate) {
  const int cv = C / 8;
  const long n = rows * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float av[8], bv[8], v[8];
    ld8<T>(a + r * lda + c, av);
    if (b) ld8<T>(b + r * ldb + c, bv);
    T* dp = d + r * ldd + c;
    float o[8];
    if (accumulate) ld8<T>(dp, o);
    const float rs = (OP == 0 && rowscale) ? rowscale[r / rps] : 1.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (OP == 0) {
        v[e] = alpha * av[e];
        if (b) v[e] *= bv[e];
        if (colscale) v[e] *= colscale[c + e];
        v[e] *= rs;
      } else if (OP == 1) {
        v[e] = av[e] * gelu_grad_f(bv[e]);
      } else {
        v[e] = bv[e] > 0.f ? av[e] : 0.f;
      }
      if (accumulate) v[e] += o[e];
    }
    st8<T>(dp, v);
  }
}

template <typename T>
bool ew_al(const void* p, long ld) {
  return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 8 == 0);
}

unsigned ew_grid(long n) { return (unsigned)min((long)8192, max(1L, (n + 255) / 256)); }

template <int OP>
int ew2d(int dtype, long rows, int C, const void* a, long lda, const void* b, long ldb, const float* cs,
         const float* rs, long rps, float alpha, void* d, long ldd, int acc, hipStream_t s) {
  if (rows * C == 0) return DFM_OK;
  if (C % 8 == 0 && ew_al<float>(a, lda) && ew_al<float>(b, ldb) && ew_al<float>(d, ldd) &&
      (dtype == DFM_BF16 || dtype == DFM_F16 || dtype == DFM_F32)) {
    const unsigned gv = ew_grid(rows * C / 8);
    if (dtype == DFM_BF16)
      DFM_LAUNCH((ew2d_vec_kernel<bf16_t, OP>), dim3(gv), dim3(256), 0, s, rows, C, (const bf16_t*)a, lda,
                         (const bf16_t*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (bf16_t*)d, ldd, acc);
    else if (dtype == DFM_F16)
      DFM_LAUNCH((ew2d_vec_kernel<f16_t, OP>), dim3(gv), dim3(256), 0, s, rows, C, (const f16_t*)a, lda,
                         (const f16_t*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (f16_t*)d, ldd, acc);
    else
      DFM_LAUNCH((ew2d_vec_kernel<float, OP>), dim3(gv), dim3(256), 0, s, rows, C, (const float*)a, lda,
                         (const float*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (float*)d, ldd, acc);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  const unsigned g = ew_grid(rows * C);
  if (dtype == DFM_BF16)
    DFM_LAUNCH((ew2d_kernel<bf16_t, OP>), dim3(g), dim3(256), 0, s, rows, C, (const bf16_t*)a, lda,
                       (const bf16_t*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (bf16_t*)d, ldd, acc);
  else if (dtype == DFM_F16)
    DFM_LAUNCH((ew2d_kernel<f16_t, OP>), dim3(g), dim3(256), 0, s, rows, C, (const f16_t*)a, lda,
                       (const f16_t*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (f16_t*)d, ldd, acc);
  else if (dtype == DFM_F32)
    DFM_LAUNCH((ew2d_kernel<float, OP>), dim3(g), dim3(256), 0, s, rows, C, (const float*)a, lda,
                       (const float*)b, ldb, cs, rs, rps > 0 ? rps : 1, alpha, (float*)d, ldd, acc);
  else {
    dfm_set_error("elementwise: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename TI, typename TO>
__global__ void cast_kernel(long n, const TI* __restrict__ x, TO* __restrict__ y) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    stf(y + i, ldf(x + i));
}

// ---- BatchNorm
__global__ void bn_finalize_kernel(int C, const float* __restrict__ st, double count, float eps, float mom,
                                   float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rm,
                                   float* __restrict__ rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // st = (sum (x-K), sum (x-K)^2, K): mean = K + d, var = E[(x-K)^2] - d^2 with d = E[x-K] small
  const double d = st[c] / count;
  const double mu = st[2 * C + c] + d;
  double var = st[C + c] / count - d * d;
  if (var < 0) var = 0;
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + eps));
  if (rm) rm[c] = (1.f - mom) * rm[c] + mom * (float)mu;
  if (rv) rv[c] = (1.f - mom) * rv[c] + mom * (float)(var * count / max(count - 1.0, 1.0));
}

// SyncBN: per-rank shifted sums [S][3][C] (as dfm_bn_stats writes them) -> one triple of the union,
// re-shifted onto shard 0's K: S1 = sum_s S1_s + n_s d_s, S2 = sum_s S2_s + 2 d_s S1_s + n_s d_s^2 with
// d_s = K_s - K_0, in fp64 and in shard order (deterministic; for one shard the output is the input).
__global__ void bn_merge_kernel(int S, int C, const float* __restrict__ parts, const float* __restrict__ counts,
                                float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double k0 = parts[2 * C + c];
  double s1 = 0.0, s2 = 0.0;
  for (int s = 0; s < S; ++s) {
    const float* p = parts + (long)s * 3 * C;
    const double n = counts[s], a = p[c], b = p[C + c], d = (double)p[2 * C + c] - k0;
    s1 += a + n * d;
    s2 += b + 2.0 * d * a + n * d * d;
  }
  out[c] = (float)s1;
  out[C + c] = (float)s2;
  out[2 * C + c] = (float)k0;
}

template <typename T>
__global__ void bn_apply_kernel(long rows, int C, const T* __restrict__ x, long ldx, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const T* __restrict__ res, long ldres, int act,
                                T* __restrict__ y, long ldy) {
  const long n = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = i % C;
    float v = (ldf(x + r * ldx + c) - mean[c]) * rstd[c] * gamma[c] + beta[c];
    if (res) v += ldf(res + r * ldres + c);
    if (act == 2) v = fmaxf(v, 0.f);
    stf(y + r * ldy + c, v);
  }
}

template <typename T>
__global__ void bn_bwd_apply_kernel(long rows, int C, const T* __restrict__ x, long ldx, const T* __restrict__ dy,
                                    long lddy, const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ gamma, const float* __restrict__ st, float inv_n,
                                    T* __restrict__ dx, long lddx, int accumulate) {
  const long n = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = i % C;
    const float xh = (ldf(x + r * ldx + c) - mean[c]) * rstd[c];
    float v = gamma[c] * rstd[c] * (ldf(dy + r * lddy + c) - st[c] * inv_n - xh * st[C + c] * inv_n);
    T* dp = dx + r * lddx + c;
    if (accumulate) v += ldf(dp);
    stf(dp, v);
  }
}


// 8-column vector forms of the BatchNorm apply kernels (rows 16-byte aligned, C % 8 == 0)
template <typename T>
__global__ void bn_apply_vec_kernel(long rows, int C, const T* __restrict__ x, long ldx, const float* __restrict__ mean,
                                    const float* __restrict__ rstd, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, const T* __restrict__ res, long ldres, int act,
                                    T* __restrict__ y, long ldy) {
  const int cv = C / 8;
  const long n = rows * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float v[8], rv[8];
    ld8<T>(x + r * ldx + c, v);
    if (res) ld8<T>(res + r * ldres + c, rv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = (v[e] - mean[c + e]) * rstd[c + e] * gamma[c + e] + beta[c + e];
      if (res) v[e] += rv[e];
      if (act == 2) v[e] = fmaxf(v[e], 0.f);
    }
    st8<T>(y + r * ldy + c, v);
  }
}

template <typename T>
__global__ void bn_bwd_apply_vec_kernel(long rows, int C, const T* __restrict__ x, long ldx, const T* __restrict__ dy,
                                        long lddy, const float* __restrict__ mean, const float* __restrict__ rstd,
                                        const float* __restrict__ gamma, const float* __restrict__ st, float inv_n,
                                        T* __restrict__ dx, long lddx, int accumulate) {
  const int cv = C / 8;
  const long n = rows * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float xv[8], g[8], o[8];
    ld8<T>(x + r * ldx + c, xv);
    ld8<T>(dy + r * lddy + c, g);
    T* dp = dx + r * lddx + c;
    if (accumulate) ld8<T>(dp, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (xv[e] - mean[c + e]) * rstd[c + e];
      float v = gamma[c + e] * rstd[c + e] * (g[e] - st[c + e] * inv_n - xh * st[C + c + e] * inv_n);
      if (accumulate) v += o[e];
      o[e] = v;
    }
    st8<T>(dp, o);
  }
}

// ---- NMF multiplicative update
// out16 / gnum16 (optional): bf16 copies of the result for the bf16-operand NMF GEMMs
template <typename TC>
__global__ void nmf_update_kernel(long n, const float* __restrict__ a, const float* __restrict__ num,
                                  const float* __restrict__ den, float eps, float* __restrict__ out,
                                  TC* __restrict__ out16) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = a[i] * num[i] / (den[i] + eps);
    out[i] = v;
    if (out16) out16[i] = Num<TC>::from_f(v);
  }
}
template <typename TC>
__global__ void nmf_update_bwd_kernel(long n, const float* __restrict__ g, const float* __restrict__ a,
                                      const float* __restrict__ num, const float* __restrict__ den,
                                      const float* __restrict__ out, float eps, float* __restrict__ ga, int acc,
                                      float* __restrict__ gnum, float* __restrict__ gden,
                                      TC* __restrict__ gnum16) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float r = 1.f / (den[i] + eps);
    const float gi = g[i];
    const float v = gi * num[i] * r;
    ga[i] = acc ? ga[i] + v : v;
    const float gn = gi * a[i] * r;
    gnum[i] = gn;
    if (gnum16) gnum16[i] = Num<TC>::from_f(gn);
    gden[i] = -gi * out[i] * r;
  }
}

// ---- row softmax (one wave per row)
__global__ void softmax_rows_kernel(long rows, int R, const float* __restrict__ x, float* __restrict__ y) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + row * R;
  float m = -INFINITY;
  for (int c = lane; c < R; c += 64) m = fmaxf(m, xr[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < R; c += 64) s += __expf(xr[c] - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int c = lane; c < R; c += 64) y[row * R + c] = __expf(xr[c] - m) * inv;
}
__global__ void softmax_rows_bwd_kernel(long rows, int R, const float* __restrict__ y, const float* __restrict__ dy,
                                        float* __restrict__ dx, int acc) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float d = 0.f;
  for (int c = lane; c < R; c += 64) d += y[row * R + c] * dy[row * R + c];
  d = wave_sum(d);
  for (int c = lane; c < R; c += 64) {
    const float v = y[row * R + c] * (dy[row * R + c] - d);
    dx[row * R + c] = acc ? dx[row * R + c] + v : v;
  }
}

// ---- AdamW (torch.optim.AdamW semantics, decoupled weight decay)
template <typename TC>
__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, float lr, float b1, float b2, float eps, float wd, float bc1,
                             float bc2_sqrt, float gscale, TC* __restrict__ copy) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
    if (copy) copy[i] = Num<TC>::from_f(pi);
  }
}
// Same update with lr and step read from device memory (hyper = [lr, step]), so a captured HIP
// graph replays every optimizer step without host-baked scalars. With the fp16 loss scaler's device
// state amp = {scale, growth_tracker, applied_steps, skipped} and overflow flag: the step is skipped
// when flag[0] is set (GradScaler.step), gradients are unscaled by 1/scale and the step count is
// amp[2] + 1 (torch's AdamW counts applied steps only).
template <typename TC>
__global__ void adamw_dev_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, const float* __restrict__ hyper, float b1, float b2,
                                 float eps, float wd, float gscale, TC* __restrict__ copy,
                                 const float* __restrict__ amp, const int* __restrict__ flag) {
  if (flag && flag[0]) return;
  const float lr = hyper[0], step = amp ? amp[2] + 1.f : hyper[1];
  if (amp) gscale /= amp[0];
  const float bc1 = 1.f - powf(b1, step), bc2_sqrt = sqrtf(1.f - powf(b2, step));
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
    if (copy) copy[i] = Num<TC>::from_f(pi);
  }
}
// GradScaler.update (torch/amp/grad_scaler.py _amp_update_scale_) on the device state, after the
// step's AdamW launches have read it; clears the overflow flag for the next step. One lane.
__global__ void loss_scale_update_kernel(float* __restrict__ amp, int* __restrict__ flag, float growth,
                                         float backoff, int interval) {
  if (threadIdx.x != 0) return;
  if (flag[0]) {
    amp[0] *= backoff;
    amp[1] = 0.f;
    amp[3] += 1.f;
  } else {
    amp[2] += 1.f;
    amp[1] += 1.f;
    if (amp[1] >= (float)interval) {
      amp[0] *= growth;
      amp[1] = 0.f;
    }
  }
  flag[0] = 0;
}

// o1 = src * m1, o2 = src * m2 (the two products of one gradient against the two factors of
// an elementwise product, DFormer.py:134-135: d(q*a) -> dq = d*a, da = d*q): one read of src.
template <typename T>
__global__ void dual_mul_vec_kernel(long rows, int C, const T* __restrict__ src, long lds, const T* __restrict__ m1,
                                    long ld1, const T* __restrict__ m2, long ld2, T* __restrict__ o1, long ldo1,
                                    T* __restrict__ o2, long ldo2) {
  const int cv = C / 8;
  const long n = rows * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cv;
    const int c = (int)(i - r * cv) * 8;
    float sv[8], a[8], b[8];
    ld8<T>(src + r * lds + c, sv);
    ld8<T>(m1 + r * ld1 + c, a);
    ld8<T>(m2 + r * ld2 + c, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] *= sv[e];
      b[e] *= sv[e];
    }
    st8<T>(o1 + r * ldo1 + c, a);
    st8<T>(o2 + r * ldo2 + c, b);
  }
}

// flag[0] = 1 if any element of g is inf / nan (the GradScaler's found_inf, torch/amp/grad_scaler.py)
__global__ void nonfinite_kernel(long n, const float* __restrict__ g, int* __restrict__ flag) {
  bool bad = false;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = 1;
}
}  // namespace

// ================================================================ C ABI
extern "C" size_t dfm_colsum_workspace(long rows, int C) { return (size_t)red_blocks(rows) * 2 * C * sizeof(float); }
extern "C" size_t dfm_bn_workspace(long rows, int C) { return dfm_colsum_workspace(rows, C); }

extern "C" int dfm_colsum(int dtype, long rows, int C, const void* x, long ldx, const void* mul, long ldmul,
                          const float* rowscale, long rps, float* out, int accumulate, void* ws, dfm_stream_t stream) {
  DFM_CHECK_ARG(x && out && ws && C > 0, "dfm_colsum: bad argument");
  if (rows == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return colred<bf16_t, 0>(rows, C, x, ldx, mul, ldmul, nullptr, rowscale, rps, out, accumulate, ws, s);
  else if (dtype == DFM_F16) return colred<f16_t, 0>(rows, C, x, ldx, mul, ldmul, nullptr, rowscale, rps, out, accumulate, ws, s);
  if (dtype == DFM_F32) return colred<float, 0>(rows, C, x, ldx, mul, ldmul, nullptr, rowscale, rps, out, accumulate, ws, s);
  dfm_set_error("dfm_colsum: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_cast(int din, int dout, long n, const void* x, void* y, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return DFM_OK;
  const unsigned g = ew_grid(n);
  if (din == DFM_F32 && dout == DFM_BF16) DFM_LAUNCH((cast_kernel<float, bf16_t>), dim3(g), dim3(256), 0, s, n, (const float*)x, (bf16_t*)y);
  else if (din == DFM_BF16 && dout == DFM_F32) DFM_LAUNCH((cast_kernel<bf16_t, float>), dim3(g), dim3(256), 0, s, n, (const bf16_t*)x, (float*)y);
  else if (din == DFM_F32 && dout == DFM_F32) DFM_LAUNCH((cast_kernel<float, float>), dim3(g), dim3(256), 0, s, n, (const float*)x, (float*)y);
  else if (din == DFM_BF16 && dout == DFM_BF16) DFM_LAUNCH((cast_kernel<bf16_t, bf16_t>), dim3(g), dim3(256), 0, s, n, (const bf16_t*)x, (bf16_t*)y);
  else if (din == DFM_F32 && dout == DFM_F16) DFM_LAUNCH((cast_kernel<float, f16_t>), dim3(g), dim3(256), 0, s, n, (const float*)x, (f16_t*)y);
  else if (din == DFM_F16 && dout == DFM_F32) DFM_LAUNCH((cast_kernel<f16_t, float>), dim3(g), dim3(256), 0, s, n, (const f16_t*)x, (float*)y);
  else if (din == DFM_F16 && dout == DFM_F16) DFM_LAUNCH((cast_kernel<f16_t, f16_t>), dim3(g), dim3(256), 0, s, n, (const f16_t*)x, (f16_t*)y);
  else {
    dfm_set_error("dfm_cast: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ---- pack n row-major [rows, cols] sources (each float32 / bf16 / f16) side by side into one
// [rows, n * cols] destination (the NMF backward's rank-R input-gradient factors, ham_head.py:120-145)
constexpr int PACK_MAX = 32;
struct PackSrc {
  const void* p[PACK_MAX];
  int dt[PACK_MAX];
};

template <typename TO>
__global__ __launch_bounds__(256) void pack_slices_kernel(PackSrc src, int n, long rows, int cols, TO* __restrict__ dst) {
  const long total = rows * (long)n * cols;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long r = e / ((long)n * cols);
    const int q = (int)(e - r * n * cols), i = q / cols, c = q - i * cols;
    const long si = r * cols + c;
    float v;
    if (src.dt[i] == DFM_F32) v = ((const float*)src.p[i])[si];
    else if (src.dt[i] == DFM_BF16) v = bf2f(((const bf16_t*)src.p[i])[si]);
    else v = Num<f16_t>::to_f(((const f16_t*)src.p[i])[si]);
    dst[e] = Num<TO>::from_f(v);
  }
}

// 8 consecutive elements of one source slice per thread (cols % 8 == 0, 16-byte aligned sources):
// one or two 16-byte loads, one 16-byte store (the scalar kernel above ran at ~0.3 of HBM on the
// NMF backward's 157 MB factor pack)
template <typename TO>
__global__ __launch_bounds__(256) void pack_slices_vec_kernel(PackSrc src, int n, long rows, int cols,
                                                              TO* __restrict__ dst) {
  const int cv = cols / 8;
  const long total = rows * (long)n * cv;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const long r = v / ((long)n * cv);
    const int q = (int)(v - r * n * cv), i = q / cv, c = (q - i * cv) * 8;
    const long si = r * cols + c;
    float f[8];
    if (src.dt[i] == DFM_F32) {
      const float4 a = *reinterpret_cast<const float4*>((const float*)src.p[i] + si);
      const float4 b = *reinterpret_cast<const float4*>((const float*)src.p[i] + si + 4);
      f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    } else if (src.dt[i] == DFM_BF16) {
      ld8<bf16_t>((const bf16_t*)src.p[i] + si, f);
    } else {
      ld8<f16_t>((const f16_t*)src.p[i] + si, f);
    }
    st8<TO>(dst + v * 8, f);
  }
}

extern "C" int dfm_pack_slices(int dtype_out, int n, const void* const* srcs, const int* src_dtypes, long rows,
                               int cols, void* dst, dfm_stream_t stream) {
  DFM_CHECK_ARG(n >= 1 && n <= PACK_MAX && srcs && src_dtypes && dst && rows >= 0 && cols > 0,
                "dfm_pack_slices: 1 <= n <= %d sources, non-null pointers", PACK_MAX);
  PackSrc ps{};
  for (int i = 0; i < n; ++i) {
    DFM_CHECK_ARG(srcs[i] != nullptr, "dfm_pack_slices: null source %d", i);
    DFM_CHECK_ARG(src_dtypes[i] == DFM_F32 || src_dtypes[i] == DFM_BF16 || src_dtypes[i] == DFM_F16,
                  "dfm_pack_slices: bad source dtype %d", src_dtypes[i]);
    ps.p[i] = srcs[i];
    ps.dt[i] = src_dtypes[i];
  }
  if (rows == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  bool vec = cols % 8 == 0 && (dtype_out == DFM_BF16 || dtype_out == DFM_F16) && (uintptr_t)dst % 16 == 0;
  for (int i = 0; i < n; ++i) vec = vec && (uintptr_t)srcs[i] % 16 == 0;
  if (vec) {
    const unsigned gv = ew_grid(rows * (long)n * cols / 8);
    if (dtype_out == DFM_BF16)
      DFM_LAUNCH(pack_slices_vec_kernel<bf16_t>, dim3(gv), dim3(256), 0, s, ps, n, rows, cols, (bf16_t*)dst);
    else
      DFM_LAUNCH(pack_slices_vec_kernel<f16_t>, dim3(gv), dim3(256), 0, s, ps, n, rows, cols, (f16_t*)dst);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  const unsigned g = ew_grid(rows * (long)n * cols);
  if (dtype_out == DFM_BF16) DFM_LAUNCH(pack_slices_kernel<bf16_t>, dim3(g), dim3(256), 0, s, ps, n, rows, cols, (bf16_t*)dst);
  else if (dtype_out == DFM_F16) DFM_LAUNCH(pack_slices_kernel<f16_t>, dim3(g), dim3(256), 0, s, ps, n, rows, cols, (f16_t*)dst);
  else if (dtype_out == DFM_F32) DFM_LAUNCH(pack_slices_kernel<float>, dim3(g), dim3(256), 0, s, ps, n, rows, cols, (float*)dst);
  else {
    dfm_set_error("dfm_pack_slices: bad dtype %d", dtype_out);
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ---- deferred second stages of up to PSG_MAX reductions in one launch: block b belongs to the sum q
// with blk0[q] <= b < blk0[q + 1] and reduces its 64 columns exactly as partial_sum_kernel does
// (16 row-lanes in block order, then the 16 lanes in order), so the results are bit-identical.
constexpr int PSG_MAX = 16;
struct PsGroup {
  DfmPartialSum p[PSG_MAX];
  int blk0[PSG_MAX + 1];
  int count;
};

__global__ __launch_bounds__(1024) void partial_sum_group_kernel(PsGroup g) {
  int q = 0;
  while (q + 1 < g.count && (int)blockIdx.x >= g.blk0[q + 1]) ++q;
  const DfmPartialSum& ps = g.p[q];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const long e = (blockIdx.x - g.blk0[q]) * 64L + cl;
  const float s = e < ps.n ? ps_lane_sum(ps.part, ps.n, e, ps.nblk, rl) : 0.f;
  __shared__ float red[16][64];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && e < ps.n) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += red[r][cl];
    float* dst;
    if (ps.layout == 0) dst = ps.out0 + e;
    else if (ps.layout == 1) dst = e < ps.n0 ? ps.out0 + e : ps.out1 + (e - ps.n0);
    else {
      const long c = e / ps.n0, i = e % ps.n0;
      dst = i < ps.n0 - 1 ? ps.out0 + c * (ps.n0 - 1) + i : (ps.out1 ? ps.out1 + c : nullptr);
    }
    if (dst) *dst = ps.accumulate ? *dst + v : v;
  }
}

extern "C" int dfm_partial_sum_group(int n, const DfmPartialSum* sums, dfm_stream_t stream) {
  DFM_CHECK_ARG(n >= 0 && (n == 0 || sums), "dfm_partial_sum_group: bad argument");
  hipStream_t s = (hipStream_t)stream;
  PsGroup g{};
  auto issue = [&]() -> int {
    if (g.count == 0) return DFM_OK;
    DFM_LAUNCH(partial_sum_group_kernel, dim3(g.blk0[g.count]), dim3(1024), 0, s, g);
    DFM_LAUNCH_CHECK();
    g = PsGroup{};
    return DFM_OK;
  };
  for (int i = 0; i < n; ++i) {
    const DfmPartialSum& p = sums[i];
    if (p.n == 0) continue;  // an entry point that returned before its first stage
    DFM_CHECK_ARG(p.n > 0 && p.nblk >= 0 && p.part && p.out0 && p.layout >= 0 && p.layout <= 2 &&
                      (p.layout != 1 || (p.out1 && p.n0 > 0 && p.n0 < p.n)) && (p.layout != 2 || p.n0 >= 2),
                  "dfm_partial_sum_group: malformed sum %d", i);
    if (g.count == PSG_MAX) {
      const int r = issue();
      if (r != DFM_OK) return r;
    }
    g.p[g.count] = p;
    g.blk0[g.count + 1] = g.blk0[g.count] + (int)cdiv(p.n, 64);
    ++g.count;
  }
  return issue();
}

extern "C" int dfm_gelu_bwd(int dtype, long rows, int C, const void* dy, long lddy, const void* pre, long ldpre,
                            void* dx, long lddx, int accumulate, dfm_stream_t stream) {
  DFM_CHECK_ARG(dy && pre && dx, "dfm_gelu_bwd: null argument");
  return ew2d<1>(dtype, rows, C, dy, lddy, pre, ldpre, nullptr, nullptr, 1, 1.f, dx, lddx, accumulate, (hipStream_t)stream);
}

extern "C" int dfm_relu_bwd(int dtype, long rows, int C, const void* dy, long lddy, const void* y, long ldy, void* dx,
                            long lddx, dfm_stream_t stream) {
  DFM_CHECK_ARG(dy && y && dx, "dfm_relu_bwd: null argument");
  return ew2d<2>(dtype, rows, C, dy, lddy, y, ldy, nullptr, nullptr, 1, 1.f, dx, lddx, 0, (hipStream_t)stream);
}

extern "C" int dfm_scale_mul(int dtype, long rows, int C, const void* src, long ldsrc, const void* mul, long ldmul,
                             const float* colscale, const float* rowscale, long rps, float alpha, void* dst,
                             long lddst, int accumulate, dfm_stream_t stream) {
  DFM_CHECK_ARG(src && dst, "dfm_scale_mul: null argument");
  return ew2d<0>(dtype, rows, C, src, ldsrc, mul, ldmul, colscale, rowscale, rps, alpha, dst, lddst, accumulate,
                 (hipStream_t)stream);
}

template <typename T>
__global__ __launch_bounds__(256) void group_scale_kernel(long rows, int C, const T* __restrict__ x, long ldx,
                                                          const float* __restrict__ scale, long rpg, T* y, long ldy) {
  const int nv = C / 8;
  const long n = rows * nv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long r = i / nv;
    const int c = (int)(i - r * nv) * 8;
    const float* sc = scale + (r / rpg) * C + c;
    float v[8];
    ld8<T>(x + r * ldx + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= sc[e];
    st8<T>(y + r * ldy + c, v);
  }
}

extern "C" int dfm_group_scale(int dtype, long rows, int C, const void* x, long ldx, const float* scale,
                               long rows_per_group, void* y, long ldy, dfm_stream_t stream) {
  DFM_CHECK_ARG(x && y && scale && rows_per_group > 0 && C > 0, "dfm_group_scale: bad argument");
  DFM_CHECK_ARG(dtype == DFM_BF16 || dtype == DFM_F16 || dtype == DFM_F32, "dfm_group_scale: bad dtype %d", dtype);
  if (rows == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = C % 8 == 0 && ew_al<float>(x, ldx) && ew_al<float>(y, ldy);
  if (!vec || dtype == DFM_F32) {  // fp32 / unaligned: the elementwise path, one group at a time
    for (long r0 = 0; r0 < rows; r0 += rows_per_group) {
      const long n = std::min(rows_per_group, rows - r0);
      const long eb = dtype == DFM_F32 ? 4 : 2;
      const int rc = ew2d<0>(dtype, n, C, (const char*)x + r0 * ldx * eb, ldx, nullptr, 0,
                             scale + (r0 / rows_per_group) * C, nullptr, 1, 1.f, (char*)y + r0 * ldy * eb, ldy, 0, s);
      if (rc) return rc;
    }
    return DFM_OK;
  }
  const unsigned g = ew_grid(rows * C / 8);
  if (dtype == DFM_BF16)
    DFM_LAUNCH(group_scale_kernel<bf16_t>, dim3(g), dim3(256), 0, s, rows, C, (const bf16_t*)x, ldx, scale,
               rows_per_group, (bf16_t*)y, ldy);
  else
    DFM_LAUNCH(group_scale_kernel<f16_t>, dim3(g), dim3(256), 0, s, rows, C, (const f16_t*)x, ldx, scale,
               rows_per_group, (f16_t*)y, ldy);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_dual_mul(int dtype, long rows, int C, const void* src, long ldsrc, const void* m1, long ld1,
                            const void* m2, long ld2, void* o1, long ldo1, void* o2, long ldo2, dfm_stream_t stream) {
  DFM_CHECK_ARG(src && m1 && m2 && o1 && o2, "dfm_dual_mul: null argument");
  if (rows * C == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = C % 8 == 0 && ew_al<float>(src, ldsrc) && ew_al<float>(m1, ld1) && ew_al<float>(m2, ld2) &&
                   ew_al<float>(o1, ldo1) && ew_al<float>(o2, ldo2);
  if (!vec) {  // two scale_mul passes
    int rc = ew2d<0>(dtype, rows, C, src, ldsrc, m1, ld1, nullptr, nullptr, 1, 1.f, o1, ldo1, 0, s);
    if (rc) return rc;
    return ew2d<0>(dtype, rows, C, src, ldsrc, m2, ld2, nullptr, nullptr, 1, 1.f, o2, ldo2, 0, s);
  }
  const unsigned g = ew_grid(rows * C / 8);
  return DFM_DTYPE_SWITCH(dtype, T, [&] {
    DFM_LAUNCH(dual_mul_vec_kernel<T>, dim3(g), dim3(256), 0, s, rows, C, (const T*)src, ldsrc, (const T*)m1, ld1,
               (const T*)m2, ld2, (T*)o1, ldo1, (T*)o2, ldo2);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }());
}

extern "C" int dfm_bn_stats(int dtype, long rows, int C, const void* x, long ldx, float* stats, void* ws,
                            dfm_stream_t stream) {
  DFM_CHECK_ARG(x && stats && ws, "dfm_bn_stats: null argument");
  hipStream_t s = (hipStream_t)stream;
  DFM_CHECK_ARG(rows > 0, "dfm_bn_stats: no rows");
  if (dtype == DFM_BF16)
    return colred<bf16_t, 1>(rows, C, x, ldx, nullptr, 0, nullptr, nullptr, 1, stats, 0, ws, s, stats + 2 * C);
  else if (dtype == DFM_F16)
    return colred<f16_t, 1>(rows, C, x, ldx, nullptr, 0, nullptr, nullptr, 1, stats, 0, ws, s, stats + 2 * C);
  if (dtype == DFM_F32)
    return colred<float, 1>(rows, C, x, ldx, nullptr, 0, nullptr, nullptr, 1, stats, 0, ws, s, stats + 2 * C);
  dfm_set_error("dfm_bn_stats: bad dtype");
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_bn_finalize(int C, const float* stats, double count, float eps, float momentum, float* mean,
                               float* rstd, float* rm, float* rv, dfm_stream_t stream) {
  DFM_LAUNCH(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, C, stats, count, eps,
                     momentum, mean, rstd, rm, rv);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_bn_merge(int shards, int C, const float* parts, const float* counts, float* stats,
                            dfm_stream_t stream) {
  DFM_CHECK_ARG(parts && counts && stats && shards > 0 && C > 0, "dfm_bn_merge: bad argument");
  DFM_LAUNCH(bn_merge_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, shards, C, parts, counts,
             stats);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_bn_apply(int dtype, long rows, int C, const void* x, long ldx, const float* mean, const float* rstd,
                            const float* gamma, const float* beta, const void* res, long ldres, int act, void* y,
                            long ldy, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (C % 8 == 0 && ew_al<float>(x, ldx) && ew_al<float>(res, ldres) && ew_al<float>(y, ldy)) {
    const unsigned gv = ew_grid(rows * C / 8);
    if (dtype == DFM_BF16)
      DFM_LAUNCH(bn_apply_vec_kernel<bf16_t>, dim3(gv), dim3(256), 0, s, rows, C, (const bf16_t*)x, ldx, mean,
                         rstd, gamma, beta, (const bf16_t*)res, ldres, act, (bf16_t*)y, ldy);
    else if (dtype == DFM_F16)
      DFM_LAUNCH(bn_apply_vec_kernel<f16_t>, dim3(gv), dim3(256), 0, s, rows, C, (const f16_t*)x, ldx, mean,
                         rstd, gamma, beta, (const f16_t*)res, ldres, act, (f16_t*)y, ldy);
    else
      DFM_LAUNCH(bn_apply_vec_kernel<float>, dim3(gv), dim3(256), 0, s, rows, C, (const float*)x, ldx, mean,
                         rstd, gamma, beta, (const float*)res, ldres, act, (float*)y, ldy);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  const unsigned g = ew_grid(rows * C);
  if (dtype == DFM_BF16)
    DFM_LAUNCH(bn_apply_kernel<bf16_t>, dim3(g), dim3(256), 0, s, rows, C, (const bf16_t*)x, ldx, mean, rstd,
                       gamma, beta, (const bf16_t*)res, ldres, act, (bf16_t*)y, ldy);
  else if (dtype == DFM_F16)
    DFM_LAUNCH(bn_apply_kernel<f16_t>, dim3(g), dim3(256), 0, s, rows, C, (const f16_t*)x, ldx, mean, rstd,
                       gamma, beta, (const f16_t*)res, ldres, act, (f16_t*)y, ldy);
  else
    DFM_LAUNCH(bn_apply_kernel<float>, dim3(g), dim3(256), 0, s, rows, C, (const float*)x, ldx, mean, rstd,
                       gamma, beta, (const float*)res, ldres, act, (float*)y, ldy);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_bn_bwd_stats(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                                const float* mean, const float* rstd, float* stats2, void* ws, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return colred<bf16_t, 2>(rows, C, x, ldx, dy, lddy, mean, rstd, 1, stats2, 0, ws, s);
  else if (dtype == DFM_F16) return colred<f16_t, 2>(rows, C, x, ldx, dy, lddy, mean, rstd, 1, stats2, 0, ws, s);
  return colred<float, 2>(rows, C, x, ldx, dy, lddy, mean, rstd, 1, stats2, 0, ws, s);
}

extern "C" int dfm_bn_bwd_apply(int dtype, long rows, int C, const void* x, long ldx, const void* dy, long lddy,
                                const float* mean, const float* rstd, const float* gamma, const float* stats2,
                                double count, void* dx, long lddx, int accumulate, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const float inv_n = (float)(1.0 / count);
  if (C % 8 == 0 && ew_al<float>(x, ldx) && ew_al<float>(dy, lddy) && ew_al<float>(dx, lddx)) {
    const unsigned gv = ew_grid(rows * C / 8);
    if (dtype == DFM_BF16)
      DFM_LAUNCH(bn_bwd_apply_vec_kernel<bf16_t>, dim3(gv), dim3(256), 0, s, rows, C, (const bf16_t*)x, ldx,
                         (const bf16_t*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (bf16_t*)dx, lddx, accumulate);
    else if (dtype == DFM_F16)
      DFM_LAUNCH(bn_bwd_apply_vec_kernel<f16_t>, dim3(gv), dim3(256), 0, s, rows, C, (const f16_t*)x, ldx,
                         (const f16_t*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (f16_t*)dx, lddx, accumulate);
    else
      DFM_LAUNCH(bn_bwd_apply_vec_kernel<float>, dim3(gv), dim3(256), 0, s, rows, C, (const float*)x, ldx,
                         (const float*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (float*)dx, lddx, accumulate);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  const unsigned g = ew_grid(rows * C);
  if (dtype == DFM_BF16)
    DFM_LAUNCH(bn_bwd_apply_kernel<bf16_t>, dim3(g), dim3(256), 0, s, rows, C, (const bf16_t*)x, ldx,
                       (const bf16_t*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (bf16_t*)dx, lddx, accumulate);
  else if (dtype == DFM_F16)
    DFM_LAUNCH(bn_bwd_apply_kernel<f16_t>, dim3(g), dim3(256), 0, s, rows, C, (const f16_t*)x, ldx,
                       (const f16_t*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (f16_t*)dx, lddx, accumulate);
  else
    DFM_LAUNCH(bn_bwd_apply_kernel<float>, dim3(g), dim3(256), 0, s, rows, C, (const float*)x, ldx,
                       (const float*)dy, lddy, mean, rstd, gamma, stats2, inv_n, (float*)dx, lddx, accumulate);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_nmf_update(long n, const float* a, const float* num, const float* den, float eps, float* out,
                              void* out16, int copy_dtype, dfm_stream_t stream) {
  DFM_CHECK_ARG(!out16 || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_nmf_update: bad copy dtype");
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(nmf_update_kernel<f16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, a, num, den, eps, out,
               (f16_t*)out16);
  else
    DFM_LAUNCH(nmf_update_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, a, num, den, eps,
               out, (bf16_t*)out16);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_nmf_update_bwd(long n, const float* g, const float* a, const float* num, const float* den,
                                  const float* out, float eps, float* ga, int acc, float* gnum, float* gden,
                                  void* gnum16, int copy_dtype, dfm_stream_t stream) {
  DFM_CHECK_ARG(!gnum16 || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_nmf_update_bwd: bad copy dtype");
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(nmf_update_bwd_kernel<f16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, g, a, num, den,
               out, eps, ga, acc, gnum, gden, (f16_t*)gnum16);
  else
    DFM_LAUNCH(nmf_update_bwd_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, g, a, num, den,
               out, eps, ga, acc, gnum, gden, (bf16_t*)gnum16);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ---- NMF updates with the R x R denominator products fused (R = 64). A block owns 64 rows of one
// batch; the 64 x 64 row tile (transposed: [k][row]) and the Gram matrices sit in LDS, and thread
// (ty, tx) computes a 4 x 4 block of the row-by-Gram product (4 + 4 operands per k for 16 FMAs).
constexpr int NMF_R = 64, NMF_P = 68;  // rank, LDS pitch (floats)

DFM_INLINE void nmf_tile_t(float* sT, const float* src, long rows, long n0) {  // sT[k][r] = src[n0 + r][k]
  for (int i = threadIdx.x; i < 64 * 16; i += 256) {
    const int r = i / 16, k4 = (i % 16) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n0 + r < rows) v = *reinterpret_cast<const float4*>(src + (n0 + r) * NMF_R + k4);
    sT[(k4 + 0) * NMF_P + r] = v.x;
    sT[(k4 + 1) * NMF_P + r] = v.y;
    sT[(k4 + 2) * NMF_P + r] = v.z;
    sT[(k4 + 3) * NMF_P + r] = v.w;
  }
}
DFM_INLINE void nmf_gram(float* sG, const float* G, bool sym) {  // sG[k][c] = G[k][c] (+ G[c][k])
  for (int i = threadIdx.x; i < 64 * 16; i += 256) {
    const int k = i / 16, c4 = (i % 16) * 4;
    float4 v = *reinterpret_cast<const float4*>(G + k * NMF_R + c4);
    if (sym) {
      v.x += G[(c4 + 0) * NMF_R + k];
      v.y += G[(c4 + 1) * NMF_R + k];
      v.z += G[(c4 + 2) * NMF_R + k];
      v.w += G[(c4 + 3) * NMF_R + k];
    }
    *reinterpret_cast<float4*>(sG + k * NMF_P + c4) = v;
  }
}
DFM_INLINE void nmf_rowmm(float (&acc)[4][4], const float* sT, const float* sG, int ty, int tx) {
#pragma unroll 8
  for (int k = 0; k < NMF_R; ++k) {
    const float4 av = *reinterpret_cast<const float4*>(sT + k * NMF_P + 4 * ty);
    const float4 gv = *reinterpret_cast<const float4*>(sG + k * NMF_P + 4 * tx);
    const float ar[4] = {av.x, av.y, av.z, av.w}, gc[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(ar[i], gc[j], acc[i][j]);
  }
}

template <typename TC>
__global__ __launch_bounds__(256) void nmf_update_mm_kernel(long rows, const float* __restrict__ a,
                                                            const float* __restrict__ num, const float* __restrict__ M,
                                                            float eps, float* __restrict__ den, float* __restrict__ out,
                                                            TC* __restrict__ out16) {
  __shared__ __attribute__((aligned(16))) float sT[NMF_R * NMF_P], sG[NMF_R * NMF_P];
  const long b = blockIdx.y, n0 = (long)blockIdx.x * 64, off = b * rows * NMF_R;
  nmf_gram(sG, M + b * NMF_R * NMF_R, false);
  nmf_tile_t(sT, a + off, rows, n0);
  __syncthreads();
  const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;
  float acc[4][4] = {};
  nmf_rowmm(acc, sT, sG, ty, tx);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long n = n0 + 4 * ty + i;
    if (n >= rows) break;
    const long e = off + n * NMF_R + 4 * tx;
    const float4 av = *reinterpret_cast<const float4*>(a + e), nv = *reinterpret_cast<const float4*>(num + e);
    const float ar[4] = {av.x, av.y, av.z, av.w}, nr[4] = {nv.x, nv.y, nv.z, nv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ar[j] * nr[j] / (acc[i][j] + eps);
    *reinterpret_cast<float4*>(den + e) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
    *reinterpret_cast<float4*>(out + e) = make_float4(o[0], o[1], o[2], o[3]);
    if (out16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) out16[e + j] = Num<TC>::from_f(o[j]);
    }
  }
}

template <typename TC>
__global__ __launch_bounds__(256) void nmf_update_bwd_mm_kernel(
    long rows, const float* __restrict__ g, const float* __restrict__ A2, const float* __restrict__ S,
    const float* __restrict__ a, const float* __restrict__ num, const float* __restrict__ den,
    const float* __restrict__ out, float eps, const float* __restrict__ Mg, float* __restrict__ ga, int acc_ga,
    float* __restrict__ gnum, float* __restrict__ gden, TC* __restrict__ gnum16) {
  __shared__ __attribute__((aligned(16))) float sT[NMF_R * NMF_P], sS[NMF_R * NMF_P], sM[NMF_R * NMF_P];
  const long b = blockIdx.y, n0 = (long)blockIdx.x * 64, off = b * rows * NMF_R;
  const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;
  if (A2) {
    nmf_gram(sS, S + b * NMF_R * NMF_R, true);
    nmf_tile_t(sT, A2 + off, rows, n0);
  }
  if (Mg) nmf_gram(sM, Mg + b * NMF_R * NMF_R, false);
  __syncthreads();
  float ge[4][4] = {};
  if (A2) nmf_rowmm(ge, sT, sS, ty, tx);
  float gd[4][4] = {}, gav[4][4] = {};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long n = n0 + 4 * ty + i;
    if (n >= rows) break;
    const long e = off + n * NMF_R + 4 * tx;
    const float4 gv = *reinterpret_cast<const float4*>(g + e), av = *reinterpret_cast<const float4*>(a + e);
    const float4 nv = *reinterpret_cast<const float4*>(num + e), dv = *reinterpret_cast<const float4*>(den + e);
    const float4 ov = *reinterpret_cast<const float4*>(out + e);
    const float gr[4] = {gv.x, gv.y, gv.z, gv.w}, ar[4] = {av.x, av.y, av.z, av.w}, nr[4] = {nv.x, nv.y, nv.z, nv.w};
    const float dr[4] = {dv.x, dv.y, dv.z, dv.w}, orr[4] = {ov.x, ov.y, ov.z, ov.w};
    float gn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gi = gr[j] + ge[i][j];
      const float r = 1.f / (dr[j] + eps);
      gav[i][j] = gi * nr[j] * r;
      gn[j] = gi * ar[j] * r;
      gd[i][j] = -gi * orr[j] * r;
    }
    *reinterpret_cast<float4*>(gnum + e) = make_float4(gn[0], gn[1], gn[2], gn[3]);
    *reinterpret_cast<float4*>(gden + e) = make_float4(gd[i][0], gd[i][1], gd[i][2], gd[i][3]);
    if (gnum16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) gnum16[e + j] = Num<TC>::from_f(gn[j]);
    }
  }
  if (Mg) {  // ga += gden Mg: this block's gden rows, transposed into the tile buffer
    __syncthreads();  // every thread is done reading the A2 tile
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sT[(4 * tx + j) * NMF_P + 4 * ty + i] = gd[i][j];
    __syncthreads();
    nmf_rowmm(gav, sT, sM, ty, tx);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long n = n0 + 4 * ty + i;
    if (n >= rows) break;
    const long e = off + n * NMF_R + 4 * tx;
    float4 v = make_float4(gav[i][0], gav[i][1], gav[i][2], gav[i][3]);
    if (acc_ga) {
      const float4 o = *reinterpret_cast<const float4*>(ga + e);
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    *reinterpret_cast<float4*>(ga + e) = v;
  }
}

static bool nmf_mm_al(const void* p) { return p == nullptr || (uintptr_t)p % 16 == 0; }

extern "C" int dfm_nmf_update_mm(int batch, long rows, int R, const float* a, const float* num, const float* M,
                                 float eps, float* den, float* out, void* out16, int copy_dtype, dfm_stream_t stream) {
  DFM_CHECK_ARG(R == NMF_R, "dfm_nmf_update_mm: R=%d unsupported (64 only)", R);
  DFM_CHECK_ARG(batch > 0 && rows >= 0 && a && num && M && den && out, "dfm_nmf_update_mm: bad argument");
  DFM_CHECK_ARG(!out16 || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_nmf_update_mm: bad copy dtype");
  DFM_CHECK_ARG(nmf_mm_al(a) && nmf_mm_al(num) && nmf_mm_al(M) && nmf_mm_al(den) && nmf_mm_al(out),
                "dfm_nmf_update_mm: 16-byte aligned operands required");
  if (rows == 0) return DFM_OK;
  const dim3 grid(cdiv(rows, 64), batch);
  hipStream_t s = (hipStream_t)stream;
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(nmf_update_mm_kernel<f16_t>, grid, dim3(256), 0, s, rows, a, num, M, eps, den, out, (f16_t*)out16);
  else
    DFM_LAUNCH(nmf_update_mm_kernel<bf16_t>, grid, dim3(256), 0, s, rows, a, num, M, eps, den, out, (bf16_t*)out16);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_nmf_update_bwd_mm(int batch, long rows, int R, const float* g, const float* A2, const float* S,
                                     const float* a, const float* num, const float* den, const float* out, float eps,
                                     const float* Mg, float* ga, int accumulate_ga, float* gnum, float* gden,
                                     void* gnum16, int copy_dtype, dfm_stream_t stream) {
  DFM_CHECK_ARG(R == NMF_R, "dfm_nmf_update_bwd_mm: R=%d unsupported (64 only)", R);
  DFM_CHECK_ARG(batch > 0 && rows >= 0 && g && a && num && den && out && ga && gnum && gden && (!A2 || S),
                "dfm_nmf_update_bwd_mm: bad argument");
  DFM_CHECK_ARG(!gnum16 || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_nmf_update_bwd_mm: bad copy dtype");
  DFM_CHECK_ARG(nmf_mm_al(g) && nmf_mm_al(A2) && nmf_mm_al(S) && nmf_mm_al(a) && nmf_mm_al(num) && nmf_mm_al(den) &&
                    nmf_mm_al(out) && nmf_mm_al(Mg) && nmf_mm_al(ga) && nmf_mm_al(gnum) && nmf_mm_al(gden),
                "dfm_nmf_update_bwd_mm: 16-byte aligned operands required");
  if (rows == 0) return DFM_OK;
  const dim3 grid(cdiv(rows, 64), batch);
  hipStream_t s = (hipStream_t)stream;
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(nmf_update_bwd_mm_kernel<f16_t>, grid, dim3(256), 0, s, rows, g, A2, S, a, num, den, out, eps, Mg, ga,
               accumulate_ga, gnum, gden, (f16_t*)gnum16);
  else
    DFM_LAUNCH(nmf_update_bwd_mm_kernel<bf16_t>, grid, dim3(256), 0, s, rows, g, A2, S, a, num, den, out, eps, Mg, ga,
               accumulate_ga, gnum, gden, (bf16_t*)gnum16);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_grad_nonfinite(long n, const float* g, int* flag, dfm_stream_t stream) {
  DFM_CHECK_ARG(g && flag && n >= 0, "dfm_grad_nonfinite: bad argument");
  if (n == 0) return DFM_OK;
  DFM_LAUNCH(nonfinite_kernel, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, g, flag);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_softmax_rows(long rows, int R, const float* x, float* y, dfm_stream_t stream) {
  DFM_LAUNCH(softmax_rows_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, rows, R, x, y);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_softmax_rows_bwd(long rows, int R, const float* y, const float* dy, float* dx, int acc,
                                    dfm_stream_t stream) {
  DFM_LAUNCH(softmax_rows_bwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, rows, R, y, dy, dx,
                     acc);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_adamw(long n, float* p, const float* g, float* m, float* v, float lr, float beta1, float beta2,
                         float eps, float wd, int step, float gscale, void* copy, int copy_dtype,
                         dfm_stream_t stream) {
  DFM_CHECK_ARG(p && g && m && v && step >= 1, "dfm_adamw: bad argument");
  DFM_CHECK_ARG(!copy || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_adamw: bad copy dtype");
  if (n == 0) return DFM_OK;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(adamw_kernel<f16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, lr, beta1,
               beta2, eps, wd, bc1, sqrtf(bc2), gscale, (f16_t*)copy);
  else
    DFM_LAUNCH(adamw_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, lr, beta1,
               beta2, eps, wd, bc1, sqrtf(bc2), gscale, (bf16_t*)copy);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_adamw_dev(long n, float* p, const float* g, float* m, float* v, const float* hyper, float beta1,
                             float beta2, float eps, float wd, float gscale, void* copy, int copy_dtype,
                             dfm_stream_t stream) {
  DFM_CHECK_ARG(p && g && m && v && hyper, "dfm_adamw_dev: bad argument");
  DFM_CHECK_ARG(!copy || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_adamw_dev: bad copy dtype");
  if (n == 0) return DFM_OK;
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(adamw_dev_kernel<f16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, hyper,
               beta1, beta2, eps, wd, gscale, (f16_t*)copy, nullptr, nullptr);
  else
    DFM_LAUNCH(adamw_dev_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, hyper,
               beta1, beta2, eps, wd, gscale, (bf16_t*)copy, nullptr, nullptr);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_adamw_amp(long n, float* p, const float* g, float* m, float* v, const float* hyper,
                             const float* amp, const int* flag, float beta1, float beta2, float eps, float wd,
                             float gscale, void* copy, int copy_dtype, dfm_stream_t stream) {
  DFM_CHECK_ARG(p && g && m && v && hyper && amp && flag, "dfm_adamw_amp: bad argument");
  DFM_CHECK_ARG(!copy || copy_dtype == DFM_BF16 || copy_dtype == DFM_F16, "dfm_adamw_amp: bad copy dtype");
  if (n == 0) return DFM_OK;
  if (copy_dtype == DFM_F16)
    DFM_LAUNCH(adamw_dev_kernel<f16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, hyper,
               beta1, beta2, eps, wd, gscale, (f16_t*)copy, amp, flag);
  else
    DFM_LAUNCH(adamw_dev_kernel<bf16_t>, dim3(ew_grid(n)), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v, hyper,
               beta1, beta2, eps, wd, gscale, (bf16_t*)copy, amp, flag);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_loss_scale_update(float* amp, int* flag, float growth, float backoff, int interval,
                                     dfm_stream_t stream) {
  DFM_CHECK_ARG(amp && flag && interval > 0, "dfm_loss_scale_update: bad argument");
  DFM_LAUNCH(loss_scale_update_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, amp, flag, growth, backoff,
             interval);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

// ================================================================ residual / layer-scale backward
namespace {
constexpr int RES_BLOCKS = 512;

// One pass over dout and f: df = dout * colscale * rowscale (written) and per-block partial column
// sums of dout * f * rowscale. Thread layout: 8 consecutive columns per thread (16-byte vectors for
// bf16), TPR = C/8 threads per row, 256/TPR rows in flight per block.
template <typename T>
__global__ __launch_bounds__(256) void residual_bwd_kernel(long rows, int C, const T* __restrict__ dout, long ldo,
                                                           const T* __restrict__ f, long ldf_,
                                                           const float* __restrict__ colscale,
                                                           const float* __restrict__ rowscale, long rps,
                                                           T* __restrict__ df, long lddf, float* __restrict__ part) {
  const int TPR = C / 8;
  const int RL = 256 / TPR;
  const int tc = threadIdx.x % TPR, rl = threadIdx.x / TPR;
  const int c0 = tc * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = colscale ? colscale[c0 + e] : 1.f;
  const long per = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = (long)blockIdx.x * per, r1 = min(rows, r0 + per);
  if (rl < RL) {
    for (long r = r0 + rl; r < r1; r += RL) {
      const float rs = rowscale ? rowscale[r / rps] : 1.f;
      float d[8], fv[8], o[8];
      ld8<T>(dout + r * ldo + c0, d);
      ld8<T>(f + r * ldf_ + c0, fv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[e] += d[e] * fv[e] * rs;
        o[e] = d[e] * cs[e] * rs;
      }
      st8<T>(df + r * lddf + c0, o);
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int t = c / 8, e = c % 8;
    float s = 0.f;
    for (int q = 0; q < RL; ++q) s += red[q * TPR + t][e];
    part[(long)blockIdx.x * C + c] = s;
  }
}
}  // namespace

extern "C" size_t dfm_residual_bwd_workspace(long rows, int C) { return (size_t)RES_BLOCKS * C * sizeof(float); }

extern "C" int dfm_residual_bwd(int dtype, long rows, int C, const void* dout, long lddout, const void* f, long ldf_,
                                const float* colscale, const float* rowscale, long rps, void* df, long lddf,
                                float* dscale, void* ws, DfmPartialSum* defer, dfm_stream_t stream) {
  if (defer) *defer = DfmPartialSum{};
  DFM_CHECK_ARG(dout && f && df && dscale && ws && C % 8 == 0 && C <= 2048, "dfm_residual_bwd: bad argument");
  DFM_CHECK_ARG(lddout % 8 == 0 && ldf_ % 8 == 0 && lddf % 8 == 0 && (uintptr_t)dout % 16 == 0 &&
                    (uintptr_t)f % 16 == 0 && (uintptr_t)df % 16 == 0,
                "dfm_residual_bwd: rows must be 16-byte aligned");
  if (rows == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (int)min((long)RES_BLOCKS, max(1L, rows / 64));
  if (dtype == DFM_BF16)
    DFM_LAUNCH(residual_bwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, rows, C, (const bf16_t*)dout, lddout,
                       (const bf16_t*)f, ldf_, colscale, rowscale, rps > 0 ? rps : 1, (bf16_t*)df, lddf, (float*)ws);
  else if (dtype == DFM_F16)
    DFM_LAUNCH(residual_bwd_kernel<f16_t>, dim3(nblk), dim3(256), 0, s, rows, C, (const f16_t*)dout, lddout,
                       (const f16_t*)f, ldf_, colscale, rowscale, rps > 0 ? rps : 1, (f16_t*)df, lddf, (float*)ws);
  else if (dtype == DFM_F32)
    DFM_LAUNCH(residual_bwd_kernel<float>, dim3(nblk), dim3(256), 0, s, rows, C, (const float*)dout, lddout,
                       (const float*)f, ldf_, colscale, rowscale, rps > 0 ? rps : 1, (float*)df, lddf, (float*)ws);
  else {
    dfm_set_error("dfm_residual_bwd: bad dtype");
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return second_stage(0, nblk, (long)C, (const float*)ws, dscale, nullptr, 0L, 0, defer, s);
}
