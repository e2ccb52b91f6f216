// DFormer's pooled-query RGB-D attention (DFormer.py:106-131) on NHWC:
//   AdaptiveAvgPool2d(7) of cat(LN x, LN x_e)  -> 49 queries (after short_cut_linear, a GEMM)
//   softmax(q k^T / sqrt(dh)) v over ALL H*W keys of the image, per head
//   bilinear 7x7 -> HxW (align_corners=False) written straight into its slice of the fusion tensor.
// The attention is split over key chunks (flash-style partial max / sum / output + a combine
// pass), so K and V are read exactly once per head; the backward recomputes P from the saved
// log-sum-exp and writes dK/dV per chunk directly, dQ through per-chunk partials.
#include "common.h"

namespace {
// ------------------------------------------------------------------ adaptive average pool 7x7
DFM_INLINE int bin_lo(int i, int n) { return (i * n) / 7; }
DFM_INLINE int bin_hi(int i, int n) { return ((i + 1) * n + 6) / 7; }

template <typename T>
__global__ void pool7_fwd_kernel(int B, int H, int W, int C, const T* __restrict__ x, long ldx, T* __restrict__ y,
                                 long ldy) {
  const int cell = blockIdx.x % 49, b = blockIdx.x / 49;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const int i = cell / 7, j = cell % 7;
  const int h0 = bin_lo(i, H), h1 = bin_hi(i, H), w0 = bin_lo(j, W), w1 = bin_hi(j, W);
  float s = 0.f;
  for (int h = h0; h < h1; ++h)
    for (int w = w0; w < w1; ++w) s += ldf(x + ((long)(b * H + h) * W + w) * ldx + c);
  stf(y + ((long)b * 49 + cell) * ldy + c, s / (float)((h1 - h0) * (w1 - w0)));
}

template <typename T>
__global__ void pool7_bwd_kernel(int B, int H, int W, int C, const T* __restrict__ dy, long lddy, T* __restrict__ dx,
                                 long lddx, int accumulate) {
  const long n = (long)B * H * W * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % C;
    const long pix = e / C;
    const int w = pix % W, h = (pix / W) % H, b = pix / ((long)W * H);
    float s = 0.f;
    for (int i = 0; i < 7; ++i) {  // bins overlap (and repeat rows when H < 7): test all 7
      const int h0 = bin_lo(i, H), h1 = bin_hi(i, H);
      if (h < h0 || h >= h1) continue;
      for (int j = 0; j < 7; ++j) {
        const int w0 = bin_lo(j, W), w1 = bin_hi(j, W);
        if (w < w0 || w >= w1) continue;
        s += ldf(dy + ((long)b * 49 + i * 7 + j) * lddy + c) / (float)((h1 - h0) * (w1 - w0));
      }
    }
    T* p = dx + pix * lddx + c;
    if (accumulate) s += ldf(p);
    stf(p, s);
  }
}

// ------------------------------------------------------------------ bilinear, align_corners=False
DFM_INLINE void src_index(int dst, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = scale * (dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

template <typename T>
__global__ void bilinear_fwd_kernel(int B, int Hi, int Wi, int Ho, int Wo, int C, const T* __restrict__ x, long ldx,
                                    T* __restrict__ y, long ldy, int accumulate) {
  const long n = (long)B * Ho * Wo * C;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % C;
    const long pix = e / C;
    const int wo = pix % Wo, ho = (pix / Wo) % Ho, b = pix / ((long)Wo * Ho);
    int h0, h1, w0, w1;
    float lh, lw;
    src_index(ho, Hi, Ho, h0, h1, lh);
    src_index(wo, Wi, Wo, w0, w1, lw);
    const T* xb = x + (long)b * Hi * Wi * ldx + c;
    const float v = (1.f - lh) * ((1.f - lw) * ldf(xb + ((long)h0 * Wi + w0) * ldx) + lw * ldf(xb + ((long)h0 * Wi + w1) * ldx)) +
                    lh * ((1.f - lw) * ldf(xb + ((long)h1 * Wi + w0) * ldx) + lw * ldf(xb + ((long)h1 * Wi + w1) * ldx));
    T* p = y + pix * ldy + c;
    stf(p, accumulate ? v + ldf(p) : v);
  }
}

// weight with which output index o reads input index i (0 if none)
DFM_INLINE float tap_weight(int o, int i, int in, int out) {
  int i0, i1;
  float l1;
  src_index(o, in, out, i0, i1, l1);
  float w = 0.f;
  if (i0 == i) w += 1.f - l1;
  if (i1 == i) w += l1;
  return w;
}

template <typename T>
__global__ void bilinear_bwd_kernel(int B, int Hi, int Wi, int Ho, int Wo, int C, const T* __restrict__ dy, long lddy,
                                    T* __restrict__ dx, long lddx, int accumulate) {
  const long n = (long)B * Hi * Wi * C;
  const float sh = (float)Ho / (float)Hi, sw = (float)Wo / (float)Wi;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % C;
    const long pix = e / C;
    const int wi = pix % Wi, hi = (pix / Wi) % Hi, b = pix / ((long)Wi * Hi);
    // outputs that can touch input row hi: src in (hi-1, hi+1)  =>  o in ((hi-0.5)*s-0.5, (hi+1.5)*s-0.5)
    const int ho0 = max(0, (int)floorf((hi - 0.5f) * sh - 0.5f) - 1);
    const int ho1 = min(Ho - 1, (int)ceilf((hi + 1.5f) * sh - 0.5f) + 1);
    const int wo0 = max(0, (int)floorf((wi - 0.5f) * sw - 0.5f) - 1);
    const int wo1 = min(Wo - 1, (int)ceilf((wi + 1.5f) * sw - 0.5f) + 1);
    float s = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho) {
      const float wh = tap_weight(ho, hi, Hi, Ho);
      if (wh == 0.f) continue;
      float r = 0.f;
      for (int wo = wo0; wo <= wo1; ++wo) {
        const float ww = tap_weight(wo, wi, Wi, Wo);
        if (ww != 0.f) r += ww * ldf(dy + ((long)(b * Ho + ho) * Wo + wo) * lddy + c);
      }
      s += wh * r;
    }
    T* p = dx + pix * lddx + c;
    stf(p, accumulate ? s + ldf(p) : s);
  }
}


// ------------------------------------------------------------------ 8-channel vector forms
// (C % 8 == 0, 16-byte aligned rows). Each lane moves 8 channels per 16-byte access.
inline bool vec_ok(int C, const void* p, long ld) {
  return C % 8 == 0 && ld % 8 == 0 && (uintptr_t)p % 16 == 0;
}

// pool: one block per (image, cell); CV = C/8 lanes per pixel, 256/CV pixels of the bin in
// flight, partial sums meet in LDS in a fixed order.
template <typename T>
__global__ __launch_bounds__(256) void pool7_fwd_vec_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                            long ldx, T* __restrict__ y, long ldy) {
  extern __shared__ float pred[];  // [PG][C]
  const int cell = blockIdx.x % 49, b = blockIdx.x / 49;
  const int CV = C / 8, PG = 256 / CV;
  const int cv = threadIdx.x % CV, pg = threadIdx.x / CV;
  const int i = cell / 7, j = cell % 7;
  const int h0 = bin_lo(i, H), h1 = bin_hi(i, H), w0 = bin_lo(j, W), w1 = bin_hi(j, W);
  const int nw = w1 - w0, npix = (h1 - h0) * nw;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pg < PG) {
    for (int q = pg; q < npix; q += PG) {
      const int h = h0 + q / nw, w = w0 + q % nw;
      float v[8];
      ld8<T>(x + ((long)(b * H + h) * W + w) * ldx + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) pred[pg * C + cv * 8 + e] = acc[e];
  }
  __syncthreads();
  const float inv = 1.f / (float)npix;
  for (int c = threadIdx.x; c < C; c += 256) {
    float t = 0.f;
    for (int g = 0; g < PG; ++g) t += pred[g * C + c];
    stf(y + ((long)b * 49 + cell) * ldy + c, t * inv);
  }
}

// pool backward: one lane per (pixel, 8 channels), gathering the overlapping bins it lies in.
template <typename T>
__global__ void pool7_bwd_vec_kernel(int B, int H, int W, int C, const T* __restrict__ dy, long lddy,
                                     T* __restrict__ dx, long lddx, int accumulate) {
  const int CV = C / 8;
  const long n = (long)B * H * W * CV;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % CV) * 8;
    const long pix = e / CV;
    const int w = pix % W, h = (pix / W) % H, b = pix / ((long)W * H);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // for n >= 7 a row lies in bins ic-1..ic+1 only; smaller maps repeat rows over more bins
    const int ic = (h * 7) / H, jc = (w * 7) / W;
    const int ia = H >= 7 ? max(0, ic - 1) : 0, ib = H >= 7 ? min(6, ic + 1) : 6;
    const int ja = W >= 7 ? max(0, jc - 1) : 0, jb = W >= 7 ? min(6, jc + 1) : 6;
    for (int i = ia; i <= ib; ++i) {
      const int ha = bin_lo(i, H), hb = bin_hi(i, H);
      if (h < ha || h >= hb) continue;
      for (int j = ja; j <= jb; ++j) {
        const int wa = bin_lo(j, W), wb = bin_hi(j, W);
        if (w < wa || w >= wb) continue;
        const float inv = 1.f / (float)((hb - ha) * (wb - wa));
        float v[8];
        ld8<T>(dy + ((long)b * 49 + i * 7 + j) * lddy + c, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) s[q] += v[q] * inv;
      }
    }
    T* p = dx + pix * lddx + c;
    if (accumulate) {
      float o[8];
      ld8<T>(p, o);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += o[q];
    }
    st8<T>(p, s);
  }
}

template <typename T>
__global__ void bilinear_fwd_vec_kernel(int B, int Hi, int Wi, int Ho, int Wo, int C, const T* __restrict__ x,
                                        long ldx, T* __restrict__ y, long ldy, int accumulate) {
  const int CV = C / 8;
  const long n = (long)B * Ho * Wo * CV;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % CV) * 8;
    const long pix = e / CV;
    const int wo = pix % Wo, ho = (pix / Wo) % Ho, b = pix / ((long)Wo * Ho);
    int h0, h1, w0, w1;
    float lh, lw;
    src_index(ho, Hi, Ho, h0, h1, lh);
    src_index(wo, Wi, Wo, w0, w1, lw);
    const T* xb = x + (long)b * Hi * Wi * ldx + c;
    float v00[8], v01[8], v10[8], v11[8], o[8];
    ld8<T>(xb + ((long)h0 * Wi + w0) * ldx, v00);
    ld8<T>(xb + ((long)h0 * Wi + w1) * ldx, v01);
    ld8<T>(xb + ((long)h1 * Wi + w0) * ldx, v10);
    ld8<T>(xb + ((long)h1 * Wi + w1) * ldx, v11);
    T* p = y + pix * ldy + c;
    if (accumulate) ld8<T>(p, o);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float v = (1.f - lh) * ((1.f - lw) * v00[q] + lw * v01[q]) + lh * ((1.f - lw) * v10[q] + lw * v11[q]);
      o[q] = accumulate ? o[q] + v : v;
    }
    st8<T>(p, o);
  }
}

// bilinear backward (a gather): one block per input cell (b, hi, wi); the output rows / columns
// that read the cell and their tap weights go to LDS once, then CV lanes per output pixel walk the
// window with 16-byte loads and the partial sums meet in LDS in a fixed order.
constexpr int BL_MAXT = 64;
template <typename T>
__global__ __launch_bounds__(256) void bilinear_bwd_vec_kernel(int B, int Hi, int Wi, int Ho, int Wo, int C,
                                                               const T* __restrict__ dy, long lddy,
                                                               T* __restrict__ dx, long lddx, int accumulate) {
  extern __shared__ float bred[];  // [PG][C]
  __shared__ int rows[BL_MAXT], cols[BL_MAXT];
  __shared__ float rw[BL_MAXT], cw[BL_MAXT];
  __shared__ int nr, nc;
  const int wi = blockIdx.x % Wi, hi = (blockIdx.x / Wi) % Hi, b = blockIdx.x / (Wi * Hi);
  if (threadIdx.x == 0) {
    const float sh = (float)Ho / (float)Hi, sw = (float)Wo / (float)Wi;
    const int ho0 = max(0, (int)floorf((hi - 0.5f) * sh - 0.5f) - 1);
    const int ho1 = min(Ho - 1, (int)ceilf((hi + 1.5f) * sh - 0.5f) + 1);
    const int wo0 = max(0, (int)floorf((wi - 0.5f) * sw - 0.5f) - 1);
    const int wo1 = min(Wo - 1, (int)ceilf((wi + 1.5f) * sw - 0.5f) + 1);
    int k = 0;
    for (int ho = ho0; ho <= ho1 && k < BL_MAXT; ++ho) {
      const float t = tap_weight(ho, hi, Hi, Ho);
      if (t != 0.f) { rows[k] = ho; rw[k] = t; ++k; }
    }
    nr = k;
    k = 0;
    for (int wo = wo0; wo <= wo1 && k < BL_MAXT; ++wo) {
      const float t = tap_weight(wo, wi, Wi, Wo);
      if (t != 0.f) { cols[k] = wo; cw[k] = t; ++k; }
    }
    nc = k;
  }
  __syncthreads();
  const int CV = C / 8, PG = 256 / CV;
  const int cv = threadIdx.x % CV, pg = threadIdx.x / CV;
  const int npix = nr * nc;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (pg < PG) {
    for (int q = pg; q < npix; q += PG) {
      const int r = q / nc, k = q % nc;
      const float wgt = rw[r] * cw[k];
      float v[8];
      ld8<T>(dy + ((long)(b * Ho + rows[r]) * Wo + cols[k]) * lddy + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(wgt, v[e], acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) bred[pg * C + cv * 8 + e] = acc[e];
  }
  __syncthreads();
  const long pix = (long)(b * Hi + hi) * Wi + wi;
  for (int c = threadIdx.x; c < C; c += 256) {
    float t = 0.f;
    for (int g = 0; g < PG; ++g) t += bred[g * C + c];
    T* p = dx + pix * lddx + c;
    stf(p, accumulate ? t + ldf(p) : t);
  }
}

// ------------------------------------------------------------------ pooled attention
constexpr int NQ = 49;
constexpr int NC = 64;  // keys per chunk

struct AttnArgs {
  int B, heads, N, dh, nchunk;
  const void* q;
  long ldq;
  const void* k;
  const void* v;
  long ldkv;
  float scale;
  void* o;
  long ldo;
  float* lse;
  float* ws;  // partial O [b][h][chunk][49][dh], m, l [b][h][chunk][49]
  const void* dout;
  long lddo;
  void* dq;
  void* dk;
  void* dv;
  long lddkv;
};

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_chunk_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int dh = a.dh, DP = dh + 1;
  float* sQ = sm;                // [49][DP]
  float* sK = sQ + NQ * DP;      // [NC][DP]
  float* sV = sK + NC * DP;      // [NC][DP]
  float* sS = sV + NC * DP;      // [49][NC+1]
  const int chunk = blockIdx.x % a.nchunk;
  const int bh = blockIdx.x / a.nchunk;
  const int h = bh % a.heads, b = bh / a.heads;
  const int n0 = chunk * NC, nc = min(NC, a.N - n0);
  const T* q = (const T*)a.q + (long)b * NQ * a.ldq + h * dh;
  const T* k = (const T*)a.k + ((long)b * a.N + n0) * a.ldkv + h * dh;
  const T* v = (const T*)a.v + ((long)b * a.N + n0) * a.ldkv + h * dh;
  for (int e = threadIdx.x; e < NQ * dh; e += 256) sQ[(e / dh) * DP + e % dh] = ldf(q + (long)(e / dh) * a.ldq + e % dh) * a.scale;
  for (int e = threadIdx.x; e < NC * dh; e += 256) {
    const int r = e / dh, d = e % dh;
    sK[r * DP + d] = r < nc ? ldf(k + (long)r * a.ldkv + d) : 0.f;
    sV[r * DP + d] = r < nc ? ldf(v + (long)r * a.ldkv + d) : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NQ * NC; e += 256) {
    const int qi = e / NC, ki = e % NC;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += sQ[qi * DP + d] * sK[ki * DP + d];
    sS[qi * (NC + 1) + ki] = ki < nc ? s : -INFINITY;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* pm = a.ws + (long)a.B * a.heads * a.nchunk * NQ * dh;
  float* pl = pm + (long)a.B * a.heads * a.nchunk * NQ;
  const long base = ((long)bh * a.nchunk + chunk) * NQ;
  for (int qi = wid; qi < NQ; qi += 4) {
    const float s = sS[qi * (NC + 1) + lane];
    const float m = wave_max(s);
    const float p = __expf(s - m);
    sS[qi * (NC + 1) + lane] = p;
    const float l = wave_sum(p);
    if (lane == 0) {
      pm[base + qi] = m;
      pl[base + qi] = l;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NQ * dh; e += 256) {
    const int qi = e / dh, d = e % dh;
    float s = 0.f;
    for (int ki = 0; ki < nc; ++ki) s += sS[qi * (NC + 1) + ki] * sV[ki * DP + d];
    a.ws[(base + qi) * dh + d] = s;
  }
}

template <typename T>
__global__ void attn_fwd_combine_kernel(AttnArgs a) {
  const long n = (long)a.B * a.heads * NQ * a.dh;
  const float* pm = a.ws + (long)a.B * a.heads * a.nchunk * NQ * a.dh;
  const float* pl = pm + (long)a.B * a.heads * a.nchunk * NQ;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int d = e % a.dh;
    const long bhq = e / a.dh;
    const int qi = bhq % NQ;
    const long bh = bhq / NQ;
    const int h = bh % a.heads, b = bh / a.heads;
    float M = -INFINITY;
    for (int c = 0; c < a.nchunk; ++c) M = fmaxf(M, pm[(bh * a.nchunk + c) * NQ + qi]);
    float L = 0.f, O = 0.f;
    for (int c = 0; c < a.nchunk; ++c) {
      const long idx = (bh * a.nchunk + c) * NQ + qi;
      const float f = __expf(pm[idx] - M);
      L += pl[idx] * f;
      O += a.ws[idx * a.dh + d] * f;
    }
    stf((T*)a.o + ((long)b * NQ + qi) * a.ldo + h * a.dh + d, O / L);
    if (d == 0) a.lse[bhq] = M + __logf(L);
  }
}

// backward per chunk: recompute P, dV = P^T dO, dP = dO V^T, dS = P (dP - D), dK = scale dS^T Q,
// dQ_partial = scale dS K.
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_chunk_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int dh = a.dh, DP = dh + 1;
  float* sQ = sm;               // [49][DP] (unscaled q)
  float* sO = sQ + NQ * DP;     // [49][DP] dO
  float* sK = sO + NQ * DP;     // [NC][DP]
  float* sV = sK + NC * DP;     // [NC][DP]
  float* sP = sV + NC * DP;     // [49][NC+1]  P, then dS
  float* sD = sP + NQ * (NC + 1);  // [49] D, [49] lse
  const int chunk = blockIdx.x % a.nchunk;
  const int bh = blockIdx.x / a.nchunk;
  const int h = bh % a.heads, b = bh / a.heads;
  const int n0 = chunk * NC, nc = min(NC, a.N - n0);
  const T* q = (const T*)a.q + (long)b * NQ * a.ldq + h * dh;
  const T* o = (const T*)a.o + (long)b * NQ * a.ldo + h * dh;
  const T* go = (const T*)a.dout + (long)b * NQ * a.lddo + h * dh;
  const T* k = (const T*)a.k + ((long)b * a.N + n0) * a.ldkv + h * dh;
  const T* v = (const T*)a.v + ((long)b * a.N + n0) * a.ldkv + h * dh;
  for (int e = threadIdx.x; e < NQ * dh; e += 256) {
    const int qi = e / dh, d = e % dh;
    sQ[qi * DP + d] = ldf(q + (long)qi * a.ldq + d);
    sO[qi * DP + d] = ldf(go + (long)qi * a.lddo + d);
  }
  for (int e = threadIdx.x; e < NC * dh; e += 256) {
    const int r = e / dh, d = e % dh;
    sK[r * DP + d] = r < nc ? ldf(k + (long)r * a.ldkv + d) : 0.f;
    sV[r * DP + d] = r < nc ? ldf(v + (long)r * a.ldkv + d) : 0.f;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // D[q] = sum_d dO * O
  for (int qi = wid; qi < NQ; qi += 4) {
    float s = 0.f;
    for (int d = lane; d < dh; d += 64) s += ldf(go + (long)qi * a.lddo + d) * ldf(o + (long)qi * a.ldo + d);
    s = wave_sum(s);
    if (lane == 0) {
      sD[qi] = s;
      sD[NQ + qi] = a.lse[(long)bh * NQ + qi];
    }
  }
  __syncthreads();
  // P
  for (int e = threadIdx.x; e < NQ * NC; e += 256) {
    const int qi = e / NC, ki = e % NC;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += sQ[qi * DP + d] * sK[ki * DP + d];
    sP[qi * (NC + 1) + ki] = ki < nc ? __expf(s * a.scale - sD[NQ + qi]) : 0.f;
  }
  __syncthreads();
  // dV[key][d] = sum_q P[q][key] dO[q][d]   (written directly)
  T* dvp = (T*)a.dv + ((long)b * a.N + n0) * a.lddkv + h * dh;
  for (int e = threadIdx.x; e < nc * dh; e += 256) {
    const int ki = e / dh, d = e % dh;
    float s = 0.f;
    for (int qi = 0; qi < NQ; ++qi) s += sP[qi * (NC + 1) + ki] * sO[qi * DP + d];
    stf(dvp + (long)ki * a.lddkv + d, s);
  }
  __syncthreads();  // every dV reader of P is done before P is overwritten by dS
  // dS = P * (dO V^T - D)   (in place; each element read/written by one thread)
  for (int e = threadIdx.x; e < NQ * NC; e += 256) {
    const int qi = e / NC, ki = e % NC;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += sO[qi * DP + d] * sV[ki * DP + d];
    float& p = sP[qi * (NC + 1) + ki];
    p = p * (s - sD[qi]);
  }
  __syncthreads();
  // dK[key][d] = scale * sum_q dS[q][key] Q[q][d]
  T* dkp = (T*)a.dk + ((long)b * a.N + n0) * a.lddkv + h * dh;
  for (int e = threadIdx.x; e < nc * dh; e += 256) {
    const int ki = e / dh, d = e % dh;
    float s = 0.f;
    for (int qi = 0; qi < NQ; ++qi) s += sP[qi * (NC + 1) + ki] * sQ[qi * DP + d];
    stf(dkp + (long)ki * a.lddkv + d, s * a.scale);
  }
  // dQ partial
  const long base = ((long)bh * a.nchunk + chunk) * NQ;
  for (int e = threadIdx.x; e < NQ * dh; e += 256) {
    const int qi = e / dh, d = e % dh;
    float s = 0.f;
    for (int ki = 0; ki < nc; ++ki) s += sP[qi * (NC + 1) + ki] * sK[ki * DP + d];
    a.ws[(base + qi) * dh + d] = s * a.scale;
  }
}

template <typename T>
__global__ void attn_dq_reduce_kernel(AttnArgs a) {
  const long n = (long)a.B * a.heads * NQ * a.dh;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int d = e % a.dh;
    const long bhq = e / a.dh;
    const int qi = bhq % NQ;
    const long bh = bhq / NQ;
    const int h = bh % a.heads, b = bh / a.heads;
    float s = 0.f;
    for (int c = 0; c < a.nchunk; ++c) s += a.ws[((bh * a.nchunk + c) * NQ + qi) * a.dh + d];
    stf((T*)a.dq + ((long)b * NQ + qi) * a.ldq + h * a.dh + d, s);
  }
}

unsigned grid_for(long n) { return (unsigned)min((long)8192, max(1L, (n + 255) / 256)); }

template <typename F8, typename F32>
int dispatch(int dtype, F8 f8, F32 f32) {
  if (dtype == DFM_BF16) return f8();
  if (dtype == DFM_F32) return f32();
  dfm_set_error("attention: bad dtype");
  return DFM_ERR_DTYPE;
}
}  // namespace

extern "C" int dfm_adaptive_pool7_fwd(int dtype, int B, int H, int W, int C, const void* x, long ldx, void* y,
                                      long ldy, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (C <= 2048 && vec_ok(C, x, ldx)) {
    const size_t lds = (size_t)(256 / (C / 8)) * C * sizeof(float);
    return dispatch(
        dtype,
        [&] {
          hipLaunchKernelGGL(pool7_fwd_vec_kernel<bf16_t>, dim3(B * 49), dim3(256), lds, s, B, H, W, C,
                             (const bf16_t*)x, ldx, (bf16_t*)y, ldy);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          hipLaunchKernelGGL(pool7_fwd_vec_kernel<float>, dim3(B * 49), dim3(256), lds, s, B, H, W, C,
                             (const float*)x, ldx, (float*)y, ldy);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  dim3 grid(B * 49, cdiv(C, 256));
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(pool7_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, B, H, W, C, (const bf16_t*)x, ldx, (bf16_t*)y, ldy);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(pool7_fwd_kernel<float>, grid, dim3(256), 0, s, B, H, W, C, (const float*)x, ldx, (float*)y, ldy);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

extern "C" int dfm_adaptive_pool7_bwd(int dtype, int B, int H, int W, int C, const void* dy, long lddy, void* dx,
                                      long lddx, int accumulate, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (vec_ok(C, dy, lddy) && vec_ok(C, dx, lddx)) {
    const unsigned gv = grid_for((long)B * H * W * (C / 8));
    return dispatch(
        dtype,
        [&] {
          hipLaunchKernelGGL(pool7_bwd_vec_kernel<bf16_t>, dim3(gv), dim3(256), 0, s, B, H, W, C, (const bf16_t*)dy,
                             lddy, (bf16_t*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          hipLaunchKernelGGL(pool7_bwd_vec_kernel<float>, dim3(gv), dim3(256), 0, s, B, H, W, C, (const float*)dy,
                             lddy, (float*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * H * W * C);
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(pool7_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, s, B, H, W, C, (const bf16_t*)dy, lddy, (bf16_t*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(pool7_bwd_kernel<float>, dim3(g), dim3(256), 0, s, B, H, W, C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

extern "C" int dfm_bilinear_fwd(int dtype, int B, int Hi, int Wi, int Ho, int Wo, int C, const void* x, long ldx,
                                void* y, long ldy, int accumulate, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (vec_ok(C, x, ldx) && vec_ok(C, y, ldy)) {
    const unsigned gv = grid_for((long)B * Ho * Wo * (C / 8));
    return dispatch(
        dtype,
        [&] {
          hipLaunchKernelGGL(bilinear_fwd_vec_kernel<bf16_t>, dim3(gv), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C,
                             (const bf16_t*)x, ldx, (bf16_t*)y, ldy, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          hipLaunchKernelGGL(bilinear_fwd_vec_kernel<float>, dim3(gv), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C,
                             (const float*)x, ldx, (float*)y, ldy, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * Ho * Wo * C);
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(bilinear_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const bf16_t*)x, ldx, (bf16_t*)y, ldy, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(bilinear_fwd_kernel<float>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const float*)x, ldx, (float*)y, ldy, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

extern "C" int dfm_bilinear_bwd(int dtype, int B, int Hi, int Wi, int Ho, int Wo, int C, const void* dy, long lddy,
                                void* dx, long lddx, int accumulate, dfm_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  // taps per axis: ~2 * out/in + 3 must fit the block's LDS lists
  const bool taps_fit = 2 * (Ho / Hi) + 6 <= BL_MAXT && 2 * (Wo / Wi) + 6 <= BL_MAXT && Ho >= Hi && Wo >= Wi;
  if (C <= 2048 && taps_fit && vec_ok(C, dy, lddy) && (uintptr_t)dx % 4 == 0) {
    const size_t lds = (size_t)(256 / (C / 8)) * C * sizeof(float);
    return dispatch(
        dtype,
        [&] {
          hipLaunchKernelGGL(bilinear_bwd_vec_kernel<bf16_t>, dim3(B * Hi * Wi), dim3(256), lds, s, B, Hi, Wi, Ho, Wo,
                             C, (const bf16_t*)dy, lddy, (bf16_t*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          hipLaunchKernelGGL(bilinear_bwd_vec_kernel<float>, dim3(B * Hi * Wi), dim3(256), lds, s, B, Hi, Wi, Ho, Wo,
                             C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * Hi * Wi * C);
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(bilinear_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const bf16_t*)dy, lddy, (bf16_t*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(bilinear_bwd_kernel<float>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

static int nchunks(int N) { return (N + NC - 1) / NC; }

extern "C" size_t dfm_pooled_attn_workspace(int B, int heads, int N, int dh) {
  const long nchk = nchunks(N);
  return (size_t)B * heads * nchk * NQ * (dh + 2) * sizeof(float);
}

extern "C" int dfm_pooled_attn_fwd(int dtype, int B, int heads, int N, int dh, const void* q, long ldq, const void* k,
                                   const void* v, long ldkv, float scale, void* o, long ldo, float* lse,
                                   void* workspace, dfm_stream_t stream) {
  DFM_CHECK_ARG(q && k && v && o && lse && workspace && N > 0 && dh > 0 && dh <= 64, "dfm_pooled_attn_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  AttnArgs a{};
  a.B = B; a.heads = heads; a.N = N; a.dh = dh; a.nchunk = nchunks(N);
  a.q = q; a.ldq = ldq; a.k = k; a.v = v; a.ldkv = ldkv; a.scale = scale; a.o = o; a.ldo = ldo; a.lse = lse;
  a.ws = (float*)workspace;
  const int DP = dh + 1;
  const size_t lds = (size_t)(NQ * DP + 2 * NC * DP + NQ * (NC + 1)) * sizeof(float);
  const unsigned nblk = B * heads * a.nchunk;
  const unsigned g = grid_for((long)B * heads * NQ * dh);
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(attn_fwd_chunk_kernel<bf16_t>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_fwd_combine_kernel<bf16_t>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(attn_fwd_chunk_kernel<float>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_fwd_combine_kernel<float>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

extern "C" int dfm_pooled_attn_bwd(int dtype, int B, int heads, int N, int dh, const void* q, long ldq, const void* k,
                                   const void* v, long ldkv, float scale, const void* o, long ldo, const void* dout,
                                   long lddo, const float* lse, void* dq, void* dk, void* dv, long lddkv,
                                   void* workspace, dfm_stream_t stream) {
  DFM_CHECK_ARG(q && k && v && o && dout && lse && dq && dk && dv && workspace && dh <= 64,
                "dfm_pooled_attn_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  AttnArgs a{};
  a.B = B; a.heads = heads; a.N = N; a.dh = dh; a.nchunk = nchunks(N);
  a.q = q; a.ldq = ldq; a.k = k; a.v = v; a.ldkv = ldkv; a.scale = scale; a.o = const_cast<void*>(o); a.ldo = ldo; a.lse = (float*)lse;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.dk = dk; a.dv = dv; a.lddkv = lddkv;
  a.ws = (float*)workspace;
  const int DP = dh + 1;
  const size_t lds = (size_t)(2 * NQ * DP + 2 * NC * DP + NQ * (NC + 1) + 2 * NQ) * sizeof(float);
  const unsigned nblk = B * heads * a.nchunk;
  const unsigned g = grid_for((long)B * heads * NQ * dh);
  return dispatch(
      dtype,
      [&] {
        hipLaunchKernelGGL(attn_bwd_chunk_kernel<bf16_t>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_dq_reduce_kernel<bf16_t>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        hipLaunchKernelGGL(attn_bwd_chunk_kernel<float>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_dq_reduce_kernel<float>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}
