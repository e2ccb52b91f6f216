// DFormer's pooled-query RGB-D attention (DFormer.py:106-131) on NHWC:
//   AdaptiveAvgPool2d(7) of cat(LN x, LN x_e)  -> 49 queries (after short_cut_linear, a GEMM)
//   softmax(q k^T / sqrt(dh)) v over ALL H*W keys of the image, per head
//   bilinear 7x7 -> HxW (align_corners=False) written straight into its slice of the fusion tensor.
// The attention is split over key chunks (flash-style partial max / sum / output + a combine
// pass), so K and V are read exactly once per head; the backward recomputes P from the saved
// log-sum-exp and writes dK/dV per chunk directly, dQ through per-chunk partials.
#include <cstdlib>

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
inline bool vec_ok(int C, const void* p, long ld) { return C % 8 == 0 && ld % 8 == 0 && (uintptr_t)p % 16 == 0; }

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

// Combine for the MFMA path (dh % 4 == 0): one thread per (b, h, query, 4 dims) reads its partials as
// float4 and walks the chunks 4 at a time with independent maxima / sums, so a thread's loads of a
// group of chunks are in flight together instead of one dependent load per chunk.
template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_combine_v4_kernel(AttnArgs a) {
  const int d4n = a.dh / 4;
  const long n = (long)a.B * a.heads * NQ * d4n;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= n) return;
  const int d = (int)(e % d4n) * 4;
  const long bhq = e / d4n;
  const int qi = bhq % NQ;
  const long bh = bhq / NQ;
  const int h = bh % a.heads, b = bh / a.heads;
  const float* pm = a.ws + (long)a.B * a.heads * a.nchunk * NQ * a.dh;
  const float* pl = pm + (long)a.B * a.heads * a.nchunk * NQ;
  const long i0 = bh * a.nchunk * NQ + qi;  // partial (chunk c) at i0 + c * NQ
  const int nc = a.nchunk, nc4 = nc & ~3;
  float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int c = 0; c < nc4; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) m4[u] = fmaxf(m4[u], pm[i0 + (long)(c + u) * NQ]);
  }
  for (int c = nc4; c < nc; ++c) m4[0] = fmaxf(m4[0], pm[i0 + (long)c * NQ]);
  const float M = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
  float L4[4] = {0.f, 0.f, 0.f, 0.f};
  float4 O4[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) O4[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto acc = [&](int u, int c) {
    const long idx = i0 + (long)c * NQ;
    const float f = __expf(pm[idx] - M);
    const float4 o = *reinterpret_cast<const float4*>(a.ws + idx * a.dh + d);
    L4[u] += pl[idx] * f;
    O4[u].x += o.x * f;
    O4[u].y += o.y * f;
    O4[u].z += o.z * f;
    O4[u].w += o.w * f;
  };
  for (int c = 0; c < nc4; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc(u, c + u);
  }
  for (int c = nc4; c < nc; ++c) acc(0, c);
  const float L = (L4[0] + L4[1]) + (L4[2] + L4[3]);
  const float inv = 1.0f / L;
  float ov[4] = {((O4[0].x + O4[1].x) + (O4[2].x + O4[3].x)) * inv, ((O4[0].y + O4[1].y) + (O4[2].y + O4[3].y)) * inv,
                 ((O4[0].z + O4[1].z) + (O4[2].z + O4[3].z)) * inv, ((O4[0].w + O4[1].w) + (O4[2].w + O4[3].w)) * inv};
  T* op = (T*)a.o + ((long)b * NQ + qi) * a.ldo + h * a.dh + d;
#pragma unroll
  for (int u = 0; u < 4; ++u) stf(op + u, ov[u]);
  if (d == 0) a.lse[bhq] = M + __logf(L);
}

// dQ = sum over chunks of the per-chunk partials, MFMA path: float4 partials, 4 chunks in flight
template <typename T>
__global__ __launch_bounds__(256) void attn_dq_reduce_v4_kernel(AttnArgs a) {
  const int d4n = a.dh / 4;
  const long n = (long)a.B * a.heads * NQ * d4n;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= n) return;
  const int d = (int)(e % d4n) * 4;
  const long bhq = e / d4n;
  const int qi = bhq % NQ;
  const long bh = bhq / NQ;
  const int h = bh % a.heads, b = bh / a.heads;
  const float* p0 = a.ws + (bh * a.nchunk * NQ + qi) * a.dh + d;
  const long cs = (long)NQ * a.dh;  // chunk stride
  const int nc = a.nchunk, nc4 = nc & ~3;
  float4 s4[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) s4[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto add = [&](int u, int c) {
    const float4 v = *reinterpret_cast<const float4*>(p0 + c * cs);
    s4[u].x += v.x;
    s4[u].y += v.y;
    s4[u].z += v.z;
    s4[u].w += v.w;
  };
  for (int c = 0; c < nc4; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) add(u, c + u);
  }
  for (int c = nc4; c < nc; ++c) add(0, c);
  const float ov[4] = {(s4[0].x + s4[1].x) + (s4[2].x + s4[3].x), (s4[0].y + s4[1].y) + (s4[2].y + s4[3].y),
                       (s4[0].z + s4[1].z) + (s4[2].z + s4[3].z), (s4[0].w + s4[1].w) + (s4[2].w + s4[3].w)};
  T* qp = (T*)a.dq + ((long)b * NQ + qi) * a.ldq + h * a.dh + d;
#pragma unroll
  for (int u = 0; u < 4; ++u) stf(qp + u, ov[u]);
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


// ------------------------------------------------------------------ MFMA pooled attention (bf16)
// One wave owns a chunk of `kpw` keys of one (image, head) and walks it in 32-key blocks with
// v_mfma_f32_16x16x32_bf16 (fp32 accumulate); the 49 queries are padded to 64. Fragment lanes:
// A (m = lane&15, k = 8*(lane>>4)+e), B (n = lane&15, k = 8*(lane>>4)+e), C (n = lane&15,
// m = 4*(lane>>4)+r). Loading the A operand's rows in the permuted order
// row(i) = 8*(i>>2) + 4t + (i&3) for the two 16-row tiles t of a 32-row block makes the C tiles
// of the pair hold, per lane, rows 8*(lane>>4)+e in natural order: exactly a B (or A) fragment
// of the next product, so P and dS never leave registers except where a transpose is needed
// (K^T and dS^T for dQ, V^T for O: staged in LDS and read with ds_read_b64_tr_b16).
// Softmax row statistics are reduced with lane shuffles (xor 16, 32) across the 4 lane groups.
DFM_INLINE bf16x8_t ldfrag16(const bf16_t* p, bool ok) {
  if (!ok) return bf16x8_t{};
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
DFM_INLINE bf16x8_t pack_bf16x8(const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  return __builtin_bit_cast(bf16x8_t, make_uint4(w[0], w[1], w[2], w[3]));
}
// fragment (r = r0 + (lane&15), k = k0 + 8*(lane>>4) + e) of an LDS image stored [k][r] (r contiguous)
DFM_INLINE bf16x8_t frag_tr(const bf16_t* lds, int LD, int r0, int k0, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  typedef __attribute__((address_space(3))) short4_t lds_s4;
  const bf16_t* a0 = lds + (k0 + 8 * g + q) * LD + r0 + 4 * p;
  const bf16_t* a1 = a0 + 4 * LD;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a1));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  short8_t sv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, sv);
}
DFM_INLINE void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
#define MFMA16(A, B, C) mma16<T>((A), (B), (C))

// Block -> (image, head, chunk group). Heads run fastest in the logical order and the logical order
// is dealt to the XCDs in contiguous runs (blocks p and p + 8 share an XCD): the heads of one image
// whose K / V column slices share 128-byte lines (DH = 32: two heads per line) are read by blocks of
// the same XCD at the same time, so each line comes from HBM once instead of once per head.
DFM_INLINE void attn_block(int heads, int groups, int& bh, int& cg) {
  const int nblk = gridDim.x, id = blockIdx.x;
  const int xcd = id & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int h = L % heads, t = L / heads;
  cg = t % groups;
  bh = (t / groups) * heads + h;
}

// Forward: S^T = K Q^T (keys as rows), online softmax per query, O^T += V^T P^T.
// Each wave walks one chunk of keys; the block's 4 wave states (unnormalised O [49][DH], running max m
// and sum l, scaled units) are merged through LDS and wave 0 writes ONE partial per block (chunk group
// cg), so the combine kernel reads groups = nchunk / 4 partials (round 5 wrote one per wave: 7.65 MB of
// fp32 partials per launch against ~0.2 MB of output, 1.66x the kernel's algorithmic bytes). Isolated,
// forward + combine (tools/attn_kernels_bench.py): 25.5 -> 18.2 us (stage 1), 18.1 -> 13.1 (2), 11.8 ->
// 10.6 (3); the step is within noise (479.7 / 479.5 vs 479.5 / 479.1 images/s).
template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_fwd_mfma_kernel(AttnArgs a, int kpw, int groups) {
  constexpr int KD = (DH + 31) / 32, ND = DH / 16, LDV = DH + 8;
  __shared__ __attribute__((aligned(16))) bf16_t sV[4][32 * LDV];
  __shared__ float4 mO[3][4][ND][64];  // waves 1..3: O in the C-fragment layout, lane-contiguous
  __shared__ float mML[3][4][2][16];   // waves 1..3: m, l per (row tile, row)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  int bh, cg;
  attn_block(a.heads, groups, bh, cg);
  const int chunk = cg * 4 + w;  // a wave past the last chunk contributes an empty state (m = -inf, l = 0)
  const int h = bh % a.heads, b = bh / a.heads;
  const int n0 = min(a.N, chunk * kpw), n1 = chunk < a.nchunk ? min(a.N, n0 + kpw) : n0;
  const bf16_t* Q = (const bf16_t*)a.q + (long)b * NQ * a.ldq + h * DH;
  const bf16_t* K = (const bf16_t*)a.k + (long)b * a.N * a.ldkv + h * DH;
  const bf16_t* V = (const bf16_t*)a.v + (long)b * a.N * a.ldkv + h * DH;
  bf16_t* sv = sV[w];
  bf16x8_t qf[4][KD];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int ks = 0; ks < KD; ++ks) {
      const int q = 16 * nt + j, d0 = 32 * ks + 8 * g;
      qf[nt][ks] = ldfrag16(Q + (long)q * a.ldq + d0, q < NQ && d0 < DH);
    }
  float mrun[4], lrun[4];
  float4_t o[ND][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    mrun[nt] = -INFINITY;
    lrun[nt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) o[dt][nt] = float4_t{0.f, 0.f, 0.f, 0.f};
  }
  // the next 32-key block's V rows and K fragments are loaded into registers while this block is
  // multiplied (one global round trip per block hidden behind the MFMAs instead of paid in series)
  constexpr int VCH = DH / 8, VIT = (32 * VCH + 63) / 64;
  uint4 vreg[VIT];
  bf16x8_t kf[2][KD];
  auto load_block = [&](int kb, uint4 (&vr)[VIT], bf16x8_t (&kr)[2][KD]) {
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int idx = lane + 64 * it;
      const int key = idx / VCH, ch = idx % VCH;
      vr[it] = idx < 32 * VCH && kb + key < n1
                   ? *reinterpret_cast<const uint4*>(V + (long)(kb + key) * a.ldkv + ch * 8)
                   : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < KD; ++ks) {
        const int key = kb + 8 * (j >> 2) + 4 * t + (j & 3), d0 = 32 * ks + 8 * g;
        kr[t][ks] = ldfrag16(K + (long)key * a.ldkv + d0, key < n1 && d0 < DH);
      }
  };
  if (n0 < n1) load_block(n0, vreg, kf);
  for (int kb = n0; kb < n1; kb += 32) {
    // V block -> LDS [key][d] (zero rows past the chunk)
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int idx = lane + 64 * it;
      if (idx < 32 * VCH) {
        const int key = idx / VCH, ch = idx % VCH;
        *reinterpret_cast<uint4*>(sv + key * LDV + ch * 8) = vreg[it];
      }
    }
    bf16x8_t kc[2][KD];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < KD; ++ks) kc[t][ks] = kf[t][ks];
    if (kb + 32 < n1) load_block(kb + 32, vreg, kf);
    float4_t st[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        float4_t acc = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KD; ++ks) acc = MFMA16(kc[t][ks], qf[nt][ks], acc);
        st[t][nt] = acc;
      }
    bf16x8_t pf[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float sv8[8];
      float mx = -INFINITY;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int key = kb + 8 * g + e;
        const float x = key < n1 ? st[e >> 2][nt][e & 3] * a.scale : -INFINITY;
        sv8[e] = x;
        mx = fmaxf(mx, x);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(mrun[nt], mx);
      const float alpha = __expf(mrun[nt] - mnew);
      float ps = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sv8[e] = __expf(sv8[e] - mnew);
        ps += sv8[e];
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      lrun[nt] = lrun[nt] * alpha + ps;
      mrun[nt] = mnew;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) o[dt][nt] *= alpha;
      pf[nt] = pack16x8<T>(sv8);
    }
    lds_wave_sync();
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const bf16x8_t vf = frag_tr(sv, LDV, 16 * dt, 0, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) o[dt][nt] = MFMA16(vf, pf[nt], o[dt][nt]);
    }
    lds_wave_sync();  // the next block's V stage overwrites sv
  }
  if (w > 0) {  // waves 1..3 hand their state to wave 0
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
        mO[w - 1][nt][dt][lane] = make_float4(o[dt][nt][0], o[dt][nt][1], o[dt][nt][2], o[dt][nt][3]);
      if (g == 0) {
        mML[w - 1][nt][0][j] = mrun[nt];
        mML[w - 1][nt][1][j] = lrun[nt];
      }
    }
  }
  __syncthreads();
  if (w > 0) return;
  // the block's partial = the log-sum-exp merge of its waves' states (wave 0 always holds a chunk)
  const int groups_total = (a.nchunk + 3) / 4;
  float* pm = a.ws + (long)a.B * a.heads * groups_total * NQ * DH;
  float* pl = pm + (long)a.B * a.heads * groups_total * NQ;
  const long base = ((long)bh * groups_total + cg) * NQ;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int q = 16 * nt + j;
    float mw[3], M = mrun[nt];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      mw[u] = mML[u][nt][0][j];
      M = fmaxf(M, mw[u]);
    }
    const float s0 = __expf(mrun[nt] - M);
    float L = lrun[nt] * s0, su[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      su[u] = __expf(mw[u] - M);  // an empty state (m = -inf) scales to 0
      L += mML[u][nt][1][j] * su[u];
    }
    if (q >= NQ) continue;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      float4 v = make_float4(o[dt][nt][0] * s0, o[dt][nt][1] * s0, o[dt][nt][2] * s0, o[dt][nt][3] * s0);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const float4 ou = mO[u][nt][dt][lane];
        v.x += ou.x * su[u];
        v.y += ou.y * su[u];
        v.z += ou.z * su[u];
        v.w += ou.w * su[u];
      }
      *reinterpret_cast<float4*>(a.ws + (base + q) * DH + 16 * dt + 4 * g) = v;
    }
    if (g == 0) {
      pm[base + q] = M;
      pl[base + q] = L;
    }
  }
}

// Backward per wave chunk: S' = Q K^T and dP' = dO V^T with keys as columns (lane = key), then
// P' = exp(S' scale - lse), dS' = P' (dP' - D); dV^T += dO^T P', dK^T += Q^T dS' (scale), both
// complete per 32-key block and stored directly; dQ^T += K^T dS'^T through LDS (partial per chunk).
template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_bwd_mfma_kernel(AttnArgs a, int kpw, int groups) {
  constexpr int KD = (DH + 31) / 32, ND = DH / 16, LDD = DH + 8, LDQ = 64 + 8;
  __shared__ __attribute__((aligned(16))) bf16_t sQ[64 * LDD], sO[64 * LDD];
  __shared__ __attribute__((aligned(16))) bf16_t sK[4][32 * LDD], sS[4][32 * LDQ];
  __shared__ float sL[64], sD[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  int bh, cg;
  attn_block(a.heads, groups, bh, cg);
  const int chunk = cg * 4 + w;
  const int h = bh % a.heads, b = bh / a.heads;
  const bf16_t* Q = (const bf16_t*)a.q + (long)b * NQ * a.ldq + h * DH;
  const bf16_t* GO = (const bf16_t*)a.dout + (long)b * NQ * a.lddo + h * DH;
  const bf16_t* Op = (const bf16_t*)a.o + (long)b * NQ * a.ldo + h * DH;
  constexpr int VCH = DH / 8;
  for (int idx = threadIdx.x; idx < 64 * VCH; idx += 256) {  // Q, dO -> LDS [q][d], rows >= 49 zero
    const int q = idx / VCH, ch = idx % VCH;
    uint4 uq = make_uint4(0, 0, 0, 0), uo = make_uint4(0, 0, 0, 0);
    if (q < NQ) {
      uq = *reinterpret_cast<const uint4*>(Q + (long)q * a.ldq + ch * 8);
      uo = *reinterpret_cast<const uint4*>(GO + (long)q * a.lddo + ch * 8);
    }
    *reinterpret_cast<uint4*>(sQ + q * LDD + ch * 8) = uq;
    *reinterpret_cast<uint4*>(sO + q * LDD + ch * 8) = uo;
  }
  if (threadIdx.x < 64) {  // lse and D = rowsum(dO * O)
    const int q = threadIdx.x;
    float dsum = 0.f, l = 0.f;
    if (q < NQ) {
      for (int d = 0; d < DH; d += 8) {
        float x[8], y[8];
        ld8<T>((const T*)(GO + (long)q * a.lddo + d), x);
        ld8<T>((const T*)(Op + (long)q * a.ldo + d), y);
#pragma unroll
        for (int e = 0; e < 8; ++e) dsum += x[e] * y[e];
      }
      l = a.lse[(long)bh * NQ + q];
    }
    sL[q] = l;
    sD[q] = dsum;
  }
  __syncthreads();
  if (chunk >= a.nchunk) return;
  const int n0 = chunk * kpw, n1 = min(a.N, n0 + kpw);
  const bf16_t* K = (const bf16_t*)a.k + (long)b * a.N * a.ldkv + h * DH;
  const bf16_t* V = (const bf16_t*)a.v + (long)b * a.N * a.ldkv + h * DH;
  bf16_t* dK = (bf16_t*)a.dk + (long)b * a.N * a.lddkv + h * DH;
  bf16_t* dV = (bf16_t*)a.dv + (long)b * a.N * a.lddkv + h * DH;
  bf16_t* sk = sK[w];
  bf16_t* ss = sS[w];
  // per-wave constant fragments
  bf16x8_t qa[2][2][KD], oa[2][2][KD];  // A (m = q permuted, k = d)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < KD; ++ks) {
        const int q = 32 * qb + 8 * (j >> 2) + 4 * t + (j & 3), d0 = 32 * ks + 8 * g;
        qa[qb][t][ks] = ldfrag16(sQ + q * LDD + d0, d0 < DH);
        oa[qb][t][ks] = ldfrag16(sO + q * LDD + d0, d0 < DH);
      }
  bf16x8_t qt[ND][2], ot[ND][2];  // A (m = d, k = q): Q^T, dO^T
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      qt[dt][qb] = frag_tr(sQ, LDD, 16 * dt, 32 * qb, lane);
      ot[dt][qb] = frag_tr(sO, LDD, 16 * dt, 32 * qb, lane);
    }
  float Lq[2][8], Dq[2][8];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      Lq[qb][e] = sL[32 * qb + 8 * g + e];
      Dq[qb][e] = sD[32 * qb + 8 * g + e];
    }
  float4_t dq[ND][4];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dq[dt][nt] = float4_t{0.f, 0.f, 0.f, 0.f};

  // the next 32-key block's K rows and K / V fragments are loaded into registers while this block
  // is processed (its global round trip hidden behind the MFMAs)
  constexpr int KIT = (32 * VCH + 63) / 64;
  uint4 kreg[KIT];
  bf16x8_t kn[2][KD], vn[2][KD];  // B (k = d, n = key)
  auto load_block = [&](int kb) {
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int idx = lane + 64 * it;
      const int key = idx / VCH, ch = idx % VCH;
      kreg[it] = idx < 32 * VCH && kb + key < n1
                     ? *reinterpret_cast<const uint4*>(K + (long)(kb + key) * a.ldkv + ch * 8)
                     : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int ks = 0; ks < KD; ++ks) {
        const int key = kb + 16 * kt + j, d0 = 32 * ks + 8 * g;
        kn[kt][ks] = ldfrag16(K + (long)key * a.ldkv + d0, key < n1 && d0 < DH);
        vn[kt][ks] = ldfrag16(V + (long)key * a.ldkv + d0, key < n1 && d0 < DH);
      }
  };
  if (n0 < n1) load_block(n0);
  for (int kb = n0; kb < n1; kb += 32) {
#pragma unroll
    for (int it = 0; it < KIT; ++it) {  // K block -> LDS [key][d]
      const int idx = lane + 64 * it;
      if (idx < 32 * VCH) {
        const int key = idx / VCH, ch = idx % VCH;
        *reinterpret_cast<uint4*>(sk + key * LDD + ch * 8) = kreg[it];
      }
    }
    bf16x8_t kf[2][KD], vf[2][KD];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int ks = 0; ks < KD; ++ks) {
        kf[kt][ks] = kn[kt][ks];
        vf[kt][ks] = vn[kt][ks];
      }
    if (kb + 32 < n1) load_block(kb + 32);
    bf16x8_t pb[2][2], dsb[2][2];  // [kt][qb]: B (k = q 32qb + 8g + e, n = key 16kt + j)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const bool kvalid = kb + 16 * kt + j < n1;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float4_t sp[2], dp[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float4_t s4 = float4_t{0.f, 0.f, 0.f, 0.f}, d4 = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < KD; ++ks) {
            s4 = MFMA16(qa[qb][t][ks], kf[kt][ks], s4);
            d4 = MFMA16(oa[qb][t][ks], vf[kt][ks], d4);
          }
          sp[t] = s4;
          dp[t] = d4;
        }
        float p8[8], ds8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int q = 32 * qb + 8 * g + e;
          const float p = (kvalid && q < NQ) ? __expf(sp[e >> 2][e & 3] * a.scale - Lq[qb][e]) : 0.f;
          p8[e] = p;
          ds8[e] = p * (dp[e >> 2][e & 3] - Dq[qb][e]);
        }
        pb[kt][qb] = pack16x8<T>(p8);
        dsb[kt][qb] = pack16x8<T>(ds8);
        // dS' row (key) -> LDS [key][q] for the dS^T operand of dQ
        *reinterpret_cast<bf16x8_t*>(ss + (16 * kt + j) * LDQ + 32 * qb + 8 * g) = dsb[kt][qb];
      }
    }
    // dV^T, dK^T tiles of this key block (contraction over the 64 queries = 2 k-steps)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int key = kb + 16 * kt + j;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        float4_t v4 = float4_t{0.f, 0.f, 0.f, 0.f}, k4 = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          v4 = MFMA16(ot[dt][qb], pb[kt][qb], v4);
          k4 = MFMA16(qt[dt][qb], dsb[kt][qb], k4);
        }
        if (key < n1) {
          const int d = 16 * dt + 4 * g;
          uint2 uv, uk;
          uv.x = (uint32_t)bits16<T>(v4[0]) | ((uint32_t)bits16<T>(v4[1]) << 16);
          uv.y = (uint32_t)bits16<T>(v4[2]) | ((uint32_t)bits16<T>(v4[3]) << 16);
          uk.x = (uint32_t)bits16<T>(k4[0] * a.scale) | ((uint32_t)bits16<T>(k4[1] * a.scale) << 16);
          uk.y = (uint32_t)bits16<T>(k4[2] * a.scale) | ((uint32_t)bits16<T>(k4[3] * a.scale) << 16);
          *reinterpret_cast<uint2*>(dV + (long)key * a.lddkv + d) = uv;
          *reinterpret_cast<uint2*>(dK + (long)key * a.lddkv + d) = uk;
        }
      }
    }
    lds_wave_sync();
    // dQ^T[d][q] += sum_key K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const bf16x8_t ka = frag_tr(sk, LDD, 16 * dt, 0, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) dq[dt][nt] = MFMA16(ka, frag_tr(ss, LDQ, 16 * nt, 0, lane), dq[dt][nt]);
    }
    lds_wave_sync();
  }
  const long base = ((long)bh * a.nchunk + chunk) * NQ;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int q = 16 * nt + j;
    if (q >= NQ) continue;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
      *reinterpret_cast<float4*>(a.ws + (base + q) * DH + 16 * dt + 4 * g) =
          make_float4(dq[dt][nt][0] * a.scale, dq[dt][nt][1] * a.scale, dq[dt][nt][2] * a.scale,
                      dq[dt][nt][3] * a.scale);
  }
}
#undef MFMA16

// dst[r][h*ddst + d] = d < dsrc ? src[r][h*dsrc + d] : 0   (2-byte elements, d < ddst)
__global__ void head_repack_kernel(long rows, int heads, int dsrc, long lds, int ddst, long ldd,
                                   const uint16_t* __restrict__ src, uint16_t* __restrict__ dst) {
  const long n = rows * heads * ddst;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % ddst);
    const long t = i / ddst;
    const int h = (int)(t % heads);
    const long r = t / heads;
    dst[r * ldd + (long)h * ddst + d] = d < dsrc ? src[r * lds + (long)h * dsrc + d] : (uint16_t)0;
  }
}

// the same on 4-element (8-byte) chunks with 32-bit index math (dsrc, ddst, both strides multiples of 4,
// 8-byte aligned operands, rows * heads * ddst / 4 < 2^31; the host checks): the scalar kernel's 64-bit
// div / mod per 2-byte element made it ~12 us a launch on DFormer-Large's stage-2 heads
__global__ void head_repack4_kernel(int n4, int heads, int q4s, int ls4, int q4d, int ld4, const uint2* __restrict__ src,
                                    uint2* __restrict__ dst) {
  const int per_row = heads * q4d;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int r = i / per_row, c = i - r * per_row;
    const int h = c / q4d, d = c - h * q4d;
    dst[(long)r * ld4 + c] = d < q4s ? src[(long)r * ls4 + h * q4s + d] : make_uint2(0u, 0u);
  }
}

unsigned grid_for(long n) { return (unsigned)min((long)8192, max(1L, (n + 255) / 256)); }

// f16: the 16-bit lambda is generic over its storage type (bf16_t or f16_t)
template <typename F16, typename F32>
int dispatch(int dtype, F16 f16, F32 f32) {
  if (dtype == DFM_BF16) return f16(bf16_t{});
  if (dtype == DFM_F16) return f16(f16_t{});
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
        [&](auto tag16) {
        using T16 = decltype(tag16);
          DFM_LAUNCH(pool7_fwd_vec_kernel<T16>, dim3(B * 49), dim3(256), lds, s, B, H, W, C,
                             (const T16*)x, ldx, (T16*)y, ldy);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          DFM_LAUNCH(pool7_fwd_vec_kernel<float>, dim3(B * 49), dim3(256), lds, s, B, H, W, C,
                             (const float*)x, ldx, (float*)y, ldy);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  dim3 grid(B * 49, cdiv(C, 256));
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(pool7_fwd_kernel<T16>, grid, dim3(256), 0, s, B, H, W, C, (const T16*)x, ldx, (T16*)y, ldy);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(pool7_fwd_kernel<float>, grid, dim3(256), 0, s, B, H, W, C, (const float*)x, ldx, (float*)y, ldy);
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
        [&](auto tag16) {
        using T16 = decltype(tag16);
          DFM_LAUNCH(pool7_bwd_vec_kernel<T16>, dim3(gv), dim3(256), 0, s, B, H, W, C, (const T16*)dy,
                             lddy, (T16*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          DFM_LAUNCH(pool7_bwd_vec_kernel<float>, dim3(gv), dim3(256), 0, s, B, H, W, C, (const float*)dy,
                             lddy, (float*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * H * W * C);
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(pool7_bwd_kernel<T16>, dim3(g), dim3(256), 0, s, B, H, W, C, (const T16*)dy, lddy, (T16*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(pool7_bwd_kernel<float>, dim3(g), dim3(256), 0, s, B, H, W, C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
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
        [&](auto tag16) {
        using T16 = decltype(tag16);
          DFM_LAUNCH(bilinear_fwd_vec_kernel<T16>, dim3(gv), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C,
                             (const T16*)x, ldx, (T16*)y, ldy, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          DFM_LAUNCH(bilinear_fwd_vec_kernel<float>, dim3(gv), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C,
                             (const float*)x, ldx, (float*)y, ldy, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * Ho * Wo * C);
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(bilinear_fwd_kernel<T16>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const T16*)x, ldx, (T16*)y, ldy, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(bilinear_fwd_kernel<float>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const float*)x, ldx, (float*)y, ldy, accumulate);
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
        [&](auto tag16) {
        using T16 = decltype(tag16);
          DFM_LAUNCH(bilinear_bwd_vec_kernel<T16>, dim3(B * Hi * Wi), dim3(256), lds, s, B, Hi, Wi, Ho, Wo,
                             C, (const T16*)dy, lddy, (T16*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        },
        [&] {
          DFM_LAUNCH(bilinear_bwd_vec_kernel<float>, dim3(B * Hi * Wi), dim3(256), lds, s, B, Hi, Wi, Ho, Wo,
                             C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
          DFM_LAUNCH_CHECK();
          return DFM_OK;
        });
  }
  const unsigned g = grid_for((long)B * Hi * Wi * C);
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(bilinear_bwd_kernel<T16>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const T16*)dy, lddy, (T16*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(bilinear_bwd_kernel<float>, dim3(g), dim3(256), 0, s, B, Hi, Wi, Ho, Wo, C, (const float*)dy, lddy, (float*)dx, lddx, accumulate);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}

static int nchunks(int N) { return (N + NC - 1) / NC; }

// bf16 MFMA path: head dim a multiple of 16 (<= 48), 16-byte aligned rows
static bool attn_mfma_ok(int dtype, int dh, const void* const* ptrs, const long* lds, int n) {
  if ((dtype != DFM_BF16 && dtype != DFM_F16) || !(dh == 16 || dh == 32 || dh == 48)) return false;
  for (int i = 0; i < n; ++i)
    if ((uintptr_t)ptrs[i] % 16 != 0 || lds[i] % 8 != 0) return false;
  return true;
}
// Other bf16 head dims below 48 (DFormer-Large: 576 / 16 heads = 36 in stages 2-3) run the same
// MFMA kernels on head slices zero-padded to the next multiple of 16 in the workspace: padded
// dims add 0 to Q K^T and produce 0 output columns, which the unpack drops.
static int attn_pad_dh(int dtype, int dh) {
  if ((dtype != DFM_BF16 && dtype != DFM_F16) || dh % 16 == 0 || dh > 48) return 0;
  return (dh + 15) / 16 * 16;
}
static int attn_kpw(int N) { return N >= 2048 ? 128 : 64; }  // keys per wave (a multiple of 32 and of NC)

template <typename T, int DH>
static void attn_mfma_launch(AttnArgs& a, bool bwd, hipStream_t s) {
  const int kpw = attn_kpw(a.N);
  const int groups = (a.nchunk + 3) / 4;
  const dim3 grid((unsigned)(a.B * a.heads * groups));
  if (bwd) DFM_LAUNCH((attn_bwd_mfma_kernel<T, DH>), grid, dim3(256), 0, s, a, kpw, groups);
  else DFM_LAUNCH((attn_fwd_mfma_kernel<T, DH>), grid, dim3(256), 0, s, a, kpw, groups);
}
template <typename T>
static void attn_mfma_t(AttnArgs& a, bool bwd, hipStream_t s) {
  if (a.dh == 16) attn_mfma_launch<T, 16>(a, bwd, s);
  else if (a.dh == 32) attn_mfma_launch<T, 32>(a, bwd, s);
  else attn_mfma_launch<T, 48>(a, bwd, s);
}
// the 16-bit MFMA kernels (bf16 / f16 storage) and their combine / dQ-reduce kernels
static void attn_mfma(int dtype, AttnArgs& a, bool bwd, hipStream_t s) {
  if (dtype == DFM_F16) attn_mfma_t<f16_t>(a, bwd, s);
  else attn_mfma_t<bf16_t>(a, bwd, s);
}
static void attn_combine16(int dtype, AttnArgs& a, hipStream_t s) {
  const dim3 g(cdiv((long)a.B * a.heads * NQ * (a.dh / 4), 256));
  if (dtype == DFM_F16) DFM_LAUNCH(attn_fwd_combine_v4_kernel<f16_t>, g, dim3(256), 0, s, a);
  else DFM_LAUNCH(attn_fwd_combine_v4_kernel<bf16_t>, g, dim3(256), 0, s, a);
}
static void attn_dq_reduce16(int dtype, AttnArgs& a, hipStream_t s) {
  const dim3 g(cdiv((long)a.B * a.heads * NQ * (a.dh / 4), 256));
  if (dtype == DFM_F16) DFM_LAUNCH(attn_dq_reduce_v4_kernel<f16_t>, g, dim3(256), 0, s, a);
  else DFM_LAUNCH(attn_dq_reduce_v4_kernel<bf16_t>, g, dim3(256), 0, s, a);
}

static size_t attn_partials_bytes(int B, int heads, int N, int dh) {
  return ((size_t)B * heads * nchunks(N) * NQ * (dh + 2) * sizeof(float) + 255) / 256 * 256;
}
// padded-head buffers (bf16): Q, O, dO, dQ [B*49][heads*dp]; K, V, dK, dV [B*N][heads*dp]
static size_t attn_pad_elems_q(int B, int heads, int dp) { return ((size_t)B * NQ * heads * dp + 127) / 128 * 128; }
static size_t attn_pad_elems_k(int B, int heads, int N, int dp) { return ((size_t)B * N * heads * dp + 127) / 128 * 128; }

extern "C" size_t dfm_pooled_attn_workspace(int B, int heads, int N, int dh) {
  const int dp = attn_pad_dh(DFM_BF16, dh);
  if (dp == 0) return (size_t)B * heads * nchunks(N) * NQ * (dh + 2) * sizeof(float);
  return attn_partials_bytes(B, heads, N, dp) +
         (4 * attn_pad_elems_q(B, heads, dp) + 4 * attn_pad_elems_k(B, heads, N, dp)) * sizeof(uint16_t);
}

static void head_repack(long rows, int heads, int dsrc, long lds, int ddst, long ldd, const void* src, void* dst,
                        hipStream_t s) {
  const long n4 = rows * heads * (ddst / 4);
  if (dsrc % 4 == 0 && ddst % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && (uintptr_t)src % 8 == 0 &&
      (uintptr_t)dst % 8 == 0 && n4 < (1L << 31) && rows * (lds / 4) < (1L << 31) && rows * (ldd / 4) < (1L << 31)) {
    DFM_LAUNCH(head_repack4_kernel, dim3(grid_for(n4)), dim3(256), 0, s, (int)n4, heads, dsrc / 4, (int)(lds / 4),
               ddst / 4, (int)(ldd / 4), (const uint2*)src, (uint2*)dst);
    return;
  }
  DFM_LAUNCH(head_repack_kernel, dim3(grid_for(rows * heads * ddst)), dim3(256), 0, s, rows, heads, dsrc, lds, ddst,
             ldd, (const uint16_t*)src, (uint16_t*)dst);
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
  if (const int dp = attn_pad_dh(dtype, dh)) {
    uint16_t* pq = (uint16_t*)((char*)workspace + attn_partials_bytes(B, heads, N, dp));
    uint16_t* po = pq + attn_pad_elems_q(B, heads, dp);
    uint16_t* pk = po + attn_pad_elems_q(B, heads, dp);
    uint16_t* pv = pk + attn_pad_elems_k(B, heads, N, dp);
    const long ldp = (long)heads * dp;
    head_repack((long)B * NQ, heads, dh, ldq, dp, ldp, q, pq, s);
    head_repack((long)B * N, heads, dh, ldkv, dp, ldp, k, pk, s);
    head_repack((long)B * N, heads, dh, ldkv, dp, ldp, v, pv, s);
    a.dh = dp; a.q = pq; a.ldq = ldp; a.k = pk; a.v = pv; a.ldkv = ldp; a.o = po; a.ldo = ldp;
    a.nchunk = (N + attn_kpw(N) - 1) / attn_kpw(N);
    attn_mfma(dtype, a, false, s);
    a.nchunk = (a.nchunk + 3) / 4;  // one merged partial per block (chunk group)
    attn_combine16(dtype, a, s);
    head_repack((long)B * NQ, heads, dp, ldp, dh, ldo, po, o, s);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  {
    const void* ptrs[] = {q, k, v, o};
    const long lds_[] = {ldq, ldkv, ldkv, ldo};
    if (attn_mfma_ok(dtype, dh, ptrs, lds_, 4)) {
      a.nchunk = (N + attn_kpw(N) - 1) / attn_kpw(N);
      attn_mfma(dtype, a, false, s);
      DFM_LAUNCH_CHECK();
      a.nchunk = (a.nchunk + 3) / 4;  // one merged partial per block (chunk group)
      attn_combine16(dtype, a, s);
      DFM_LAUNCH_CHECK();
      return DFM_OK;
    }
  }
  const int DP = dh + 1;
  const size_t lds = (size_t)(NQ * DP + 2 * NC * DP + NQ * (NC + 1)) * sizeof(float);
  const unsigned nblk = B * heads * a.nchunk;
  const unsigned g = grid_for((long)B * heads * NQ * dh);
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(attn_fwd_chunk_kernel<T16>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        DFM_LAUNCH(attn_fwd_combine_kernel<T16>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(attn_fwd_chunk_kernel<float>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        DFM_LAUNCH(attn_fwd_combine_kernel<float>, dim3(g), dim3(256), 0, s, a);
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
  if (const int dp = attn_pad_dh(dtype, dh)) {
    const size_t eq = attn_pad_elems_q(B, heads, dp), ek = attn_pad_elems_k(B, heads, N, dp);
    uint16_t* pq = (uint16_t*)((char*)workspace + attn_partials_bytes(B, heads, N, dp));
    uint16_t* po = pq + eq;
    uint16_t* pdo = po + eq;
    uint16_t* pdq = pdo + eq;
    uint16_t* pk = pdq + eq;
    uint16_t* pv = pk + ek;
    uint16_t* pdk = pv + ek;
    uint16_t* pdv = pdk + ek;
    const long ldp = (long)heads * dp;
    head_repack((long)B * NQ, heads, dh, ldq, dp, ldp, q, pq, s);
    head_repack((long)B * NQ, heads, dh, ldo, dp, ldp, o, po, s);
    head_repack((long)B * NQ, heads, dh, lddo, dp, ldp, dout, pdo, s);
    head_repack((long)B * N, heads, dh, ldkv, dp, ldp, k, pk, s);
    head_repack((long)B * N, heads, dh, ldkv, dp, ldp, v, pv, s);
    a.dh = dp; a.q = pq; a.ldq = ldp; a.k = pk; a.v = pv; a.ldkv = ldp; a.o = po; a.ldo = ldp;
    a.dout = pdo; a.lddo = ldp; a.dq = pdq; a.dk = pdk; a.dv = pdv; a.lddkv = ldp;
    a.nchunk = (N + attn_kpw(N) - 1) / attn_kpw(N);
    attn_mfma(dtype, a, true, s);
    attn_dq_reduce16(dtype, a, s);
    head_repack((long)B * NQ, heads, dp, ldp, dh, ldq, pdq, dq, s);
    head_repack((long)B * N, heads, dp, ldp, dh, lddkv, pdk, dk, s);
    head_repack((long)B * N, heads, dp, ldp, dh, lddkv, pdv, dv, s);
    DFM_LAUNCH_CHECK();
    return DFM_OK;
  }
  {
    const void* ptrs[] = {q, k, v, o, dout, dq, dk, dv};
    const long lds_[] = {ldq, ldkv, ldkv, ldo, lddo, ldq, lddkv, lddkv};
    if (attn_mfma_ok(dtype, dh, ptrs, lds_, 8)) {
      a.nchunk = (N + attn_kpw(N) - 1) / attn_kpw(N);
      attn_mfma(dtype, a, true, s);
      DFM_LAUNCH_CHECK();
      attn_dq_reduce16(dtype, a, s);
      DFM_LAUNCH_CHECK();
      return DFM_OK;
    }
  }
  const int DP = dh + 1;
  const size_t lds = (size_t)(2 * NQ * DP + 2 * NC * DP + NQ * (NC + 1) + 2 * NQ) * sizeof(float);
  const unsigned nblk = B * heads * a.nchunk;
  const unsigned g = grid_for((long)B * heads * NQ * dh);
  return dispatch(
      dtype,
      [&](auto tag16) {
        using T16 = decltype(tag16);
        DFM_LAUNCH(attn_bwd_chunk_kernel<T16>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        DFM_LAUNCH(attn_dq_reduce_kernel<T16>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      },
      [&] {
        DFM_LAUNCH(attn_bwd_chunk_kernel<float>, dim3(nblk), dim3(256), lds, s, a);
        DFM_LAUNCH_CHECK();
        DFM_LAUNCH(attn_dq_reduce_kernel<float>, dim3(g), dim3(256), 0, s, a);
        DFM_LAUNCH_CHECK();
        return DFM_OK;
      });
}
