// Depthwise k x k convolution over NHWC (DFormer.py:80-81 7x7 conv/e_conv, DFormer.py:54,62 3x3
// pos + identity). HBM-bound: a (TH+k-1) x (TW+k-1) x CB halo tile is staged in LDS once and
// every thread produces a TW-pixel output row of one channel from register sliding windows.
// The weight gradient is reduced deterministically: per-block partials [block][C][k*k+1] and a
// second pass that sums them in a fixed order.
#include "common.h"

namespace {
constexpr int TH = 8, TW = 16;

template <typename T, int K, int CB, bool FLIP>
__global__ __launch_bounds__(256) void dw_fwd_kernel(int B, int H, int W, int C, const T* __restrict__ x, long ldx,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     int add_identity, T* __restrict__ y, long ldy, int accumulate,
                                                     T* __restrict__ gout, long ldg) {
  constexpr int R = K / 2, IH = TH + K - 1, IW = TW + K - 1;
  constexpr int RG = 256 / CB;  // row groups
  static_assert(RG == TH, "thread layout: one output row per thread");
  __shared__ float tile[IH * IW * CB];
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  int bid = blockIdx.x;
  const int tw = bid % tiles_w; bid /= tiles_w;
  const int th = bid % tiles_h; bid /= tiles_h;
  const int b = bid;
  const int c0 = blockIdx.y * CB;
  const int h0 = th * TH, w0 = tw * TW;
  const long img = (long)b * H * W;
  for (int e = threadIdx.x; e < IH * IW * CB; e += 256) {
    const int c = e % CB, pix = e / CB;
    const int ih = pix / IW, iw = pix % IW;
    const int hh = h0 + ih - R, ww = w0 + iw - R;
    float v = 0.f;
    if (hh >= 0 && hh < H && ww >= 0 && ww < W && c0 + c < C) v = ldf(x + (img + (long)hh * W + ww) * ldx + c0 + c);
    tile[e] = v;
  }
  __syncthreads();
  const int c = threadIdx.x % CB, r = threadIdx.x / CB;
  const int cc = c0 + c;
  if (cc >= C || h0 + r >= H) return;
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = w[(long)cc * K * K + (FLIP ? (K * K - 1 - i) : i)];
  float acc[TW];
  const float b0 = bias ? bias[cc] : 0.f;
#pragma unroll
  for (int j = 0; j < TW; ++j) acc[j] = b0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    float row[IW];
#pragma unroll
    for (int j = 0; j < IW; ++j) row[j] = tile[((r + i) * IW + j) * CB + c];
#pragma unroll
    for (int kj = 0; kj < K; ++kj)
#pragma unroll
      for (int j = 0; j < TW; ++j) acc[j] += wk[i * K + kj] * row[j + kj];
  }
  if (add_identity) {
#pragma unroll
    for (int j = 0; j < TW; ++j) acc[j] += tile[((r + R) * IW + j + R) * CB + c];
  }
  T* yr = y + (img + (long)(h0 + r) * W + w0) * ldy + cc;
#pragma unroll
  for (int j = 0; j < TW; ++j) {
    if (w0 + j < W) {
      float v = acc[j];
      if (accumulate) v += ldf(yr + (long)j * ldy);
      stf(yr + (long)j * ldy, v);
      if (gout) stf(gout + (img + (long)(h0 + r) * W + w0 + j) * ldg + cc, gelu_f(v));
    }
  }
}

// dW partials. Block (tile_chunk, cblock) loops over `tpb` output tiles of one channel block.
template <typename T, int K, int CB>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(int B, int H, int W, int C, const T* __restrict__ x, long ldx,
                                                       const T* __restrict__ dy, long lddy, int tpb,
                                                       float* __restrict__ part) {
  constexpr int R = K / 2, IH = TH + K - 1, IW = TW + K - 1, KK = K * K;
  __shared__ float tile[IH * IW * CB];
  __shared__ float red[4][KK + 1][CB];
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  const int ntiles = B * tiles_h * tiles_w;
  const int c0 = blockIdx.y * CB;
  const int c = threadIdx.x % CB, r = threadIdx.x / CB;
  const int cc = c0 + c;
  float acc[KK + 1];
#pragma unroll
  for (int i = 0; i <= KK; ++i) acc[i] = 0.f;
  for (int t = blockIdx.x * tpb; t < min(ntiles, (int)(blockIdx.x + 1) * tpb); ++t) {
    int bid = t;
    const int tw = bid % tiles_w; bid /= tiles_w;
    const int th = bid % tiles_h; bid /= tiles_h;
    const int b = bid;
    const int h0 = th * TH, w0 = tw * TW;
    const long img = (long)b * H * W;
    __syncthreads();
    for (int e = threadIdx.x; e < IH * IW * CB; e += 256) {
      const int ce = e % CB, pix = e / CB;
      const int ih = pix / IW, iw = pix % IW;
      const int hh = h0 + ih - R, ww = w0 + iw - R;
      float v = 0.f;
      if (hh >= 0 && hh < H && ww >= 0 && ww < W && c0 + ce < C) v = ldf(x + (img + (long)hh * W + ww) * ldx + c0 + ce);
      tile[e] = v;
    }
    __syncthreads();
    if (cc < C && h0 + r < H) {
      float g[TW];
      const T* gr = dy + (img + (long)(h0 + r) * W + w0) * lddy + cc;
#pragma unroll
      for (int j = 0; j < TW; ++j) g[j] = (w0 + j < W) ? ldf(gr + (long)j * lddy) : 0.f;
#pragma unroll
      for (int j = 0; j < TW; ++j) acc[KK] += g[j];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        float row[IW];
#pragma unroll
        for (int j = 0; j < IW; ++j) row[j] = tile[((r + i) * IW + j) * CB + c];
#pragma unroll
        for (int kj = 0; kj < K; ++kj) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < TW; ++j) s += g[j] * row[j + kj];
          acc[i * K + kj] += s;
        }
      }
    }
  }
  // reduce over the TH row-threads of each channel: lanes c and c+32 share a wave when CB == 32
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  for (int i = 0; i <= KK; ++i) {
    float v = acc[i];
    v += __shfl_xor(v, 32, 64);  // the wave holds rows r = 2*wave, 2*wave+1 of the same 32 channels
    if ((threadIdx.x & 63) < CB) red[wave][i][c] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < (KK + 1) * CB; e += 256) {
    const int ce = e % CB, i = e / CB;
    if (c0 + ce < C) {
      const float v = red[0][i][ce] + red[1][i][ce] + red[2][i][ce] + red[3][i][ce];
      part[((long)blockIdx.x * C + c0 + ce) * (KK + 1) + i] = v;
    }
  }
}

__global__ void dw_wgrad_sum_kernel(int nblk, int C, int KK1, const float* __restrict__ part, float* __restrict__ dw,
                                    float* __restrict__ db) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= C * KK1) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += part[(long)b * C * KK1 + e];
  const int c = e / KK1, i = e % KK1;
  if (i < KK1 - 1) dw[c * (KK1 - 1) + i] = s;
  else if (db) db[c] = s;
}

int pick_cb(int) { return 32; }  // channels beyond C are masked

int tiles_of(int B, int H, int W) { return B * ((H + TH - 1) / TH) * ((W + TW - 1) / TW); }

template <typename T, bool FLIP>
int dw_fwd(int B, int H, int W, int C, int k, const void* x, long ldx, const float* w, const float* bias, int id,
           void* y, long ldy, int acc, void* gout, long ldg, hipStream_t s) {
  const int CB = pick_cb(C);
  dim3 grid(tiles_of(B, H, W), cdiv(C, CB));
#define GO(KK, CBB)                                                                                             \
  hipLaunchKernelGGL((dw_fwd_kernel<T, KK, CBB, FLIP>), grid, dim3(256), 0, s, B, H, W, C, (const T*)x, ldx, w, \
                     bias, id, (T*)y, ldy, acc, (T*)gout, ldg)
  if (k == 7) GO(7, 32);
  else if (k == 3) GO(3, 32);
  else {
    dfm_set_error("dwconv: k=%d unsupported", k);
    return DFM_ERR_ARG;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  return DFM_OK;
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

static int wgrad_blocks(int B, int H, int W, int& tpb) {
  const int nt = tiles_of(B, H, W);
  tpb = max(1, (nt + 255) / 256);  // ~256 blocks per channel block
  return (nt + tpb - 1) / tpb;
}

extern "C" size_t dfm_dwconv_bwd_weight_workspace(int B, int H, int W, int C, int k) {
  int tpb;
  const int nb = wgrad_blocks(B, H, W, tpb);
  return (size_t)nb * C * (k * k + 1) * sizeof(float);
}

extern "C" int dfm_dwconv_bwd_weight(int dtype, int B, int H, int W, int C, int k, const void* x, long ldx,
                                     const void* dy, long lddy, float* dw, float* db, void* workspace,
                                     dfm_stream_t stream) {
  DFM_CHECK_ARG(x && dy && dw && workspace, "dfm_dwconv_bwd_weight: null argument");
  DFM_CHECK_ARG(k == 3 || k == 7, "dfm_dwconv_bwd_weight: k=%d unsupported", k);
  hipStream_t s = (hipStream_t)stream;
  int tpb;
  const int nb = wgrad_blocks(B, H, W, tpb);
  const int CB = 32;
  dim3 grid(nb, cdiv(C, CB));
  float* part = (float*)workspace;
#define GO(TT, KK)                                                                                            \
  hipLaunchKernelGGL((dw_wgrad_kernel<TT, KK, 32>), grid, dim3(256), 0, s, B, H, W, C, (const TT*)x, ldx,      \
                     (const TT*)dy, lddy, tpb, part)
  if (dtype == DFM_BF16) {
    if (k == 7) GO(bf16_t, 7); else GO(bf16_t, 3);
  } else if (dtype == DFM_F32) {
    if (k == 7) GO(float, 7); else GO(float, 3);
  } else {
    dfm_set_error("dfm_dwconv_bwd_weight: bad dtype");
    return DFM_ERR_DTYPE;
  }
#undef GO
  DFM_LAUNCH_CHECK();
  hipLaunchKernelGGL(partial_sum_kernel<2>, dim3(cdiv((long)C * (k * k + 1), 64)), dim3(1024), 0, s, nb,
                     (long)C * (k * k + 1), (const float*)part, dw, db, (long)(k * k + 1), 0);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
