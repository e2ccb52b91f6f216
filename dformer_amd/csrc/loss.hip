// Segmentation loss of EncoderDecoder.forward (builder.py:203,230): bilinear upsampling of the
// low-resolution logits to the label size + cross-entropy(ignore_index) + mean over valid pixels.
// Fused: the full-resolution logits (786 MB fp32 for DFormer-B bs16) are never materialised.
// Forward: one thread per label pixel interpolates its ncls logits from the 4 taps, computes the
// log-sum-exp and the CE term; block partials are summed in a fixed order.
// Backward: each block owns a 4 x 64 tile of label pixels, accumulates
// (softmax - onehot) * tap weight into an LDS copy of the low-res patch the tile touches, then
// flushes the patch with global float atomics (<= 4 blocks add into any low-res cell).
#include "common.h"

namespace {
constexpr int TY = 4, TX = 64;
constexpr int MAXC = 64;
constexpr int PATCH = 8192;

DFM_INLINE void src_idx(int dst, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = scale * (dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

template <typename T>
DFM_INLINE void interp(const T* lg, int b, int h, int w, int ncls, int y, int x, int H, int W, float* z, int& h0,
                       int& h1, int& w0, int& w1, float& lh, float& lw) {
  src_idx(y, h, H, h0, h1, lh);
  src_idx(x, w, W, w0, w1, lw);
  const T* p00 = lg + (((long)b * h + h0) * w + w0) * ncls;
  const T* p01 = lg + (((long)b * h + h0) * w + w1) * ncls;
  const T* p10 = lg + (((long)b * h + h1) * w + w0) * ncls;
  const T* p11 = lg + (((long)b * h + h1) * w + w1) * ncls;
  for (int c = 0; c < ncls; ++c)
    z[c] = (1.f - lh) * ((1.f - lw) * ldf(p00 + c) + lw * ldf(p01 + c)) + lh * ((1.f - lw) * ldf(p10 + c) + lw * ldf(p11 + c));
}

template <typename T>
__global__ __launch_bounds__(256) void seg_loss_fwd_kernel(int B, int h, int w, int ncls, const T* __restrict__ lg,
                                                           int H, int W, const long* __restrict__ label, int ignore,
                                                           float* __restrict__ lse_out, float* __restrict__ part) {
  const long n = (long)B * H * W;
  float s = 0.f, cnt = 0.f;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    const int x = p % W, y = (p / W) % H, b = p / ((long)W * H);
    const long lab = label[p];
    float z[MAXC];
    int h0, h1, w0, w1;
    float lh, lw;
    interp(lg, b, h, w, ncls, y, x, H, W, z, h0, h1, w0, w1, lh, lw);
    float m = -INFINITY;
    for (int c = 0; c < ncls; ++c) m = fmaxf(m, z[c]);
    float se = 0.f;
    for (int c = 0; c < ncls; ++c) se += __expf(z[c] - m);
    const float lse = m + __logf(se);
    if (lse_out) lse_out[p] = lse;
    if (lab != ignore && lab >= 0 && lab < ncls) {
      s += lse - z[lab];
      cnt += 1.f;
    }
  }
  s = wave_sum(s);
  cnt = wave_sum(cnt);
  __shared__ float red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[blockIdx.x * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void seg_loss_sum_kernel(int nblk, const float* __restrict__ part, float* __restrict__ out) {
  if (threadIdx.x < 2) {
    float s = 0.f;
    for (int b = 0; b < nblk; ++b) s += part[b * 2 + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

__global__ void zero_kernel(long n, float* __restrict__ p) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = 0.f;
}

template <typename T>
__global__ __launch_bounds__(256) void seg_loss_bwd_kernel(int B, int h, int w, int ncls, const T* __restrict__ lg,
                                                           int H, int W, const long* __restrict__ label, int ignore,
                                                           const float* __restrict__ loss_out, const float* __restrict__ gscale,
                                                           float* __restrict__ dlg) {
  __shared__ float patch[PATCH];
  const int tiles_x = (W + TX - 1) / TX, tiles_y = (H + TY - 1) / TY;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int y0 = ty * TY, x0 = tx * TX;
  const int y1 = min(H, y0 + TY) - 1, x1 = min(W, x0 + TX) - 1;
  int a0, a1, c0, c1;
  float t;
  src_idx(y0, h, H, a0, c0, t);
  src_idx(y1, h, H, c0, a1, t);
  int b0, b1, d0, d1;
  src_idx(x0, w, W, b0, d0, t);
  src_idx(x1, w, W, d0, b1, t);
  const int pr = a1 - a0 + 1, pc = b1 - b0 + 1;
  const bool use_lds = pr * pc * ncls <= PATCH;
  if (use_lds) {
    for (int e = threadIdx.x; e < pr * pc * ncls; e += 256) patch[e] = 0.f;
    __syncthreads();
  }
  const float inv = (gscale ? gscale[0] : 1.f) / fmaxf(loss_out[1], 1.f);
  const int y = y0 + threadIdx.x / TX, x = x0 + threadIdx.x % TX;
  if (y < H && x < W) {
    const long p = ((long)b * H + y) * W + x;
    const long lab = label[p];
    if (lab != ignore && lab >= 0 && lab < ncls) {
      float z[MAXC];
      int h0, h1, w0, w1;
      float lh, lw;
      interp(lg, b, h, w, ncls, y, x, H, W, z, h0, h1, w0, w1, lh, lw);
      float m = -INFINITY;
      for (int c = 0; c < ncls; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
      for (int c = 0; c < ncls; ++c) {
        z[c] = __expf(z[c] - m);
        se += z[c];
      }
      const float rs = 1.f / se;
      const float wt[4] = {(1.f - lh) * (1.f - lw), (1.f - lh) * lw, lh * (1.f - lw), lh * lw};
      const int hh[4] = {h0, h0, h1, h1}, ww[4] = {w0, w1, w0, w1};
      for (int c = 0; c < ncls; ++c) {
        const float g = (z[c] * rs - (c == lab ? 1.f : 0.f)) * inv;
        for (int k = 0; k < 4; ++k) {
          if (wt[k] == 0.f) continue;
          if (use_lds) atomicAdd(&patch[((hh[k] - a0) * pc + (ww[k] - b0)) * ncls + c], g * wt[k]);
          else atomicAdd(&dlg[(((long)b * h + hh[k]) * w + ww[k]) * ncls + c], g * wt[k]);
        }
      }
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int e = threadIdx.x; e < pr * pc * ncls; e += 256) {
      const float v = patch[e];
      if (v != 0.f) {
        const int c = e % ncls, cell = e / ncls;
        const int i = a0 + cell / pc, j = b0 + cell % pc;
        atomicAdd(&dlg[(((long)b * h + i) * w + j) * ncls + c], v);
      }
    }
  }
}

constexpr int LOSS_BLOCKS = 1024;
}  // namespace

extern "C" size_t dfm_seg_loss_workspace(int, int, int) { return LOSS_BLOCKS * 2 * sizeof(float); }

extern "C" int dfm_seg_loss_fwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, float* lse, float* loss_out, void* workspace,
                                dfm_stream_t stream) {
  DFM_CHECK_ARG(logits && label && loss_out && workspace && ncls <= MAXC, "dfm_seg_loss_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)B * H * W;
  const int nblk = (int)min((long)LOSS_BLOCKS, (n + 255) / 256);
  if (dtype == DFM_BF16)
    hipLaunchKernelGGL(seg_loss_fwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const bf16_t*)logits, H,
                       W, label, ignore, lse, (float*)workspace);
  else
    hipLaunchKernelGGL(seg_loss_fwd_kernel<float>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const float*)logits, H,
                       W, label, ignore, lse, (float*)workspace);
  DFM_LAUNCH_CHECK();
  hipLaunchKernelGGL(seg_loss_sum_kernel, dim3(1), dim3(64), 0, s, nblk, (const float*)workspace, loss_out);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_seg_loss_bwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, const float* lse, const float* loss_out, const float* gscale,
                                float* dlogits, dfm_stream_t stream) {
  (void)lse;
  DFM_CHECK_ARG(logits && label && loss_out && dlogits && ncls <= MAXC, "dfm_seg_loss_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const long nl = (long)B * h * w * ncls;
  hipLaunchKernelGGL(zero_kernel, dim3(min(4096L, (nl + 255) / 256)), dim3(256), 0, s, nl, dlogits);
  DFM_LAUNCH_CHECK();
  const unsigned nblk = B * ((H + TY - 1) / TY) * ((W + TX - 1) / TX);
  if (dtype == DFM_BF16)
    hipLaunchKernelGGL(seg_loss_bwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const bf16_t*)logits, H,
                       W, label, ignore, loss_out, gscale, dlogits);
  else
    hipLaunchKernelGGL(seg_loss_bwd_kernel<float>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const float*)logits, H,
                       W, label, ignore, loss_out, gscale, dlogits);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
