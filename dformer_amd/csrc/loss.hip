// Segmentation loss of EncoderDecoder.forward (builder.py:203,230): bilinear upsampling of the
// low-resolution logits to the label size + cross-entropy(ignore_index) + mean over valid pixels.
// Fused: the full-resolution logits (786 MB fp32 for DFormer-B bs16) are never materialised.
// Forward: one thread per label pixel interpolates its ncls logits from the 4 taps (registers,
//   compile-time unrolled over MAXC classes), computes log-sum-exp and the CE term; block partials
//   are summed in a fixed order.
// Backward: a block owns a TY x TX tile of label pixels. Phase 1: every thread writes its pixel's
//   (softmax - onehot) / count row into LDS. Phase 2 (separable): each pixel row is reduced onto the
//   patch's low-res columns (<= 2 taps per pixel), then the pixel rows onto its low-res rows.
//   Phase 3: one global float atomic per (cell, class) per block (a cell is shared by <= ~10 blocks).
#include <algorithm>

#include "common.h"

namespace {
constexpr int TY = 4, TX = 64;
constexpr int MAXC = 64;

DFM_INLINE void src_idx(int dst, int in, int out, int& i0, int& i1, float& l1) {
  const float scale = (float)in / (float)out;
  float src = scale * (dst + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

// z[c] for c < ncls (others -inf); returns the logit of class `lab` through a predicated select
template <typename T>
DFM_INLINE void interp(const T* lg, int b, int h, int w, int ncls, int y, int x, int H, int W, float (&z)[MAXC],
                       bool vec) {
  int h0, h1, w0, w1;
  float lh, lw;
  src_idx(y, h, H, h0, h1, lh);
  src_idx(x, w, W, w0, w1, lw);
  const T* p00 = lg + (((long)b * h + h0) * w + w0) * ncls;
  const T* p01 = lg + (((long)b * h + h0) * w + w1) * ncls;
  const T* p10 = lg + (((long)b * h + h1) * w + w0) * ncls;
  const T* p11 = lg + (((long)b * h + h1) * w + w1) * ncls;
  const float a00 = (1.f - lh) * (1.f - lw), a01 = (1.f - lh) * lw, a10 = lh * (1.f - lw), a11 = lh * lw;
  if constexpr (sizeof(T) == 2) {
    if (vec) {  // 16-byte rows of 8 classes: 4 vector loads per 8 classes instead of 32 scalar ones
#pragma unroll
      for (int v = 0; v < MAXC / 8; ++v) {
        if (v * 8 < ncls) {
          float f00[8], f01[8], f10[8], f11[8];
          ld8<T>(p00 + v * 8, f00);
          ld8<T>(p01 + v * 8, f01);
          ld8<T>(p10 + v * 8, f10);
          ld8<T>(p11 + v * 8, f11);
#pragma unroll
          for (int e = 0; e < 8; ++e) z[v * 8 + e] = a00 * f00[e] + a01 * f01[e] + a10 * f10[e] + a11 * f11[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) z[v * 8 + e] = -INFINITY;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    z[c] = c < ncls ? a00 * ldf(p00 + c) + a01 * ldf(p01 + c) + a10 * ldf(p10 + c) + a11 * ldf(p11 + c) : -INFINITY;
}

template <typename T>
__global__ __launch_bounds__(256) void seg_loss_fwd_kernel(int B, int h, int w, int ncls, const T* __restrict__ lg,
                                                           int H, int W, const long* __restrict__ label, int ignore,
                                                           float* __restrict__ lse_out, float* __restrict__ part) {
  const long n = (long)B * H * W;
  const bool vec = ncls % 8 == 0 && ((uintptr_t)lg & 15) == 0;
  float s = 0.f, cnt = 0.f;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    const int x = p % W, y = (p / W) % H, b = p / ((long)W * H);
    const long lab = label[p];
    float z[MAXC];
    interp(lg, b, h, w, ncls, y, x, H, W, z, vec);
    float m = -INFINITY, zl = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      m = fmaxf(m, z[c]);
      zl = (c == lab) ? z[c] : zl;
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) se += c < ncls ? __expf(z[c] - m) : 0.f;
    const float lse = m + __logf(se);
    if (lse_out) lse_out[p] = lse;
    if (lab != ignore && lab >= 0 && lab < ncls) {
      s += lse - zl;
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

// one wave: lane l sums partials l, l+64, ... (both outputs), then a fixed-order wave reduction
// (a single-thread serial sum over the 1024 partials cost ~80 us of dependent loads)
__global__ void seg_loss_sum_kernel(int nblk, const float* __restrict__ part, float* __restrict__ out) {
  float s0 = 0.f, s1 = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 64) {
    s0 += part[b * 2];
    s1 += part[b * 2 + 1];
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (threadIdx.x == 0) {
    out[0] = s0;
    out[1] = s1;
  }
}

__global__ void zero_kernel(long n, float* __restrict__ p) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = 0.f;
}


template <typename T>
__global__ __launch_bounds__(256) void seg_loss_bwd_kernel(int B, int h, int w, int ncls, const T* __restrict__ lg,
                                                           int H, int W, const long* __restrict__ label, int ignore,
                                                           const float* __restrict__ loss_out,
                                                           const float* __restrict__ gscale, float* __restrict__ dlg,
                                                           int pcmax) {
  extern __shared__ __attribute__((aligned(16))) float gt[];  // [TY*TX][ncls+1], then rx
  const int GLD = ncls + 1;
  const int tiles_x = (W + TX - 1) / TX, tiles_y = (H + TY - 1) / TY;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x; bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int y0 = ty * TY, x0 = tx * TX;
  const int ny = min(TY, H - y0), nx = min(TX, W - x0);
  const float inv = (gscale ? gscale[0] : 1.f) / fmaxf(loss_out[1], 1.f);
  const bool vec = ncls % 8 == 0 && ((uintptr_t)lg & 15) == 0;
  // phase 1: per-pixel d loss / d upsampled logits
  {
    const int py = threadIdx.x / TX, px = threadIdx.x % TX;
    float* row = gt + threadIdx.x * GLD;
    const int y = y0 + py, x = x0 + px;
    long lab = -1;
    if (py < ny && px < nx) lab = label[((long)b * H + y) * W + x];
    const bool valid = lab != ignore && lab >= 0 && lab < ncls;
    if (valid) {
      float z[MAXC];
      interp(lg, b, h, w, ncls, y, x, H, W, z, vec);
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        z[c] = c < ncls ? __expf(z[c] - m) : 0.f;
        se += z[c];
      }
      const float rs = inv / se;
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (c < ncls) row[c] = z[c] * rs - (c == lab ? inv : 0.f);
    } else {
      for (int c = 0; c < ncls; ++c) row[c] = 0.f;
    }
  }
  __syncthreads();
  // phase 2 (separable): (a) x-reduction of each pixel row onto the patch's low-res columns,
  // (b) y-reduction onto its low-res rows; every pixel has <= 2 taps per axis.
  int a0, a1, b0, b1, t0;
  float tl;
  src_idx(y0, h, H, a0, t0, tl);
  src_idx(y0 + ny - 1, h, H, t0, a1, tl);
  src_idx(x0, w, W, b0, t0, tl);
  src_idx(x0 + nx - 1, w, W, t0, b1, tl);
  const int pr = a1 - a0 + 1, pc = b1 - b0 + 1;
  float* rx = gt + TY * TX * GLD;                      // [TY][pcmax][GLD]
  __shared__ int xj0[TX], xj1[TX], yi0[TY], yi1[TY];   // taps relative to b0 / a0
  __shared__ float xw0[TX], xw1[TX], yw0[TY], yw1[TY];
  __shared__ int jlo[TX + 2], jhi[TX + 2];
  if (threadIdx.x < nx) {
    int i0, i1;
    float l1;
    src_idx(x0 + threadIdx.x, w, W, i0, i1, l1);
    xj0[threadIdx.x] = i0 - b0; xj1[threadIdx.x] = i1 - b0;
    xw0[threadIdx.x] = 1.f - l1; xw1[threadIdx.x] = l1;
  }
  if (threadIdx.x >= 64 && threadIdx.x < 64 + ny) {
    const int py = threadIdx.x - 64;
    int i0, i1;
    float l1;
    src_idx(y0 + py, h, H, i0, i1, l1);
    yi0[py] = i0 - a0; yi1[py] = i1 - a0;
    yw0[py] = 1.f - l1; yw1[py] = l1;
  }
  __syncthreads();
  if (threadIdx.x < pc) {  // pixel-column range touching low-res column jj (taps are monotone in px)
    const int jj = threadIdx.x;
    int lo = nx, hi = -1;
    for (int px = 0; px < nx; ++px)
      if (xj0[px] == jj || xj1[px] == jj) {
        lo = min(lo, px);
        hi = px;
      }
    jlo[jj] = lo;
    jhi[jj] = hi;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < ny * pc * ncls; e += 256) {
    const int c = e % ncls, t = e / ncls, jj = t % pc, py = t / pc;
    float r = 0.f;
    const float* grow = gt + (py * TX) * GLD + c;
    for (int px = jlo[jj]; px <= jhi[jj]; ++px) {
      const float wx = (xj0[px] == jj ? xw0[px] : 0.f) + (xj1[px] == jj ? xw1[px] : 0.f);
      r = fmaf(wx, grow[px * GLD], r);
    }
    rx[(py * pcmax + jj) * GLD + c] = r;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < pr * pc * ncls; e += 256) {
    const int c = e % ncls, t = e / ncls, jj = t % pc, ii = t / pc;
    float acc = 0.f;
    for (int py = 0; py < ny; ++py) {
      const float wy = (yi0[py] == ii ? yw0[py] : 0.f) + (yi1[py] == ii ? yw1[py] : 0.f);
      acc = fmaf(wy, rx[(py * pcmax + jj) * GLD + c], acc);
    }
    if (acc != 0.f) atomicAdd(&dlg[(((long)b * h + a0 + ii) * w + b0 + jj) * ncls + c], acc);
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
    DFM_LAUNCH(seg_loss_fwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const bf16_t*)logits, H,
                       W, label, ignore, lse, (float*)workspace);
  else
    DFM_LAUNCH(seg_loss_fwd_kernel<float>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const float*)logits, H,
                       W, label, ignore, lse, (float*)workspace);
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(seg_loss_sum_kernel, dim3(1), dim3(64), 0, s, nblk, (const float*)workspace, loss_out);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_seg_loss_bwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, const float* lse, const float* loss_out,
                                const float* gscale, float* dlogits, dfm_stream_t stream) {
  (void)lse;
  DFM_CHECK_ARG(logits && label && loss_out && dlogits && ncls <= MAXC && h <= H && w <= W,
                "dfm_seg_loss_bwd: bad argument (needs ncls <= 64 and an upsampling resize)");
  hipStream_t s = (hipStream_t)stream;
  const long nl = (long)B * h * w * ncls;
  DFM_LAUNCH(zero_kernel, dim3(min(4096L, (nl + 255) / 256)), dim3(256), 0, s, nl, dlogits);
  DFM_LAUNCH_CHECK();
  const unsigned nblk = B * ((H + TY - 1) / TY) * ((W + TX - 1) / TX);
  // low-res columns one TX-wide pixel tile can touch (+2 for the taps at both ends)
  const int pcmax = std::min(TX + 2, (int)(((long)TX * w + W - 1) / W) + 3);
  const size_t lds = ((size_t)TY * TX + (size_t)TY * pcmax) * (ncls + 1) * sizeof(float);
  if (lds > 64 * 1024) {  // only small upsampling ratios need more than the default
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    (void)hipGetLastError();  // a refused attribute must not read as this launch's error
  }
  if (dtype == DFM_BF16)
    DFM_LAUNCH(seg_loss_bwd_kernel<bf16_t>, dim3(nblk), dim3(256), lds, s, B, h, w, ncls, (const bf16_t*)logits,
                       H, W, label, ignore, loss_out, gscale, dlogits, pcmax);
  else
    DFM_LAUNCH(seg_loss_bwd_kernel<float>, dim3(nblk), dim3(256), lds, s, B, h, w, ncls, (const float*)logits,
                       H, W, label, ignore, loss_out, gscale, dlogits, pcmax);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
