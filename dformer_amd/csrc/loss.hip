// Segmentation loss of EncoderDecoder.forward (builder.py:203,230): bilinear upsampling of the
// low-resolution logits to the label size + cross-entropy(ignore_index) + mean over valid pixels.
// Fused: the full-resolution logits (786 MB fp32 for DFormer-B bs16) are never materialised.
//
// Forward: one thread per label pixel interpolates its ncls logits from the 4 taps (registers),
//   computes log-sum-exp and the CE term; block partials are summed in a fixed order.
// Backward, integer upsampling factor (the DFormer heads: x8 ham, x4 MLP decoder at 480x640):
//   seg_loss_bwd_tile_kernel + seg_loss_gather_kernel (below): deterministic, no atomics.
// Backward, other factors: seg_loss_bwd_kernel — per tile of label pixels a separable reduction
//   in LDS, then one float atomic per (cell, class) per block into a zeroed gradient.
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

// ---- backward for an integer upsampling factor S (H = S h, W = S w, S even, S*S <= 64): the label
// pixels y in [S ty - S/2, S ty + S/2) all take their y-taps from low-res rows {ty - 1, ty} (edges
// clamp), likewise for x, so each S x S pixel tile ("corner tile" (ty, tx), ty in [0, h]) feeds
// exactly the 2 x 2 low-res cells around its corner. One wave owns 64 / S^2 tiles: every lane
// forms its pixel's scaled (softmax - onehot) row in LDS, then each lane of a (tile, class) pair sums
// the tile's pixels into the 4 corner partials (fixed order). seg_loss_gather_kernel adds, for every
// low-res cell, the 4 corner partials that touch it in a fixed order: deterministic, no atomics.
constexpr int TILE_NT = 128;  // 2 waves; res[] stays under 64 KB of static LDS at MAXC

template <typename T, int S>
__global__ __launch_bounds__(TILE_NT) void seg_loss_bwd_tile_kernel(int B, int h, int w, int ncls,
                                                                    const T* __restrict__ lg, int H, int W,
                                                                    const long* __restrict__ label, int ignore,
                                                                    const float* __restrict__ loss_out,
                                                                    const float* __restrict__ gscale,
                                                                    float* __restrict__ part, long ntiles) {
  constexpr int TP = S * S, TPW = 64 / TP;   // pixels per tile, tiles per wave
  constexpr int RP = MAXC + 1;               // LDS row pitch of a pixel's residual
  __shared__ float res[TILE_NT][RP];
  __shared__ float wts[TILE_NT][4];          // per pixel: weights of corner slots (y0 x0, y0 x1, y1 x0, y1 x1)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long tile = ((long)blockIdx.x * (TILE_NT / 64) + wid) * TPW + lane / TP;
  const int d = lane % TP, dy = d / S, dx = d % S;
  const int tw = w + 1, th = h + 1;
  const float inv = (gscale ? gscale[0] : 1.f) / fmaxf(loss_out[1], 1.f);
  const bool vec = ncls % 8 == 0 && ((uintptr_t)lg & 15) == 0;
  float* row = res[threadIdx.x];
  float wv[4] = {0.f, 0.f, 0.f, 0.f};
  if (tile < ntiles) {
    const int tx = tile % tw, ty = (tile / tw) % th, b = tile / ((long)tw * th);
    const int y = S * ty - S / 2 + dy, x = S * tx - S / 2 + dx;
    long lab = -1;
    if (y >= 0 && y < H && x >= 0 && x < W) lab = label[((long)b * H + y) * W + x];
    if (lab != ignore && lab >= 0 && lab < ncls) {
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
      int a0, a1, b0, b1;
      float ly, lx;
      src_idx(y, h, H, a0, a1, ly);
      src_idx(x, w, W, b0, b1, lx);
      // taps -> the tile's corner slots (row ty - 1 -> 0, ty -> 1; clamped duplicates merge)
      const float wy[2] = {(a0 == ty - 1 ? 1.f - ly : 0.f) + (a1 == ty - 1 ? ly : 0.f),
                           (a0 == ty ? 1.f - ly : 0.f) + (a1 == ty ? ly : 0.f)};
      const float wx[2] = {(b0 == tx - 1 ? 1.f - lx : 0.f) + (b1 == tx - 1 ? lx : 0.f),
                           (b0 == tx ? 1.f - lx : 0.f) + (b1 == tx ? lx : 0.f)};
      wv[0] = wy[0] * wx[0]; wv[1] = wy[0] * wx[1]; wv[2] = wy[1] * wx[0]; wv[3] = wy[1] * wx[1];
    } else {
      for (int c = 0; c < ncls; ++c) row[c] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) wts[threadIdx.x][k] = wv[k];
  __syncthreads();
  // (tile of this wave, class) pairs: sum the tile's pixels into the 4 corner partials
  for (int pr = lane; pr < TPW * ncls; pr += 64) {
    const int tt = pr / ncls, c = pr % ncls;
    const long t = ((long)blockIdx.x * (TILE_NT / 64) + wid) * TPW + tt;
    if (t >= ntiles) continue;
    const int base = wid * 64 + tt * TP;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 8
    for (int q = 0; q < TP; ++q) {
      const float r = res[base + q][c];
      s0 = fmaf(wts[base + q][0], r, s0);
      s1 = fmaf(wts[base + q][1], r, s1);
      s2 = fmaf(wts[base + q][2], r, s2);
      s3 = fmaf(wts[base + q][3], r, s3);
    }
    float* o = part + t * 4 * ncls + c;
    o[0] = s0;
    o[ncls] = s1;
    o[2 * ncls] = s2;
    o[3 * ncls] = s3;
  }
}

// dlogits[b][i][j][c] = sum of the corner partials of the 4 tiles around cell (i, j), fixed order
__global__ void seg_loss_gather_kernel(int B, int h, int w, int ncls, const float* __restrict__ part,
                                       float* __restrict__ dlg) {
  const long n = (long)B * h * w * ncls;
  const int tw = w + 1, th = h + 1;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % ncls;
    const long cell = e / ncls;
    const int j = cell % w, i = (cell / w) % h, b = cell / ((long)w * h);
    auto P = [&](int ty, int tx, int slot) { return part[((((long)b * th + ty) * tw + tx) * 4 + slot) * ncls + c]; };
    // cell (i, j) is slot (row 1, col 1) of tile (i, j), (1, 0) of (i, j + 1), (0, 1) of (i + 1, j),
    // (0, 0) of (i + 1, j + 1)
    dlg[e] = P(i, j, 3) + P(i, j + 1, 2) + P(i + 1, j, 1) + P(i + 1, j + 1, 0);
  }
}

template <typename T>
int launch_bwd_tiles(int S, int B, int h, int w, int ncls, const void* lg, int H, int W, const long* label,
                     int ignore, const float* loss_out, const float* gscale, float* part, float* dlg,
                     hipStream_t s) {
  const long ntiles = (long)B * (h + 1) * (w + 1);
  const long tiles_per_block = (TILE_NT / 64) * (64 / (S * S));
  const unsigned nb = cdiv(ntiles, tiles_per_block);
  if (S == 8)
    DFM_LAUNCH((seg_loss_bwd_tile_kernel<T, 8>), dim3(nb), dim3(TILE_NT), 0, s, B, h, w, ncls, (const T*)lg, H, W,
               label, ignore, loss_out, gscale, part, ntiles);
  else if (S == 4)
    DFM_LAUNCH((seg_loss_bwd_tile_kernel<T, 4>), dim3(nb), dim3(TILE_NT), 0, s, B, h, w, ncls, (const T*)lg, H, W,
               label, ignore, loss_out, gscale, part, ntiles);
  else
    DFM_LAUNCH((seg_loss_bwd_tile_kernel<T, 2>), dim3(nb), dim3(TILE_NT), 0, s, B, h, w, ncls, (const T*)lg, H, W,
               label, ignore, loss_out, gscale, part, ntiles);
  DFM_LAUNCH_CHECK();
  const long n = (long)B * h * w * ncls;
  DFM_LAUNCH(seg_loss_gather_kernel, dim3(min(8192L, (n + 255) / 256)), dim3(256), 0, s, B, h, w, ncls,
             (const float*)part, dlg);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

int tile_scale(int h, int w, int H, int W) {
  for (int S : {8, 4, 2})
    if (H == S * h && W == S * w) return S;
  return 0;
}

constexpr int LOSS_BLOCKS = 1024;
}  // namespace

extern "C" size_t dfm_seg_loss_workspace(int B, int H, int W) {
  (void)B; (void)H; (void)W;
  return (size_t)LOSS_BLOCKS * 2 * sizeof(float);
}

/* backward workspace of the integer-scale tile path: corner partials of every tile (0 otherwise) */
extern "C" size_t dfm_seg_loss_bwd_workspace(int B, int h, int w, int ncls, int H, int W) {
  if (!tile_scale(h, w, H, W)) return 0;
  return (size_t)B * (h + 1) * (w + 1) * 4 * ncls * sizeof(float);
}

extern "C" int dfm_seg_loss_fwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, float* lse, float* loss_out, void* workspace,
                                dfm_stream_t stream) {
  DFM_CHECK_ARG(logits && label && loss_out && workspace && ncls <= MAXC, "dfm_seg_loss_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)B * H * W;
  const int nblk = (int)min((long)LOSS_BLOCKS, (n + 255) / 256);
  if (dtype == DFM_BF16)
    DFM_LAUNCH(seg_loss_fwd_kernel<bf16_t>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const bf16_t*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  else if (dtype == DFM_F16)
    DFM_LAUNCH(seg_loss_fwd_kernel<f16_t>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const f16_t*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  else
    DFM_LAUNCH(seg_loss_fwd_kernel<float>, dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const float*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(seg_loss_sum_kernel, dim3(1), dim3(64), 0, s, nblk, (const float*)workspace, loss_out);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_seg_loss_bwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, const float* lse, const float* loss_out,
                                const float* gscale, float* dlogits, void* workspace, dfm_stream_t stream) {
  (void)lse;
  DFM_CHECK_ARG(logits && label && loss_out && dlogits && ncls <= MAXC && h <= H && w <= W,
                "dfm_seg_loss_bwd: bad argument (needs ncls <= 64 and an upsampling resize)");
  hipStream_t s = (hipStream_t)stream;
  const long nl = (long)B * h * w * ncls;
  if (workspace && tile_scale(h, w, H, W)) {
    const int S = tile_scale(h, w, H, W);
    if (dtype == DFM_BF16)
      return launch_bwd_tiles<bf16_t>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, gscale,
                                      (float*)workspace, dlogits, s);
    else if (dtype == DFM_F16)
      return launch_bwd_tiles<f16_t>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, gscale,
                                      (float*)workspace, dlogits, s);
    return launch_bwd_tiles<float>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, gscale,
                                   (float*)workspace, dlogits, s);
  }
  // other scales: the general tile kernel (float atomics into a zeroed gradient)
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
  else if (dtype == DFM_F16)
    DFM_LAUNCH(seg_loss_bwd_kernel<f16_t>, dim3(nblk), dim3(256), lds, s, B, h, w, ncls, (const f16_t*)logits,
                       H, W, label, ignore, loss_out, gscale, dlogits, pcmax);
  else
    DFM_LAUNCH(seg_loss_bwd_kernel<float>, dim3(nblk), dim3(256), lds, s, B, h, w, ncls, (const float*)logits,
                       H, W, label, ignore, loss_out, gscale, dlogits, pcmax);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
