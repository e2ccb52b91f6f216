// Segmentation loss of EncoderDecoder.forward (builder.py:203,230): bilinear upsampling of the
// low-resolution logits to the label size + cross-entropy(ignore_index) + mean over valid pixels.
// Fused: the full-resolution logits (786 MB fp32 for DFormer-B bs16) are never materialised.
//
// Forward: one thread per label pixel interpolates its ncls logits from the 4 taps (registers),
//   computes log-sum-exp and the CE term; block partials are summed in a fixed order.
// Backward, integer upsampling factor (the DFormer heads: x8 ham, x4 MLP decoder at 480x640):
//   seg_loss_bwd_tile_kernel + seg_loss_gather_kernel (below): deterministic, no atomics.
// Backward, other factors (config 5's 133x183 -> 530x730): seg_loss_bwd_xpass_kernel +
//   seg_loss_bwd_ypass_kernel, a separable fixed-order contraction: deterministic, no atomics.
#include <algorithm>

#include "common.h"

namespace {
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
template <typename T, int NC>
DFM_INLINE void interp(const T* lg, int b, int h, int w, int ncls, int y, int x, int H, int W, float (&z)[NC],
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
      for (int v = 0; v < NC / 8; ++v) {
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
  for (int c = 0; c < NC; ++c)
    z[c] = c < ncls ? a00 * ldf(p00 + c) + a01 * ldf(p01 + c) + a10 * ldf(p10 + c) + a11 * ldf(p11 + c) : -INFINITY;
}

template <typename T, int NC>
__global__ __launch_bounds__(256) void seg_loss_fwd_kernel(int B, int h, int w, int ncls, const T* __restrict__ lg,
                                                           int H, int W, const long* __restrict__ label, int ignore,
                                                           float* __restrict__ lse_out, float* __restrict__ part) {
  const long n = (long)B * H * W;
  const bool vec = ncls % 8 == 0 && ((uintptr_t)lg & 15) == 0;
  float s = 0.f, cnt = 0.f;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    const int x = p % W, y = (p / W) % H, b = p / ((long)W * H);
    const long lab = label[p];
    float z[NC];
    interp(lg, b, h, w, ncls, y, x, H, W, z, vec);
    float m = -INFINITY, zl = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      m = fmaxf(m, z[c]);
      zl = (c == lab) ? z[c] : zl;
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) se += c < ncls ? __expf(z[c] - m) : 0.f;
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


// ---- backward, any upsampling factor (h <= H, w <= W): separable and deterministic, no atomics.
// x-pass: a block owns PJ low-res columns of RY label rows; its threads form the scaled
//   (softmax - onehot) residual of every pixel whose x-taps touch those columns (a span of PX
//   pixels: the owned columns plus one low-res column either side, recomputed by the neighbouring
//   block) into LDS, then each (row, column, class) sums its pixels in ascending x:
//   rx[b][y][j][c] = sum_x wx(x, j) d(b, y, x, c).
// y-pass: dlogits[b][i][j][c] = sum_y wy(y, i) rx[b][y][j][c], ascending y. Every output element is
// a fixed-order sum, so the gradient is bitwise reproducible (the integer-factor path below is the
// faster special case of the same contraction).
constexpr int XP_NT = 256;

// first pixel index whose source coordinate can reach low-res index j (a conservative lower bound
// under the src_idx rounding; callers then test each pixel's taps exactly)
DFM_INLINE int first_pixel(int j, int in, int out) {
  const float inv = (float)out / (float)in;
  return max(0, (int)floorf(((float)j + 0.5f) * inv - 0.5f) - 2);
}

template <typename T, int NC>
__global__ __launch_bounds__(XP_NT) void seg_loss_bwd_xpass_kernel(int B, int h, int w, int ncls,
                                                                    const T* __restrict__ lg, int H, int W,
                                                                    const long* __restrict__ label, int ignore,
                                                                    const float* __restrict__ loss_out,
                                                                    const float* __restrict__ gscale,
                                                                    float* __restrict__ rx, int RY, int PJ) {
  extern __shared__ __attribute__((aligned(16))) float res[];  // [XP_NT][ncls + 1]
  const int GLD = ncls + 1, PX = XP_NT / RY;
  const int nj = (w + PJ - 1) / PJ, ny = (H + RY - 1) / RY;
  int bid = blockIdx.x;
  const int jc = bid % nj; bid /= nj;
  const int yc = bid % ny;
  const int b = bid / ny;
  const int j0 = jc * PJ, j1 = min(w, j0 + PJ);  // owned columns [j0, j1)
  const int xa = first_pixel(j0 - 1, w, W);      // pixels whose taps reach j0 start at src >= j0 - 1
  const float inv = (gscale ? gscale[0] : 1.f) / fmaxf(loss_out[1], 1.f);
  const bool vec = ncls % 8 == 0 && ((uintptr_t)lg & 15) == 0;
  __shared__ int tj0[XP_NT], tj1[XP_NT];
  __shared__ float tw0[XP_NT], tw1[XP_NT];
  __shared__ int jlo[XP_NT], jhi[XP_NT];
  {
    const int py = threadIdx.x / PX, px = threadIdx.x % PX;
    const int y = yc * RY + py, x = xa + px;
    float* row = res + threadIdx.x * GLD;
    int i0 = -1, i1 = -1;
    float l1 = 0.f;
    bool touch = false;
    if (y < H && x < W) {
      src_idx(x, w, W, i0, i1, l1);
      touch = (i0 >= j0 && i0 < j1) || (i1 >= j0 && i1 < j1);
    }
    tj0[threadIdx.x] = i0; tj1[threadIdx.x] = i1;
    tw0[threadIdx.x] = 1.f - l1; tw1[threadIdx.x] = l1;
    long lab = -1;
    if (touch) lab = label[((long)b * H + y) * W + x];
    if (lab != ignore && lab >= 0 && lab < ncls) {
      float z[NC];
      interp(lg, b, h, w, ncls, y, x, H, W, z, vec);
      float m = -INFINITY;
#pragma unroll
      for (int c = 0; c < NC; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        z[c] = c < ncls ? __expf(z[c] - m) : 0.f;
        se += z[c];
      }
      const float rs = inv / se;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < ncls) row[c] = z[c] * rs - (c == lab ? inv : 0.f);
    } else {
      for (int c = 0; c < ncls; ++c) row[c] = 0.f;
    }
  }
  __syncthreads();
  if (threadIdx.x < j1 - j0) {  // pixel range of owned column j (taps are monotone in x)
    const int j = j0 + threadIdx.x;
    int lo = PX, hi = -1;
    for (int px = 0; px < PX; ++px)
      if (tj0[px] == j || tj1[px] == j) {
        lo = min(lo, px);
        hi = px;
      }
    jlo[threadIdx.x] = lo;
    jhi[threadIdx.x] = hi;
  }
  __syncthreads();
  const int pj = j1 - j0;
  for (int e = threadIdx.x; e < RY * pj * ncls; e += XP_NT) {
    const int c = e % ncls, t = e / ncls, jj = t % pj, py = t / pj;
    const int y = yc * RY + py;
    if (y >= H) continue;
    const int j = j0 + jj;
    float r = 0.f;
    for (int px = jlo[jj]; px <= jhi[jj]; ++px) {
      const int q = py * PX + px;
      const float wx = (tj0[q] == j ? tw0[q] : 0.f) + (tj1[q] == j ? tw1[q] : 0.f);
      r = fmaf(wx, res[q * GLD + c], r);
    }
    rx[(((long)b * H + y) * w + j) * ncls + c] = r;
  }
}

__global__ void seg_loss_bwd_ypass_kernel(int B, int h, int w, int ncls, int H, const float* __restrict__ rx,
                                          float* __restrict__ dlg) {
  const long n = (long)B * h * w * ncls;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long jc = e % ((long)w * ncls);  // (j, c)
    const long bi = e / ((long)w * ncls);
    const int i = bi % h, b = bi / h;
    float acc = 0.f;
    for (int y = first_pixel(i - 1, h, H); y < H; ++y) {
      int i0, i1;
      float l1;
      src_idx(y, h, H, i0, i1, l1);
      if (i0 > i) break;  // taps are monotone in y
      const float wy = (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
      if (i0 == i || i1 == i) acc = fmaf(wy, rx[((long)b * H + y) * w * ncls + jc], acc);
    }
    dlg[e] = acc;
  }
}

// (rows per x-pass block, owned columns per block) for a W / w ratio: the touched pixel span of PJ
// columns, (PJ + 1) W / w + 6 pixels (rounding margins included), must fit the PX = 256 / RY lanes
bool xpass_shape(int w, int W, int& RY, int& PJ) {
  for (RY = 4; RY >= 1; RY /= 2) {
    const int PX = XP_NT / RY;
    PJ = (int)((double)(PX - 6) * w / W) - 1;
    if (PJ >= 1) {
      PJ = std::min(PJ, w);
      return true;
    }
  }
  return false;
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

// ---- forward + gradient in one pass (training, integer factor S in {4, 8}): the corner-tile
// geometry of seg_loss_bwd_tile_kernel, with each tile's 2 x 2 low-res logit rows staged in LDS once
// (every pixel of the tile interpolates from them: the forward kernel above re-read its 4 taps from
// L2 per pixel) and the loss terms reduced per block. The residual (softmax - onehot) and the corner
// partials are left unscaled; seg_loss_gather_scaled_kernel applies gscale / count once the count is
// known (the backward then costs one gather).
template <typename T, int S, int NC>
__global__ __launch_bounds__(TILE_NT) void seg_loss_fused_tile_kernel(int B, int h, int w, int ncls,
                                                                      const T* __restrict__ lg, int H, int W,
                                                                      const long* __restrict__ label, int ignore,
                                                                      float* __restrict__ part,
                                                                      float* __restrict__ lpart, long ntiles) {
  constexpr int TP = S * S, TPW = 64 / TP;
  constexpr int RP = NC + 1;  // NC >= ncls: class registers / LDS rows sized for the class count
  __shared__ float res[TILE_NT][RP];
  __shared__ float wts[TILE_NT][4];
  __shared__ float corner[TILE_NT / 64][TPW][4][NC];
  __shared__ float lred[2][TILE_NT / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long tile0 = ((long)blockIdx.x * (TILE_NT / 64) + wid) * TPW;
  const int tw = w + 1, th = h + 1;
  // this wave's tiles' 4 corner cells (clamped; a clamped slot always carries weight 0)
  for (int e = lane; e < TPW * 4 * ncls; e += 64) {
    const int tt = e / (4 * ncls), k = (e / ncls) % 4, c = e % ncls;
    const long t = tile0 + tt;
    float v = 0.f;
    if (t < ntiles) {
      const int tx = t % tw, ty = (t / tw) % th, b = t / ((long)tw * th);
      const int cy = min(max(ty - 1 + (k >> 1), 0), h - 1), cx = min(max(tx - 1 + (k & 1), 0), w - 1);
      v = ldf(lg + (((long)b * h + cy) * w + cx) * ncls + c);
    }
    corner[wid][tt][k][c] = v;
  }
  __syncthreads();
  const long tile = tile0 + lane / TP;
  const int tt = lane / TP, d = lane % TP, dy = d / S, dx = d % S;
  float* row = res[threadIdx.x];
  float wv[4] = {0.f, 0.f, 0.f, 0.f};
  float ls = 0.f, lc = 0.f;
  if (tile < ntiles) {
    const int tx = tile % tw, ty = (tile / tw) % th, b = tile / ((long)tw * th);
    const int y = S * ty - S / 2 + dy, x = S * tx - S / 2 + dx;
    long lab = -1;
    if (y >= 0 && y < H && x >= 0 && x < W) lab = label[((long)b * H + y) * W + x];
    if (lab != ignore && lab >= 0 && lab < ncls) {
      int a0, a1, b0, b1;
      float ly, lx;
      src_idx(y, h, H, a0, a1, ly);
      src_idx(x, w, W, b0, b1, lx);
      const float wy[2] = {(a0 == ty - 1 ? 1.f - ly : 0.f) + (a1 == ty - 1 ? ly : 0.f),
                           (a0 == ty ? 1.f - ly : 0.f) + (a1 == ty ? ly : 0.f)};
      const float wx[2] = {(b0 == tx - 1 ? 1.f - lx : 0.f) + (b1 == tx - 1 ? lx : 0.f),
                           (b0 == tx ? 1.f - lx : 0.f) + (b1 == tx ? lx : 0.f)};
      wv[0] = wy[0] * wx[0]; wv[1] = wy[0] * wx[1]; wv[2] = wy[1] * wx[0]; wv[3] = wy[1] * wx[1];
      float z[NC];
      float m = -INFINITY, zl = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c < ncls) {
          z[c] = wv[0] * corner[wid][tt][0][c] + wv[1] * corner[wid][tt][1][c] + wv[2] * corner[wid][tt][2][c] +
                 wv[3] * corner[wid][tt][3][c];
          m = fmaxf(m, z[c]);
          zl = c == lab ? z[c] : zl;
        }
      }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < ncls) {
          z[c] = __expf(z[c] - m);
          se += z[c];
        }
      ls = m + __logf(se) - zl;
      lc = 1.f;
      const float rs = 1.f / se;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < ncls) row[c] = z[c] * rs - (c == lab ? 1.f : 0.f);
    } else {
      for (int c = 0; c < ncls; ++c) row[c] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) wts[threadIdx.x][k] = wv[k];
  ls = wave_sum(ls);
  lc = wave_sum(lc);
  if (lane == 0) {
    lred[0][wid] = ls;
    lred[1][wid] = lc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
#pragma unroll
    for (int q = 0; q < TILE_NT / 64; ++q) {
      a += lred[0][q];
      c += lred[1][q];
    }
    lpart[blockIdx.x * 2] = a;
    lpart[blockIdx.x * 2 + 1] = c;
  }
  for (int pr = lane; pr < TPW * ncls; pr += 64) {
    const int t2 = pr / ncls, c = pr % ncls;
    const long t = tile0 + t2;
    if (t >= ntiles) continue;
    const int base = wid * 64 + t2 * TP;
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

// (loss sum, valid count) of nblk block partials: 1024 lanes, fixed order
__global__ __launch_bounds__(1024) void seg_loss_sum_wide_kernel(int nblk, const float* __restrict__ part,
                                                                  float* __restrict__ out) {
  float s0 = 0.f, s1 = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 1024) {
    s0 += part[b * 2];
    s1 += part[b * 2 + 1];
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  __shared__ float red[2][16];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s0;
    red[1][threadIdx.x >> 6] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
    for (int q = 0; q < 16; ++q) {
      a += red[0][q];
      c += red[1][q];
    }
    out[0] = a;
    out[1] = c;
  }
}

// dlogits = gscale / count * (the 4 corner partials around each cell, fixed order), in TO
template <typename TO>
__global__ void seg_loss_gather_scaled_kernel(int B, int h, int w, int ncls, const float* __restrict__ part,
                                              const float* __restrict__ loss_out, const float* __restrict__ gscale,
                                              TO* __restrict__ dlg) {
  const long n = (long)B * h * w * ncls;
  const int tw = w + 1, th = h + 1;
  const float inv = (gscale ? gscale[0] : 1.f) / fmaxf(loss_out[1], 1.f);
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c = e % ncls;
    const long cell = e / ncls;
    const int j = cell % w, i = (cell / w) % h, b = cell / ((long)w * h);
    auto P = [&](int ty, int tx, int slot) { return part[((((long)b * th + ty) * tw + tx) * 4 + slot) * ncls + c]; };
    stf(dlg + e, inv * (P(i, j, 3) + P(i, j + 1, 2) + P(i + 1, j, 1) + P(i + 1, j + 1, 0)));
  }
}

template <typename T>
int launch_fused_tiles(int S, int B, int h, int w, int ncls, const void* lg, int H, int W, const long* label,
                       int ignore, float* loss_out, float* part, float* lpart, hipStream_t s) {
  const long ntiles = (long)B * (h + 1) * (w + 1);
  const long tiles_per_block = (TILE_NT / 64) * (64 / (S * S));
  const unsigned nb = cdiv(ntiles, tiles_per_block);
  // class rows sized 40 (NYUDepthv2's classes, SUN RGB-D's 37) or MAXC: the 64-wide form holds
  // 2 waves per SIMD (VGPRs and the residual rows in LDS), the 40-wide one 3 (461.8-462.1 ->
  // 464.4-464.5 images/s A/B)
#define SEG_GO(SS, NCC)                                                                                        \
  DFM_LAUNCH((seg_loss_fused_tile_kernel<T, SS, NCC>), dim3(nb), dim3(TILE_NT), 0, s, B, h, w, ncls, (const T*)lg, \
             H, W, label, ignore, part, lpart, ntiles)
  if (S == 8) {
    if (ncls <= 40) SEG_GO(8, 40);
    else SEG_GO(8, MAXC);
  } else {
    if (ncls <= 40) SEG_GO(4, 40);
    else SEG_GO(4, MAXC);
  }
#undef SEG_GO
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(seg_loss_sum_wide_kernel, dim3(1), dim3(1024), 0, s, (int)nb, (const float*)lpart, loss_out);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
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

/* backward workspace: the integer-scale path's corner partials of every tile, otherwise the x-pass's
   column-reduced rows rx [B][H][w][ncls] */
extern "C" size_t dfm_seg_loss_bwd_workspace(int B, int h, int w, int ncls, int H, int W) {
  if (tile_scale(h, w, H, W)) return (size_t)B * (h + 1) * (w + 1) * 4 * ncls * sizeof(float);
  return (size_t)B * H * w * ncls * sizeof(float);
}

extern "C" int dfm_seg_loss_fwd(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                const long* label, int ignore, float* lse, float* loss_out, void* workspace,
                                dfm_stream_t stream) {
  DFM_CHECK_ARG(logits && label && loss_out && workspace && ncls <= MAXC, "dfm_seg_loss_fwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)B * H * W;
  const int nblk = (int)min((long)LOSS_BLOCKS, (n + 255) / 256);
  if (dtype == DFM_BF16)
    DFM_LAUNCH((ncls <= 40 ? seg_loss_fwd_kernel<bf16_t, 40> : seg_loss_fwd_kernel<bf16_t, MAXC>), dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const bf16_t*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  else if (dtype == DFM_F16)
    DFM_LAUNCH((ncls <= 40 ? seg_loss_fwd_kernel<f16_t, 40> : seg_loss_fwd_kernel<f16_t, MAXC>), dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const f16_t*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  else
    DFM_LAUNCH((ncls <= 40 ? seg_loss_fwd_kernel<float, 40> : seg_loss_fwd_kernel<float, MAXC>), dim3(nblk), dim3(256), 0, s, B, h, w, ncls, (const float*)logits, H, W,
               label, ignore, lse, (float*)workspace);
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(seg_loss_sum_kernel, dim3(1), dim3(64), 0, s, nblk, (const float*)workspace, loss_out);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

static int fused_scale(int h, int w, int H, int W) {
  const int S = tile_scale(h, w, H, W);
  return S == 8 || S == 4 ? S : 0;
}

extern "C" size_t dfm_seg_loss_grad_partials_size(int B, int h, int w, int ncls, int H, int W) {
  if (!fused_scale(h, w, H, W)) return 0;
  const long ntiles = (long)B * (h + 1) * (w + 1);
  const long nb = (ntiles + 1) / 2;  // upper bound of the blocks (>= 2 tiles per block)
  return (size_t)(ntiles * 4 * ncls + nb * 2) * sizeof(float);
}

extern "C" int dfm_seg_loss_fwd_grad(int dtype, int B, int h, int w, int ncls, const void* logits, int H, int W,
                                     const long* label, int ignore, float* loss_out, float* grad_partials,
                                     dfm_stream_t stream) {
  const int S = fused_scale(h, w, H, W);
  DFM_CHECK_ARG(logits && label && loss_out && grad_partials && ncls <= MAXC && S,
                "dfm_seg_loss_fwd_grad: bad argument (needs ncls <= 64 and H = S h, W = S w, S in {4, 8})");
  hipStream_t s = (hipStream_t)stream;
  float* part = grad_partials;
  float* lpart = part + (long)B * (h + 1) * (w + 1) * 4 * ncls;
  if (dtype == DFM_BF16)
    return launch_fused_tiles<bf16_t>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, part, lpart, s);
  if (dtype == DFM_F16)
    return launch_fused_tiles<f16_t>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, part, lpart, s);
  if (dtype == DFM_F32)
    return launch_fused_tiles<float>(S, B, h, w, ncls, logits, H, W, label, ignore, loss_out, part, lpart, s);
  dfm_set_error("dfm_seg_loss_fwd_grad: bad dtype %d", dtype);
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_seg_loss_bwd_gather(int dtype_out, int B, int h, int w, int ncls, const float* grad_partials,
                                       const float* loss_out, const float* gscale, void* dlogits,
                                       dfm_stream_t stream) {
  DFM_CHECK_ARG(grad_partials && loss_out && dlogits && ncls > 0 && B > 0 && h > 0 && w > 0,
                "dfm_seg_loss_bwd_gather: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)B * h * w * ncls;
  const dim3 g((unsigned)std::min(8192L, (n + 255) / 256));
  if (dtype_out == DFM_BF16)
    DFM_LAUNCH(seg_loss_gather_scaled_kernel<bf16_t>, g, dim3(256), 0, s, B, h, w, ncls, grad_partials, loss_out,
               gscale, (bf16_t*)dlogits);
  else if (dtype_out == DFM_F16)
    DFM_LAUNCH(seg_loss_gather_scaled_kernel<f16_t>, g, dim3(256), 0, s, B, h, w, ncls, grad_partials, loss_out,
               gscale, (f16_t*)dlogits);
  else if (dtype_out == DFM_F32)
    DFM_LAUNCH(seg_loss_gather_scaled_kernel<float>, g, dim3(256), 0, s, B, h, w, ncls, grad_partials, loss_out,
               gscale, (float*)dlogits);
  else {
    dfm_set_error("dfm_seg_loss_bwd_gather: bad dtype %d", dtype_out);
    return DFM_ERR_DTYPE;
  }
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
  // other scales: separable x-pass into the workspace, then the y-pass
  DFM_CHECK_ARG(workspace, "dfm_seg_loss_bwd: needs dfm_seg_loss_bwd_workspace bytes of workspace");
  int RY, PJ;
  DFM_CHECK_ARG(xpass_shape(w, W, RY, PJ), "dfm_seg_loss_bwd: upsampling ratio W / w above ~120");
  float* rx = (float*)workspace;
  const unsigned nblk = (unsigned)((long)B * ((H + RY - 1) / RY) * ((w + PJ - 1) / PJ));
  const size_t lds = (size_t)XP_NT * (ncls + 1) * sizeof(float);
  if (lds > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<bf16_t, 40>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<bf16_t, MAXC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<f16_t, 40>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<f16_t, MAXC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<float, 40>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)seg_loss_bwd_xpass_kernel<float, MAXC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipGetLastError();  // a refused attribute must not read as this launch's error
  }
  if (dtype == DFM_BF16)
    DFM_LAUNCH((ncls <= 40 ? seg_loss_bwd_xpass_kernel<bf16_t, 40> : seg_loss_bwd_xpass_kernel<bf16_t, MAXC>), dim3(nblk), dim3(XP_NT), lds, s, B, h, w, ncls,
               (const bf16_t*)logits, H, W, label, ignore, loss_out, gscale, rx, RY, PJ);
  else if (dtype == DFM_F16)
    DFM_LAUNCH((ncls <= 40 ? seg_loss_bwd_xpass_kernel<f16_t, 40> : seg_loss_bwd_xpass_kernel<f16_t, MAXC>), dim3(nblk), dim3(XP_NT), lds, s, B, h, w, ncls,
               (const f16_t*)logits, H, W, label, ignore, loss_out, gscale, rx, RY, PJ);
  else
    DFM_LAUNCH((ncls <= 40 ? seg_loss_bwd_xpass_kernel<float, 40> : seg_loss_bwd_xpass_kernel<float, MAXC>), dim3(nblk), dim3(XP_NT), lds, s, B, h, w, ncls,
               (const float*)logits, H, W, label, ignore, loss_out, gscale, rx, RY, PJ);
  DFM_LAUNCH_CHECK();
  DFM_LAUNCH(seg_loss_bwd_ypass_kernel, dim3((unsigned)std::min(8192L, (nl + 255) / 256)), dim3(256), 0, s, B, h,
             w, ncls, H, (const float*)rx, dlogits);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
