// Multi-scale + flip evaluation (utils/val_mm.py:325-472 evaluate_msf) and the mIoU confusion
// histogram (utils/metrics_new.py:16-20) on the GPU:
//   dfm_resize_nchw     F.interpolate(img, (Ho, Wo), bilinear, align_corners) [+ torch.flip(dims=3)]
//                       of the rgb / depth inputs, read with any strides (val_mm.py:362-372, 386-388)
//   dfm_msf_accumulate  acc[b, y, x, :] += softmax_c( resize_{align_corners=True}(H, W) of
//                       [flip of] resize_{align_corners=False}(Hs, Ws) of the decoder's low-res
//                       logits )  — the model's own upsampling (builder.py:203), the flip back
//                       (val_mm.py:389) and the resize to the label size (val_mm.py:377-379,
//                       390-392) composed per output pixel: 16 low-res taps, nothing materialised
//   dfm_seg_confusion   hist[t * ncls + argmax_c acc[p, c]] += 1 over pixels with t != ignore
// Every output element is owned by one thread (no float atomics); the histogram uses integer
// atomics, so all three are deterministic.
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxCls = 64;

// PyTorch's source-index rule for bilinear resizing (area_pixel_compute_source_index)
struct Lin {
  int i0, i1;
  float l0, l1;
};
DFM_INLINE Lin lin_src(int dst, int in, int out, bool align) {
  float src;
  if (align) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    src = scale * (float)dst;
  } else {
    const float scale = (float)in / (float)out;
    src = fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  }
  Lin r;
  r.i0 = min((int)src, in - 1);
  r.i1 = min(r.i0 + 1, in - 1);
  r.l1 = src - (float)r.i0;
  r.l0 = 1.f - r.l1;
  return r;
}

template <typename Ti, typename To>
__global__ __launch_bounds__(kThreads) void resize_nchw_kernel(int B, int C, int Hi, int Wi, long sb, long sc, long sh,
                                                               long sw, int Ho, int Wo, int align, int flip,
                                                               const Ti* __restrict__ x, To* __restrict__ y) {
  const long n = (long)B * C * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % Wo);
    long t = i / Wo;
    const int oy = (int)(t % Ho);
    t /= Ho;
    const int c = (int)(t % C);
    const long b = t / C;
    const Lin ly = lin_src(oy, Hi, Ho, align), lx = lin_src(flip ? Wo - 1 - ox : ox, Wi, Wo, align);
    const Ti* p = x + b * sb + c * sc;
    const float v = ly.l0 * (lx.l0 * ldf(p + ly.i0 * sh + lx.i0 * sw) + lx.l1 * ldf(p + ly.i0 * sh + lx.i1 * sw)) +
                    ly.l1 * (lx.l0 * ldf(p + ly.i1 * sh + lx.i0 * sw) + lx.l1 * ldf(p + ly.i1 * sh + lx.i1 * sw));
    stf(y + i, v);
  }
}

template <typename T, int NC>
__global__ __launch_bounds__(kThreads) void msf_accumulate_kernel(int B, int h, int w, int ncls,
                                                                  const T* __restrict__ low, long ldl, int Hs, int Ws,
                                                                  int H, int W, int flip, float* __restrict__ acc) {
  const long n = (long)B * H * W;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    const int x = (int)(p % W);
    const long t = p / W;
    const int y = (int)(t % H);
    const long b = t / H;
    float z[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) z[c] = 0.f;
    const Lin sy = lin_src(y, Hs, H, true), sx = lin_src(x, Ws, W, true);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int ys = (a >> 1) ? sy.i1 : sy.i0;
      const int xs0 = (a & 1) ? sx.i1 : sx.i0;
      const float wa = ((a >> 1) ? sy.l1 : sy.l0) * ((a & 1) ? sx.l1 : sx.l0);
      const int xs = flip ? Ws - 1 - xs0 : xs0;
      const Lin ly = lin_src(ys, h, Hs, false), lx = lin_src(xs, w, Ws, false);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int yl = (q >> 1) ? ly.i1 : ly.i0, xl = (q & 1) ? lx.i1 : lx.i0;
        const float wq = wa * ((q >> 1) ? ly.l1 : ly.l0) * ((q & 1) ? lx.l1 : lx.l0);
        const T* src = low + ((b * h + yl) * w + xl) * ldl;
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (c < ncls) z[c] = fmaf(wq, ldf(src + c), z[c]);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < ncls) mx = fmaxf(mx, z[c]);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < ncls) {
        z[c] = expf(z[c] - mx);
        s += z[c];
      }
    const float inv = 1.f / s;
    float* dst = acc + p * ncls;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < ncls) dst[c] += z[c] * inv;
  }
}

__global__ __launch_bounds__(kThreads) void confusion_kernel(long npix, int ncls, const float* __restrict__ acc,
                                                             const long long* __restrict__ label, int ignore,
                                                             unsigned long long* __restrict__ hist) {
  extern __shared__ unsigned int lh[];
  const int nb = ncls * ncls;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0u;
  __syncthreads();
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long long t = label[p];
    if (t == ignore || t < 0 || t >= ncls) continue;
    const float* a = acc + p * ncls;
    int best = 0;
    float bv = a[0];
    for (int c = 1; c < ncls; ++c) {
      const float v = a[c];
      if (v > bv) {  // first maximum wins, like torch.argmax
        bv = v;
        best = c;
      }
    }
    atomicAdd(&lh[t * ncls + best], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += blockDim.x)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}

unsigned grid_for(long n, long cap = 16384) {
  const long g = (n + kThreads - 1) / kThreads;
  return (unsigned)(g < cap ? (g < 1 ? 1 : g) : cap);
}

template <typename T>
int msf_typed(int B, int h, int w, int ncls, const void* low, long ldl, int Hs, int Ws, int H, int W, int flip,
              float* acc, hipStream_t s) {
  const unsigned g = grid_for((long)B * H * W);
  if (ncls <= 16)
    DFM_LAUNCH((msf_accumulate_kernel<T, 16>), dim3(g), dim3(kThreads), 0, s, B, h, w, ncls, (const T*)low, ldl, Hs,
               Ws, H, W, flip, acc);
  else if (ncls <= 40)
    DFM_LAUNCH((msf_accumulate_kernel<T, 40>), dim3(g), dim3(kThreads), 0, s, B, h, w, ncls, (const T*)low, ldl, Hs,
               Ws, H, W, flip, acc);
  else
    DFM_LAUNCH((msf_accumulate_kernel<T, kMaxCls>), dim3(g), dim3(kThreads), 0, s, B, h, w, ncls, (const T*)low, ldl,
               Hs, Ws, H, W, flip, acc);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

}  // namespace

extern "C" int dfm_resize_nchw(int dtype_in, int dtype_out, int B, int C, int Hi, int Wi, long sb, long sc, long sh,
                               long sw, const void* x, int Ho, int Wo, int align_corners, int flip, void* y,
                               dfm_stream_t stream) {
  DFM_CHECK_ARG(x && y && B > 0 && C > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "dfm_resize_nchw: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = grid_for((long)B * C * Ho * Wo);
#define DFM_RESIZE(TI, TO)                                                                                          \
  DFM_LAUNCH((resize_nchw_kernel<TI, TO>), dim3(g), dim3(kThreads), 0, s, B, C, Hi, Wi, sb, sc, sh, sw, Ho, Wo,      \
             align_corners, flip, (const TI*)x, (TO*)y)
  if (dtype_in == DFM_F32 && dtype_out == DFM_F32) DFM_RESIZE(float, float);
  else if (dtype_in == DFM_BF16 && dtype_out == DFM_F32) DFM_RESIZE(bf16_t, float);
  else if (dtype_in == DFM_F32 && dtype_out == DFM_BF16) DFM_RESIZE(float, bf16_t);
  else if (dtype_in == DFM_BF16 && dtype_out == DFM_BF16) DFM_RESIZE(bf16_t, bf16_t);
  else if (dtype_in == DFM_F16 && dtype_out == DFM_F32) DFM_RESIZE(f16_t, float);
  else if (dtype_in == DFM_F32 && dtype_out == DFM_F16) DFM_RESIZE(float, f16_t);
  else {
    dfm_set_error("dfm_resize_nchw: unsupported dtypes %d -> %d", dtype_in, dtype_out);
    return DFM_ERR_DTYPE;
  }
#undef DFM_RESIZE
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_msf_accumulate(int dtype, int B, int h, int w, int ncls, const void* low, long ldl, int Hs, int Ws,
                                  int H, int W, int flip, float* acc, dfm_stream_t stream) {
  DFM_CHECK_ARG(low && acc && B > 0 && h > 0 && w > 0 && Hs > 0 && Ws > 0 && H > 0 && W > 0 && ldl >= ncls,
                "dfm_msf_accumulate: bad argument");
  DFM_CHECK_ARG(ncls > 0 && ncls <= kMaxCls, "dfm_msf_accumulate: ncls=%d outside [1, %d]", ncls, kMaxCls);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return msf_typed<bf16_t>(B, h, w, ncls, low, ldl, Hs, Ws, H, W, flip, acc, s);
  if (dtype == DFM_F16) return msf_typed<f16_t>(B, h, w, ncls, low, ldl, Hs, Ws, H, W, flip, acc, s);
  if (dtype == DFM_F32) return msf_typed<float>(B, h, w, ncls, low, ldl, Hs, Ws, H, W, flip, acc, s);
  dfm_set_error("dfm_msf_accumulate: unsupported dtype %d", dtype);
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_seg_confusion(long npix, int ncls, const float* acc, const long long* label, int ignore,
                                 unsigned long long* hist, dfm_stream_t stream) {
  DFM_CHECK_ARG(acc && label && hist && npix >= 0 && ncls > 0 && ncls <= kMaxCls,
                "dfm_seg_confusion: bad argument (ncls <= %d)", kMaxCls);
  if (npix == 0) return DFM_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)ncls * ncls * sizeof(unsigned int);
  DFM_LAUNCH(confusion_kernel, dim3(grid_for(npix, 2048)), dim3(kThreads), lds, s, npix, ncls, acc, label, ignore,
             hist);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
