// Dense 3x3 stride-2 pad-1 convolution of the stems and stage downsampling (DFormer.py:194-228,
// 295-303) as an explicit gather + MFMA GEMM over NHWC rows:
//
//   cols[m, (kh*3+kw)*Cin + c] = act(bn(x[b, c, 2*oh-1+kh, 2*ow-1+kw]))  (0 outside the image)
//   y[m, :] = cols[m, :] @ Wp^T + bias          (dfm_gemm; Wp = weight packed to [Cout, (kh,kw,c)])
//
// The BatchNorm that precedes the convolution (stage i>0: BN/SyncBN -> conv; stem: conv -> BN ->
// GELU -> conv) is folded into the gather as a per-channel affine (+ exact-erf GELU), so neither
// the normalised nor the activated tensor is ever written to HBM. The input may be any strided
// NCHW-logical tensor (the raw float32 image, the depth channel view x_e[:, 0:1], or the NHWC rows
// of the previous stage), so no NCHW<->NHWC permute copy is needed on either side.
// Backward: dcols = dy @ Wp (dfm_gemm), then dfm_conv3s2_col2im gathers the <= 4 taps that touch
// every input pixel in a fixed order (deterministic, no atomics) and applies the recomputed GELU'
// of the folded BN output; the BN backward itself runs on the library's BN kernels.
#include "common.h"

namespace {

constexpr int kThreads = 256;

constexpr int kMaxAffC = 1024;  // channels of a folded BN (DFormer-Large: <= 288)

struct Affine {
  const float *mean, *rstd, *gamma, *beta;
  int gelu;
  DFM_INLINE float operator()(float v, int c) const {
    if (mean) v = (v - mean[c]) * rstd[c] * gamma[c] + beta[c];
    if (gelu) v = gelu_f(v);
    return v;
  }
};

// The folded BN as y = x * sc[c] + sh[c], staged once per block in LDS (a per-element lookup of
// four global parameter vectors costs more than the gather itself).
struct AffineLds {
  float* sc;
  float* sh;
  bool on;
  int gelu;
  DFM_INLINE float operator()(float v, int c) const {
    if (on) v = fmaf(v, sc[c], sh[c]);
    if (gelu) v = gelu_f(v);
    return v;
  }
};
DFM_INLINE AffineLds stage_affine(const Affine& af, int C, float* sc, float* sh) {
  if (af.mean) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float a = af.rstd[c] * af.gamma[c];
      sc[c] = a;
      sh[c] = af.beta[c] - af.mean[c] * a;
    }
    __syncthreads();
  }
  return AffineLds{sc, sh, af.mean != nullptr, af.gelu};
}

// Vector gather: one thread = one output row m, one tap, 8 consecutive channels (Cin % 8 == 0,
// channel stride 1, 16-byte aligned pixel rows). Kp == 9*Cin.
// I: index type (32-bit when the element count fits: no 64-bit division in the index math).
template <typename Ti, typename To, typename I>
__global__ __launch_bounds__(kThreads) void im2col_vec_kernel(long M, int Ho, int Wo, int H, int W, int Cin, long sb,
                                                              long sh, long sw, const Ti* __restrict__ x, Affine af,
                                                              To* __restrict__ cols) {
  __shared__ float s_sc[kMaxAffC], s_sh[kMaxAffC];
  const AffineLds al = stage_affine(af, Cin, s_sc, s_sh);
  const I cv = (I)(Cin >> 3);
  const I n = (I)(M * 9 * cv);
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cv);
    const I rest = i / cv;
    const int tap = (int)(rest % 9u);
    const I m = rest / 9u;
    const int ow = (int)(m % (I)Wo);
    const I t = m / (I)Wo;
    const int oh = (int)(t % (I)Ho);
    const long b = (long)(t / (I)Ho);
    const int ih = 2 * oh - 1 + tap / 3, iw = 2 * ow - 1 + tap % 3;
    float v[8];
    if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
      ld8<Ti>(x + b * sb + ih * sh + iw * sw + c8 * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = al(v[e], c8 * 8 + e);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
    }
    st8<To>(cols + (long)m * (9 * Cin) + tap * Cin + c8 * 8, v);
  }
}

// Generic gather: one thread = one output row, 8 consecutive columns of Kp (zero padded past
// 9*Cin); any input strides (the NCHW float32 image with Cin = 3, the depth view with Cin = 1).
template <typename Ti, typename To, typename I>
__global__ __launch_bounds__(kThreads) void im2col_gen_kernel(long M, int Ho, int Wo, int H, int W, int Cin, long sb,
                                                              long sc, long sh, long sw, int Kp,
                                                              const Ti* __restrict__ x, Affine af,
                                                              To* __restrict__ cols) {
  const I kv = (I)(Kp >> 3);
  const int K = 9 * Cin;
  const I n = (I)(M * kv);
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    const int k0 = (int)(i % kv) * 8;
    const long m = (long)(i / kv);
    const I mi = i / kv;
    const int ow = (int)(mi % (I)Wo);
    const I t = mi / (I)Wo;
    const int oh = (int)(t % (I)Ho);
    const long b = (long)(t / (I)Ho);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      v[e] = 0.f;
      if (k < K) {
        const int tap = k / Cin, c = k - tap * Cin;
        const int ih = 2 * oh - 1 + tap / 3, iw = 2 * ow - 1 + tap % 3;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W) v[e] = af(ldf(x + b * sb + c * sc + ih * sh + iw * sw), c);
      }
    }
    st8<To>(cols + m * (long)Kp + k0, v);
  }
}

// dx[b, ih, iw, c..c+7] (+)= act'(.) * sum over the taps (kh, kw) with 2*oh-1+kh == ih,
// 2*ow-1+kw == iw of dcols[(b, oh, ow), (kh*3+kw)*Cin + c..]; taps visited in a fixed order.
template <typename T, typename I>
__global__ __launch_bounds__(kThreads) void col2im_vec_kernel(int B, int H, int W, int Cin, int Ho, int Wo,
                                                              const T* __restrict__ dcols, long ldc,
                                                              const T* __restrict__ x, long ldx, Affine af,
                                                              T* __restrict__ dx, long lddx, int accumulate) {
  __shared__ float s_sc[kMaxAffC], s_sh[kMaxAffC];
  const AffineLds al = stage_affine(af, Cin, s_sc, s_sh);
  const I cv = (I)(Cin >> 3);
  const I n = (I)((long)B * H * W * cv);
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < n; i += (I)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cv) * 8;
    const long p = (long)(i / cv);
    const I pi = i / cv;
    const int iw = (int)(pi % (I)W);
    const I t = pi / (I)W;
    const int ih = (int)(t % (I)H);
    const long b = (long)(t / (I)H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int th = ih + 1 - kh;
      if (th < 0 || (th & 1) || (th >> 1) >= Ho) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tw = iw + 1 - kw;
        if (tw < 0 || (tw & 1) || (tw >> 1) >= Wo) continue;
        float v[8];
        ld8<T>(dcols + ((b * Ho + (th >> 1)) * Wo + (tw >> 1)) * ldc + (kh * 3 + kw) * Cin + c0, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
    if (af.gelu) {
      float xv[8];
      ld8<T>(x + p * ldx + c0, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float z = al.on ? fmaf(xv[e], al.sc[c0 + e], al.sh[c0 + e]) : xv[e];
        acc[e] *= gelu_grad_f(z);
      }
    }
    T* dp = dx + p * lddx + c0;
    if (accumulate) {
      float o[8];
      ld8<T>(dp, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += o[e];
    }
    st8<T>(dp, acc);
  }
}

// Generic input gradient of a conv without a folded BN (the stem's first conv: Cin = 3 / 1, input
// gradient of the image itself): one thread per input element, any output strides.
template <typename T, typename To>
__global__ __launch_bounds__(kThreads) void col2im_gen_kernel(int B, int Cin, int H, int W, int Ho, int Wo,
                                                              const T* __restrict__ dcols, long ldc, To* __restrict__ dx,
                                                              long sb, long sc, long sh, long sw) {
  const long n = (long)B * Cin * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int iw = (int)(i % W);
    long t = i / W;
    const int ih = (int)(t % H);
    t /= H;
    const int c = (int)(t % Cin);
    const long b = t / Cin;
    float acc = 0.f;
    for (int kh = 0; kh < 3; ++kh) {
      const int th = ih + 1 - kh;
      if (th < 0 || (th & 1) || (th >> 1) >= Ho) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int tw = iw + 1 - kw;
        if (tw < 0 || (tw & 1) || (tw >> 1) >= Wo) continue;
        acc += ldf(dcols + ((b * Ho + (th >> 1)) * Wo + (tw >> 1)) * ldc + (kh * 3 + kw) * Cin + c);
      }
    }
    stf(dx + b * sb + c * sc + ih * sh + iw * sw, acc);
  }
}

// w float32 [Cout][Cin][3][3] -> wp [Cout][Kp], wp[o][(kh*3+kw)*Cin + c] (zero past 9*Cin)
template <typename To>
__global__ void weight_pack_kernel(int Cout, int Cin, int Kp, const float* __restrict__ w, To* __restrict__ wp) {
  const long n = (long)Cout * Kp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % Kp);
    const long o = i / Kp;
    float v = 0.f;
    if (k < 9 * Cin) {
      const int tap = k / Cin, c = k - tap * Cin;
      v = w[(o * Cin + c) * 9 + tap];
    }
    stf(wp + i, v);
  }
}

// dwp float32 [Cout][Kp] -> dw float32 [Cout][Cin][3][3]
__global__ void weight_unpack_kernel(int Cout, int Cin, int Kp, const float* __restrict__ dwp, float* __restrict__ dw,
                                     int accumulate) {
  const long n = (long)Cout * Cin * 9;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int tap = (int)(i % 9);
    const long r = i / 9;
    const int c = (int)(r % Cin);
    const long o = r / Cin;
    const float v = dwp[o * Kp + tap * Cin + c];
    dw[i] = accumulate ? dw[i] + v : v;
  }
}

unsigned grid_for(long n) {
  const long g = (n + kThreads - 1) / kThreads;
  return (unsigned)(g < 65536 ? (g < 1 ? 1 : g) : 65536);
}

template <typename Ti, typename To>
int im2col_typed(int B, int H, int W, int Cin, long sb, long sc, long sh, long sw, const void* x, Affine af, int Kp,
                 void* cols, hipStream_t s) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long M = (long)B * Ho * Wo;
  const bool vec = sc == 1 && Cin % 8 == 0 && Kp == 9 * Cin && (uintptr_t)x % 16 == 0 && sb % 8 == 0 &&
                   sh % 8 == 0 && sw % 8 == 0;
  if (vec) {
    const long n = M * 9 * (Cin / 8);
    if (n < (1L << 31))
      DFM_LAUNCH((im2col_vec_kernel<Ti, To, unsigned>), dim3(grid_for(n)), dim3(kThreads), 0, s, M, Ho, Wo, H, W, Cin,
                 sb, sh, sw, (const Ti*)x, af, (To*)cols);
    else
      DFM_LAUNCH((im2col_vec_kernel<Ti, To, long>), dim3(grid_for(n)), dim3(kThreads), 0, s, M, Ho, Wo, H, W, Cin, sb,
                 sh, sw, (const Ti*)x, af, (To*)cols);
  } else {
    const long n = M * (Kp / 8);
    if (n < (1L << 31))
      DFM_LAUNCH((im2col_gen_kernel<Ti, To, unsigned>), dim3(grid_for(n)), dim3(kThreads), 0, s, M, Ho, Wo, H, W, Cin,
                 sb, sc, sh, sw, Kp, (const Ti*)x, af, (To*)cols);
    else
      DFM_LAUNCH((im2col_gen_kernel<Ti, To, long>), dim3(grid_for(n)), dim3(kThreads), 0, s, M, Ho, Wo, H, W, Cin, sb,
                 sc, sh, sw, Kp, (const Ti*)x, af, (To*)cols);
  }
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

}  // namespace

extern "C" int dfm_conv3s2_im2col(int dtype_in, int dtype_out, int B, int H, int W, int Cin, long sb, long sc,
                                  long sh, long sw, const void* x, const float* mean, const float* rstd,
                                  const float* gamma, const float* beta, int gelu, int Kp, void* cols,
                                  dfm_stream_t stream) {
  DFM_CHECK_ARG(x && cols, "dfm_conv3s2_im2col: null argument");
  DFM_CHECK_ARG(B > 0 && H > 0 && W > 0 && Cin > 0, "dfm_conv3s2_im2col: bad shape");
  DFM_CHECK_ARG(Kp % 8 == 0 && Kp >= 9 * Cin, "dfm_conv3s2_im2col: Kp=%d must be a multiple of 8 >= 9*Cin", Kp);
  DFM_CHECK_ARG((uintptr_t)cols % 16 == 0, "dfm_conv3s2_im2col: cols must be 16-byte aligned");
  DFM_CHECK_ARG(!mean || (rstd && gamma && beta), "dfm_conv3s2_im2col: partial BatchNorm parameters");
  DFM_CHECK_ARG(!mean || Cin <= kMaxAffC, "dfm_conv3s2_im2col: folded BN over %d > %d channels", Cin, kMaxAffC);
  const Affine af{mean, rstd, gamma, beta, gelu};
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == DFM_F32 && dtype_out == DFM_F32)
    return im2col_typed<float, float>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  if (dtype_in == DFM_F32 && dtype_out == DFM_BF16)
    return im2col_typed<float, bf16_t>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  if (dtype_in == DFM_BF16 && dtype_out == DFM_BF16)
    return im2col_typed<bf16_t, bf16_t>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  if (dtype_in == DFM_BF16 && dtype_out == DFM_F32)
    return im2col_typed<bf16_t, float>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  if (dtype_in == DFM_F32 && dtype_out == DFM_F16)
    return im2col_typed<float, f16_t>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  if (dtype_in == DFM_F16 && dtype_out == DFM_F16)
    return im2col_typed<f16_t, f16_t>(B, H, W, Cin, sb, sc, sh, sw, x, af, Kp, cols, s);
  dfm_set_error("dfm_conv3s2_im2col: unsupported dtypes %d -> %d", dtype_in, dtype_out);
  return DFM_ERR_DTYPE;
}

extern "C" int dfm_conv3s2_col2im(int dtype, int B, int H, int W, int Cin, const void* dcols, long ldc,
                                  const void* x, long ldx, const float* mean, const float* rstd, const float* gamma,
                                  const float* beta, int gelu, void* dx, long lddx, int accumulate,
                                  dfm_stream_t stream) {
  DFM_CHECK_ARG(dcols && dx && (!gelu || x), "dfm_conv3s2_col2im: null argument");
  DFM_CHECK_ARG(B > 0 && H > 0 && W > 0 && Cin > 0 && Cin % 8 == 0, "dfm_conv3s2_col2im: Cin=%d must be a multiple of 8",
                Cin);
  DFM_CHECK_ARG(ldc >= 9 * Cin && ldc % 8 == 0 && lddx % 8 == 0 && (!gelu || ldx % 8 == 0),
                "dfm_conv3s2_col2im: row strides must be multiples of 8");
  DFM_CHECK_ARG((uintptr_t)dcols % 16 == 0 && (uintptr_t)dx % 16 == 0 && (uintptr_t)x % 16 == 0,
                "dfm_conv3s2_col2im: operands must be 16-byte aligned");
  DFM_CHECK_ARG(!mean || (rstd && gamma && beta), "dfm_conv3s2_col2im: partial BatchNorm parameters");
  DFM_CHECK_ARG(!mean || Cin <= kMaxAffC, "dfm_conv3s2_col2im: folded BN over %d > %d channels", Cin, kMaxAffC);
  const Affine af{mean, rstd, gamma, beta, gelu};
  hipStream_t s = (hipStream_t)stream;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long n = (long)B * H * W * (Cin / 8);
#define DFM_C2IV(T, I)                                                                                     \
  DFM_LAUNCH((col2im_vec_kernel<T, I>), dim3(grid_for(n)), dim3(kThreads), 0, s, B, H, W, Cin, Ho, Wo,        \
             (const T*)dcols, ldc, (const T*)x, ldx, af, (T*)dx, lddx, accumulate)
  const bool i32 = n < (1L << 31);
  if (dtype == DFM_BF16) {
    if (i32) DFM_C2IV(bf16_t, unsigned); else DFM_C2IV(bf16_t, long);
  } else if (dtype == DFM_F16) {
    if (i32) DFM_C2IV(f16_t, unsigned); else DFM_C2IV(f16_t, long);
  } else if (dtype == DFM_F32) {
    if (i32) DFM_C2IV(float, unsigned); else DFM_C2IV(float, long);
  } else {
    dfm_set_error("dfm_conv3s2_col2im: unsupported dtype %d", dtype);
    return DFM_ERR_DTYPE;
  }
#undef DFM_C2IV
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_conv3s2_col2im_nchw(int dtype, int dtype_out, int B, int H, int W, int Cin, const void* dcols,
                                       long ldc, void* dx, long sb, long sc, long sh, long sw, dfm_stream_t stream) {
  DFM_CHECK_ARG(dcols && dx && B > 0 && H > 0 && W > 0 && Cin > 0 && ldc >= 9 * Cin,
                "dfm_conv3s2_col2im_nchw: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long n = (long)B * Cin * H * W;
#define DFM_C2I(T, TO)                                                                                        \
  DFM_LAUNCH((col2im_gen_kernel<T, TO>), dim3(grid_for(n)), dim3(kThreads), 0, s, B, Cin, H, W, Ho, Wo,       \
             (const T*)dcols, ldc, (TO*)dx, sb, sc, sh, sw)
  if (dtype == DFM_F32 && dtype_out == DFM_F32) DFM_C2I(float, float);
  else if (dtype == DFM_BF16 && dtype_out == DFM_F32) DFM_C2I(bf16_t, float);
  else if (dtype == DFM_BF16 && dtype_out == DFM_BF16) DFM_C2I(bf16_t, bf16_t);
  else if (dtype == DFM_F16 && dtype_out == DFM_F32) DFM_C2I(f16_t, float);
  else if (dtype == DFM_F16 && dtype_out == DFM_F16) DFM_C2I(f16_t, f16_t);
  else if (dtype == DFM_F32 && dtype_out == DFM_BF16) DFM_C2I(float, bf16_t);
  else {
    dfm_set_error("dfm_conv3s2_col2im_nchw: unsupported dtypes %d -> %d", dtype, dtype_out);
    return DFM_ERR_DTYPE;
  }
#undef DFM_C2I
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_conv3_weight_pack(int dtype_out, int Cout, int Cin, int Kp, const float* w, void* wp,
                                     dfm_stream_t stream) {
  DFM_CHECK_ARG(w && wp, "dfm_conv3_weight_pack: null argument");
  DFM_CHECK_ARG(Cout > 0 && Cin > 0 && Kp >= 9 * Cin, "dfm_conv3_weight_pack: bad shape");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)Cout * Kp;
  if (dtype_out == DFM_BF16)
    DFM_LAUNCH(weight_pack_kernel<bf16_t>, dim3(grid_for(n)), dim3(kThreads), 0, s, Cout, Cin, Kp, w, (bf16_t*)wp);
  else if (dtype_out == DFM_F16)
    DFM_LAUNCH(weight_pack_kernel<f16_t>, dim3(grid_for(n)), dim3(kThreads), 0, s, Cout, Cin, Kp, w, (f16_t*)wp);
  else if (dtype_out == DFM_F32)
    DFM_LAUNCH(weight_pack_kernel<float>, dim3(grid_for(n)), dim3(kThreads), 0, s, Cout, Cin, Kp, w, (float*)wp);
  else {
    dfm_set_error("dfm_conv3_weight_pack: unsupported dtype %d", dtype_out);
    return DFM_ERR_DTYPE;
  }
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

extern "C" int dfm_conv3_weight_unpack(int Cout, int Cin, int Kp, const float* dwp, float* dw, int accumulate,
                                       dfm_stream_t stream) {
  DFM_CHECK_ARG(dwp && dw, "dfm_conv3_weight_unpack: null argument");
  DFM_CHECK_ARG(Cout > 0 && Cin > 0 && Kp >= 9 * Cin, "dfm_conv3_weight_unpack: bad shape");
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)Cout * Cin * 9;
  DFM_LAUNCH(weight_unpack_kernel, dim3(grid_for(n)), dim3(kThreads), 0, s, Cout, Cin, Kp, dwp, dw, accumulate);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
