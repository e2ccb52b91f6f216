// Shared helpers for the DFormer gfx950 kernels: dtypes, bf16 packing, error reporting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dformer_hip.h"

typedef uint16_t bf16_t;  // raw bfloat16 bits
struct f16_t {            // raw IEEE binary16 bits (a distinct type so templates tell it from bf16)
  uint16_t bits;
};
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float float4_t;

#define DFM_INLINE __device__ __forceinline__

// ---- bf16 <-> f32 (round-to-nearest-even; NaN preserved by the compiler's v_cvt_pk_bf16_f32)
DFM_INLINE float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
DFM_INLINE bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> struct Num;
template <> struct Num<float> {
  static DFM_INLINE float load(const float* p) { return *p; }
  static DFM_INLINE float to_f(float v) { return v; }
  static DFM_INLINE float from_f(float v) { return v; }
};
template <> struct Num<bf16_t> {
  static DFM_INLINE float load(const bf16_t* p) { return bf2f(*p); }
  static DFM_INLINE float to_f(bf16_t v) { return bf2f(v); }
  static DFM_INLINE bf16_t from_f(float v) { return f2bf(v); }
};
DFM_INLINE float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
DFM_INLINE uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
template <> struct Num<f16_t> {
  static DFM_INLINE float load(const f16_t* p) { return h2f(p->bits); }
  static DFM_INLINE float to_f(f16_t v) { return h2f(v.bits); }
  static DFM_INLINE f16_t from_f(float v) { return f16_t{f2h(v)}; }
};
template <typename T> DFM_INLINE float ldf(const T* p) { return Num<T>::load(p); }
template <typename T> DFM_INLINE void stf(T* p, float v) { *p = Num<T>::from_f(v); }

// Exact-erf GELU (nn.GELU() default, DFormer.py:51,78) without the branchy libm erff: the
// normal CDF from Abramowitz & Stegun 7.1.26 (|erf error| <= 1.5e-7, one v_rcp + one v_exp),
// evaluated on the tail side so Phi(x) for x << 0 keeps its relative accuracy; the same
// exponential gives the normal pdf for the derivative.
DFM_INLINE void normal_cdf_pdf(float x, float& cdf, float& pdf) {
  const float u = x * 0.70710678118654752f;
  const float au = fabsf(u);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, au, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __expf(-au * au);
  const float tail = 0.5f * p * e;  // Phi(-|x|)
  cdf = u < 0.0f ? tail : 1.0f - tail;
  pdf = 0.39894228040143268f * e;
}
// The same on a channel pair: every non-transcendental step as one v_pk_* instruction (the 0.5 of the
// tail is folded into the coefficients, exact in binary), so each element is bit-identical to
// normal_cdf_pdf's; 25 instructions per pair instead of 2 x 19.
typedef __attribute__((ext_vector_type(2))) float float2_t;
DFM_INLINE void normal_cdf_pdf2(float2_t x, float2_t& cdf, float2_t& pdf) {
  const float2_t u = x * 0.70710678118654752f;
  const float2_t au = __builtin_elementwise_abs(u);
  const float2_t den = __builtin_elementwise_fma(au, float2_t{0.3275911f, 0.3275911f}, float2_t{1.0f, 1.0f});
  const float2_t t = float2_t{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  float2_t p = __builtin_elementwise_fma(float2_t{0.5307027145f, 0.5307027145f}, t,
                                         float2_t{-0.7265760135f, -0.7265760135f});
  p = __builtin_elementwise_fma(p, t, float2_t{0.7107068705f, 0.7107068705f});
  p = __builtin_elementwise_fma(p, t, float2_t{-0.142248368f, -0.142248368f});
  p = __builtin_elementwise_fma(p, t, float2_t{0.127414796f, 0.127414796f});
  p *= t;
  const float2_t z = (au * au) * -1.4426950408889634f;
  const float2_t e = float2_t{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
  const float2_t tail = p * e;  // Phi(-|x|)
  cdf.x = u.x < 0.0f ? tail.x : 1.0f - tail.x;
  cdf.y = u.y < 0.0f ? tail.y : 1.0f - tail.y;
  pdf = e * 0.39894228040143268f;
}
DFM_INLINE float gelu_f(float x) {
  float c, d;
  normal_cdf_pdf(x, c, d);
  return x * c;
}
DFM_INLINE float gelu_grad_f(float x) {
  float c, d;
  normal_cdf_pdf(x, c, d);
  return fmaf(x, d, c);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not its global
// loads or stores (__syncthreads()' fence drains vmcnt, so a register prefetch of the next k-slice or
// an epilogue's output stores would be waited for at every barrier); the inline asm's memory clobber
// keeps the compiler from moving LDS accesses across it. Global loads are still waited for before
// their registers are used (the compiler's per-register vmcnt tracking).
DFM_INLINE void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

DFM_INLINE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DFM_INLINE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// sum over aligned groups of G lanes (G power of two <= 64)
template <int G> DFM_INLINE float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 8 consecutive T elements <-> floats
template <typename T> DFM_INLINE void ld8(const T* p, float* v);
template <> DFM_INLINE void ld8<bf16_t>(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <> DFM_INLINE void ld8<f16_t>(const f16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = h2f((uint16_t)(w[i] & 0xffffu));
    v[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
  }
}
template <> DFM_INLINE void ld8<float>(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
// 8 consecutive elements as raw 16-byte words (one for bf16, two for float): lets a kernel issue
// all of its loads before it unpacks and uses any of them.
template <typename T> struct Raw8 { uint4 w[sizeof(T) / 2]; };
template <typename T> DFM_INLINE Raw8<T> ldraw8(const T* p) {
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.w[i] = reinterpret_cast<const uint4*>(p)[i];
  return r;
}
DFM_INLINE void unpack8(const Raw8<bf16_t>& r, float* v) {
  const uint32_t w[4] = {r.w[0].x, r.w[0].y, r.w[0].z, r.w[0].w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
DFM_INLINE void unpack8(const Raw8<f16_t>& r, float* v) {
  const uint32_t w[4] = {r.w[0].x, r.w[0].y, r.w[0].z, r.w[0].w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = h2f((uint16_t)(w[i] & 0xffffu));
    v[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
  }
}
DFM_INLINE void unpack8(const Raw8<float>& r, float* v) {
  v[0] = __uint_as_float(r.w[0].x); v[1] = __uint_as_float(r.w[0].y);
  v[2] = __uint_as_float(r.w[0].z); v[3] = __uint_as_float(r.w[0].w);
  v[4] = __uint_as_float(r.w[1].x); v[5] = __uint_as_float(r.w[1].y);
  v[6] = __uint_as_float(r.w[1].z); v[7] = __uint_as_float(r.w[1].w);
}

template <typename T> DFM_INLINE void st8(T* p, const float* v);
template <> DFM_INLINE void st8<bf16_t>(bf16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
template <> DFM_INLINE void st8<f16_t>(f16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2h(v[2 * i]) | ((uint32_t)f2h(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
template <> DFM_INLINE void st8<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// ---- 16-bit storage types on MFMA: fragments travel as 8 x 16-bit bit patterns (bf16x8_t is
// only the container); mma16<T> issues v_mfma_f32_16x16x32_{bf16,f16} (fp32 accumulate).
template <typename T> struct H16;
template <> struct H16<bf16_t> { static constexpr unsigned ONE = 0x3f80u; };
template <> struct H16<f16_t> { static constexpr unsigned ONE = 0x3c00u; };
template <typename T> DFM_INLINE float4_t mma16(bf16x8_t a, bf16x8_t b, float4_t c);
template <> DFM_INLINE float4_t mma16<bf16_t>(bf16x8_t a, bf16x8_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <> DFM_INLINE float4_t mma16<f16_t>(bf16x8_t a, bf16x8_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0,
                                                0, 0);
}
template <typename T> DFM_INLINE uint16_t bits16(float v);
template <> DFM_INLINE uint16_t bits16<bf16_t>(float v) { return f2bf(v); }
template <> DFM_INLINE uint16_t bits16<f16_t>(float v) { return f2h(v); }
// 8 floats -> 8 x 16-bit fragment of T (round to nearest even)
template <typename T> DFM_INLINE bf16x8_t pack16x8(const float* v);
template <> DFM_INLINE bf16x8_t pack16x8<bf16_t>(const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  return __builtin_bit_cast(bf16x8_t, make_uint4(w[0], w[1], w[2], w[3]));
}
template <> DFM_INLINE bf16x8_t pack16x8<f16_t>(const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2h(v[2 * i]) | ((uint32_t)f2h(v[2 * i + 1]) << 16);
  return __builtin_bit_cast(bf16x8_t, make_uint4(w[0], w[1], w[2], w[3]));
}

// Dispatch a 16-bit-or-float32 body on the dtype code: F(T{}) with T = float, bf16_t or f16_t.
#define DFM_DTYPE_SWITCH(dtype, T, ...)                      \
  [&]() -> int {                                             \
    if ((dtype) == DFM_BF16) {                               \
      using T = bf16_t;                                      \
      return __VA_ARGS__;                                    \
    } else if ((dtype) == DFM_F16) {                         \
      using T = f16_t;                                       \
      return __VA_ARGS__;                                    \
    } else if ((dtype) == DFM_F32) {                         \
      using T = float;                                       \
      return __VA_ARGS__;                                    \
    }                                                        \
    dfm_set_error("%s: unsupported dtype %d", __func__, (int)(dtype)); \
    return DFM_ERR_DTYPE;                                    \
  }()

// ---- second stage of the deterministic two-stage column reductions:
// out[e] (+)= sum_{b < nblk} part[b * n + e], fixed summation order; 64 columns x 16 row-lanes
// per 1024-thread block so the nblk partials of a column are read by 16 lanes in parallel.
//   MODE 0: out0[e]                      MODE 1: e < n0 ? out0[e] : out1[e - n0]
//   MODE 2: depthwise layout, n0 = k*k+1: i = e % n0, c = e / n0 -> i < n0-1 ? out0[c*(n0-1)+i] : out1[c]
// one row-lane's share of a column: sum over b = rl, rl + 16, ... < nblk of part[b * n + e], in
// that order, with 8 loads in flight (the sums are short latency-bound chains)
DFM_INLINE float ps_lane_sum(const float* __restrict__ part, long n, long e, int nblk, int rl) {
  float s = 0.f;
  int b = rl;
  for (; b + 7 * 16 < nblk; b += 8 * 16) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = part[(long)(b + 16 * i) * n + e];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  if (b < nblk) {  // the tail: every load issued before the first add (clamped index, masked add),
    float v[8];    // the same order of additions
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = part[(long)min(b + 16 * i, nblk - 1) * n + e];
#pragma unroll
    for (int i = 0; i < 8; ++i) s = b + 16 * i < nblk ? s + v[i] : s;
  }
  return s;
}

template <int MODE>
__global__ __launch_bounds__(1024) void partial_sum_kernel(int nblk, long n, const float* __restrict__ part,
                                                           float* __restrict__ out0, float* __restrict__ out1, long n0,
                                                           int accumulate) {
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const long e = blockIdx.x * 64L + cl;
  const float s = e < n ? ps_lane_sum(part, n, e, nblk, rl) : 0.f;
  __shared__ float red[16][64];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && e < n) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += red[r][cl];
    float* dst;
    if (MODE == 0) dst = out0 + e;
    else if (MODE == 1) dst = e < n0 ? out0 + e : out1 + (e - n0);
    else {
      const long c = e / n0, i = e % n0;
      dst = i < n0 - 1 ? out0 + c * (n0 - 1) + i : (out1 ? out1 + c : nullptr);
    }
    if (dst) *dst = accumulate ? *dst + v : v;
  }
}

// ---- every kernel launch goes through DFM_LAUNCH: the launch tracer (runtime.cpp) can record
// which kernels an entry point enqueued and time chosen kernels with HIP events on their stream.
extern int dfm_trace_flags;
void dfm_trace_pre(const void* func, hipStream_t s);
void dfm_trace_post(const void* func, hipStream_t s);
#define DFM_LAUNCH(kern, grid, block, lds, stream, ...)                       \
  do {                                                                       \
    const int _dfm_tr = dfm_trace_flags;                                     \
    if (_dfm_tr) dfm_trace_pre((const void*)(kern), (hipStream_t)(stream));  \
    hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);         \
    if (_dfm_tr) dfm_trace_post((const void*)(kern), (hipStream_t)(stream)); \
  } while (0)

// ---- host-side error plumbing (thread-local last error string)
void dfm_set_error(const char* fmt, ...);
#define DFM_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      dfm_set_error(__VA_ARGS__);         \
      return DFM_ERR_ARG;                 \
    }                                     \
  } while (0)
#define DFM_LAUNCH_CHECK()                                                   \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) {                                                  \
      dfm_set_error("%s: launch failed: %s", __func__, hipGetErrorString(_e)); \
      return DFM_ERR_LAUNCH;                                                 \
    }                                                                        \
  } while (0)

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// The second stage of a parameter-gradient reduction: launched now (defer NULL) or described in
// *defer for the caller's grouped launch (dfm_partial_sum_group, elementwise.hip).
static inline int second_stage(int layout, int nblk, long n, const float* part, float* out0, float* out1, long n0,
                               int accumulate, DfmPartialSum* defer, hipStream_t s) {
  if (defer) {
    *defer = DfmPartialSum{part, out0, out1, n, n0, nblk, layout, accumulate};
    return DFM_OK;
  }
  const dim3 grid(cdiv(n, 64));
  if (layout == 0) DFM_LAUNCH(partial_sum_kernel<0>, grid, dim3(1024), 0, s, nblk, n, part, out0, out1, n0, accumulate);
  else if (layout == 1) DFM_LAUNCH(partial_sum_kernel<1>, grid, dim3(1024), 0, s, nblk, n, part, out0, out1, n0, accumulate);
  else DFM_LAUNCH(partial_sum_kernel<2>, grid, dim3(1024), 0, s, nblk, n, part, out0, out1, n0, accumulate);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}
