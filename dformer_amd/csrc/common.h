// Shared helpers for the DFormer gfx950 kernels: dtypes, bf16 packing, error reporting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dformer_hip.h"

typedef uint16_t bf16_t;  // raw bfloat16 bits
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
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
template <typename T> DFM_INLINE float ldf(const T* p) { return Num<T>::load(p); }
template <typename T> DFM_INLINE void stf(T* p, float v) { *p = Num<T>::from_f(v); }

DFM_INLINE float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
DFM_INLINE float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
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
