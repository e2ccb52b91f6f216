// f32 instantiations of the MFMA GEMM (gemm_impl.h), one translation unit per dtype.
#include "gemm_impl.h"

int dfm_gemm_f32(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s) {
  return gemm_typed<float>(d, A, B, C, ws, s);
}

int dfm_gemm_group_f32(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                       void* ws, hipStream_t s) {
  return gemm_group_typed<float>(n, d, A, B, C, ws, s);
}
