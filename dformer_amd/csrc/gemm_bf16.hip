// bf16 instantiations of the MFMA GEMM (gemm_impl.h), one translation unit per dtype.
#include "gemm_impl.h"

int dfm_gemm_bf16(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s) {
  return gemm_typed<bf16_t>(d, A, B, C, ws, s);
}

int dfm_gemm_group_bf16(int n, const DfmGemmDesc* d, const void* const* A, const void* const* B, void* const* C,
                       void* ws, hipStream_t s) {
  return gemm_group_typed<bf16_t>(n, d, A, B, C, ws, s);
}
