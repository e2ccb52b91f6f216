// Experiment harness (profiling tool, not part of libdformer_hip): the library's LDS-DMA ring GEMM
// (dformer_amd/csrc/gemm_impl.h) instantiated at several tile / ring-depth / occupancy points, so
// tools/gemm_variants.py can time every variant on every forward / input-gradient shape of the step
// and the library's routing can be fitted to measurements.
//   hipcc -O3 -fPIC -shared --offload-arch=gfx950 -I dformer_amd/csrc tools/gemm_variants/gemm_variants.hip \
//         -o tools/gemm_variants/libgemm_variants.so
#include "gemm_impl.h"

namespace {
template <int BM, int BN, int NW, int WM_, int NS, int MINB>
int run(GemmArgs& a, bool bk, hipStream_t s) {
  return glds_ak<bf16_t, BM, BN, NW, WM_, NS, MINB>(a, bk, s);
}
}  // namespace

extern "C" int gv_count() { return 9; }

extern "C" int gv_run(int v, const DfmGemmDesc* d, const void* A, const void* B, void* C, void* stream) {
  GemmArgs a;
  fill_args<bf16_t>(a, d, A, B, C, nullptr, 1);
  a.xcd_map = 1;
  if (!(d->a_kcontig && a.ala && a.alb && d->K >= 128)) return -2;  // the ring's domain
  const bool bk = d->b_kcontig;
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: return run<64, 64, 4, 2, 2, 4>(a, bk, s);    // the library's choice (round 3)
    case 1: return run<64, 64, 4, 2, 3, 3>(a, bk, s);
    case 2: return run<64, 64, 4, 2, 4, 2>(a, bk, s);
    case 3: return run<64, 128, 4, 2, 2, 3>(a, bk, s);
    case 4: return run<64, 128, 8, 2, 2, 2>(a, bk, s);
    case 5: return run<128, 64, 4, 2, 2, 3>(a, bk, s);
    case 6: return run<128, 128, 8, 2, 2, 2>(a, bk, s);
    case 7: return run<64, 256, 8, 2, 2, 1>(a, bk, s);
    case 8: return run<128, 128, 8, 2, 3, 1>(a, bk, s);
    default: return -1;
  }
}
