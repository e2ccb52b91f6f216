// MFMA GEMM for gfx950 with fused epilogues (DFormer linears / 1x1 convs / NMF bmm).
//
// One templated kernel covers the three layouts of a linear layer's forward and backward:
//   forward  Y  = X W^T   : A k-contiguous, B k-contiguous
//   dgrad    dX = dY W    : A k-contiguous, B row-contiguous   (ds_read_b64_tr_b16 for B)
//   wgrad    dW = dY^T X  : A row-contiguous, B row-contiguous (split-K over pixels)
// bf16 operands use v_mfma_f32_16x16x32_bf16 (fp32 accumulate); float32 operands use the
// exact-f32 v_mfma_f32_16x16x4_f32. Both operands are staged through a double-buffered LDS
// tile filled by 16-byte register-staged loads; row-contiguous bf16 tiles are consumed with
// the hardware transposing LDS read so no operand is ever transposed in memory.
#include "common.h"

namespace {

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  float* ws;
  int M, N, K, batch, splits;
  long lda, ldb, ldc, sa, sb, sc;
  float alpha, beta;
  int c_f32;
  const float* bias;
  int act;
  void* preact;
  long ldpre;
  const void* mul;
  long ldmul;
  const void* res;
  long ldres;
  const float* colscale;
  const float* rowscale;
  long rps;
  int act_col0;
};

template <typename T> struct Mf;
template <> struct Mf<bf16_t> {
  static constexpr int VEC = 8;    // elements per 16-byte vector
  static constexpr int KSTEP = 32; // k per MFMA
  static constexpr int BK = 64;
  static constexpr int PADK = 8;   // k-contiguous row pad (elements)
  static constexpr int PADR = 8;   // row-contiguous row pad (elements)
};
template <> struct Mf<float> {
  static constexpr int VEC = 4;
  static constexpr int KSTEP = 4;
  static constexpr int BK = 32;
  static constexpr int PADK = 1;
  static constexpr int PADR = 16;
};

// Load one 16-byte vector (VEC elements) of operand tile element (r, k..k+VEC) or (k, r..r+VEC)
// with zero fill outside [0, rows) x [0, K).
template <typename T, bool KC, bool ALIGNED>
DFM_INLINE uint4 load_vec(const T* __restrict__ p, long ld, int r, int k, int rows, int K) {
  constexpr int VEC = Mf<T>::VEC;
  uint4 out = make_uint4(0, 0, 0, 0);
  if (KC) {
    if (r >= rows) return out;
    const T* src = p + (long)r * ld + k;
    if (ALIGNED && k + VEC <= K) return *reinterpret_cast<const uint4*>(src);
    T tmp[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) tmp[e] = (k + e < K) ? src[e] : T(0);
    return *reinterpret_cast<uint4*>(tmp);
  } else {
    if (k >= K) return out;
    const T* src = p + (long)k * ld + r;
    if (ALIGNED && r + VEC <= rows) return *reinterpret_cast<const uint4*>(src);
    T tmp[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) tmp[e] = (r + e < rows) ? src[e] : T(0);
    return *reinterpret_cast<uint4*>(tmp);
  }
}

template <typename T, int R, bool KC>
struct TileGeom {
  static constexpr int BK = Mf<T>::BK;
  static constexpr int VEC = Mf<T>::VEC;
  // k-contiguous: [R][BK+PADK]; row-contiguous: [BK][R+PADR]
  static constexpr int LD = KC ? (BK + Mf<T>::PADK) : (R + Mf<T>::PADR);
  static constexpr int ELEMS = KC ? R * LD : BK * LD;
  static constexpr int NVEC = R * BK / VEC / 256;  // vectors per thread
  static_assert(NVEC >= 1, "tile too small");
};

template <typename T, int R, bool KC, bool ALIGNED>
DFM_INLINE void stage_load(uint4* regs, const T* __restrict__ base, long ld,
                           int r0, int k0, int rows, int K) {
  using G = TileGeom<T, R, KC>;
  constexpr int VEC = G::VEC, BK = G::BK;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    const int v = threadIdx.x + i * 256;
    if (KC) {
      const int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
      regs[i] = load_vec<T, true, ALIGNED>(base, ld, r0 + r, k0 + kc, rows, K);
    } else {
      const int k = v / (R / VEC), rc = (v % (R / VEC)) * VEC;
      regs[i] = load_vec<T, false, ALIGNED>(base, ld, r0 + rc, k0 + k, rows, K);
    }
  }
}

template <typename T, int R, bool KC>
DFM_INLINE void stage_store(const uint4* regs, T* lds) {
  using G = TileGeom<T, R, KC>;
  constexpr int VEC = G::VEC, BK = G::BK;
#pragma unroll
  for (int i = 0; i < G::NVEC; ++i) {
    const int v = threadIdx.x + i * 256;
    if (KC) {
      const int r = v / (BK / VEC), kc = (v % (BK / VEC)) * VEC;
      *reinterpret_cast<uint4*>(lds + r * G::LD + kc) = regs[i];
    } else {
      const int k = v / (R / VEC), rc = (v % (R / VEC)) * VEC;
      *reinterpret_cast<uint4*>(lds + k * G::LD + rc) = regs[i];
    }
  }
}

// ---- fragment reads
template <bool KC, int LD>
DFM_INLINE bf16x8_t frag_bf16(const bf16_t* lds, int r0, int k0, int lane) {
  if (KC) {
    const uint4 u = *reinterpret_cast<const uint4*>(lds + (r0 + (lane & 15)) * LD + k0 + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8_t, u);
  } else {
    const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
    typedef __attribute__((address_space(3))) short4_t lds_s4;
    const bf16_t* a0 = lds + (k0 + 8 * g + q) * LD + r0 + 4 * p;
    const bf16_t* a1 = a0 + 4 * LD;
    short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a0));
    short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(a1));
    typedef __attribute__((ext_vector_type(8))) short short8_t;
    short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, s);
  }
}
template <bool KC, int LD>
DFM_INLINE float frag_f32(const float* lds, int r0, int k0, int lane) {
  if (KC) return lds[(r0 + (lane & 15)) * LD + k0 + (lane >> 4)];
  return lds[(k0 + (lane >> 4)) * LD + r0 + (lane & 15)];
}

template <typename TO>
DFM_INLINE void epilogue_store(const GemmArgs& a, int b, int m, int n, float v) {
  if (a.beta != 0.0f) {
    if (a.c_f32) v += a.beta * ((const float*)a.C)[b * a.sc + (long)m * a.ldc + n];
    else v += a.beta * ldf((const TO*)a.C + b * a.sc + (long)m * a.ldc + n);
  }
  if (a.bias) v += a.bias[n];
  if (n >= a.act_col0) {
    if (a.preact) stf((TO*)a.preact + (long)m * a.ldpre + (n - a.act_col0), v);
    if (a.act == 1) v = gelu_f(v);
    else if (a.act == 2) v = fmaxf(v, 0.0f);
  }
  if (a.mul) v *= ldf((const TO*)a.mul + (long)m * a.ldmul + n);
  if (a.res) {
    float s = a.colscale ? a.colscale[n] : 1.0f;
    if (a.rowscale) s *= a.rowscale[m / a.rps];
    v = ldf((const TO*)a.res + (long)m * a.ldres + n) + s * v;
  }
  if (a.c_f32) ((float*)a.C)[b * a.sc + (long)m * a.ldc + n] = v;
  else stf((TO*)a.C + b * a.sc + (long)m * a.ldc + n, v);
}

template <typename T, int BM, int BN, int WAVES_M, bool AK, bool BKC, bool ALA, bool ALB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs a) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int BK = Mf<T>::BK, KSTEP = Mf<T>::KSTEP;
  using GA = TileGeom<T, BM, AK>;
  using GB = TileGeom<T, BN, BKC>;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* const lds_base = reinterpret_cast<T*>(smem);
#define LDS_A(i) (lds_base + (i) * GA::ELEMS)
#define LDS_B(i) (lds_base + 2 * GA::ELEMS + (i) * GB::ELEMS)

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int bm = blockIdx.x * BM, bn = blockIdx.y * BN;
  const int b = blockIdx.z / a.splits, split = blockIdx.z % a.splits;

  const int kper = ((a.K + a.splits - 1) / a.splits + BK - 1) / BK * BK;
  const int kbeg = split * kper;
  const int kend = min(a.K, kbeg + kper);

  const T* A = (const T*)a.A + (long)b * a.sa;
  const T* Bp = (const T*)a.B + (long)b * a.sb;

  float4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[GA::NVEC], rb[GB::NVEC];
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    stage_load<T, BM, AK, ALA>(ra, A, a.lda, bm, kbeg, a.M, kend);
    stage_load<T, BN, BKC, ALB>(rb, Bp, a.ldb, bn, kbeg, a.N, kend);
    stage_store<T, BM, AK>(ra, LDS_A(0));
    stage_store<T, BN, BKC>(rb, LDS_B(0));
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      stage_load<T, BM, AK, ALA>(ra, A, a.lda, bm, kbeg + (kt + 1) * BK, a.M, kend);
      stage_load<T, BN, BKC, ALB>(rb, Bp, a.ldb, bn, kbeg + (kt + 1) * BK, a.N, kend);
    }
    const T* la = LDS_A(cur);
    const T* lb = LDS_B(cur);
#pragma unroll
    for (int ks = 0; ks < BK; ks += KSTEP) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag_bf16<AK, GA::LD>((const bf16_t*)la, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag_bf16<BKC, GB::LD>((const bf16_t*)lb, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      } else {
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag_f32<AK, GA::LD>((const float*)la, wm * WM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag_f32<BKC, GB::LD>((const float*)lb, wn * WN + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      stage_store<T, BM, AK>(ra, LDS_A(cur ^ 1));
      stage_store<T, BN, BKC>(rb, LDS_B(cur ^ 1));
    }
    __syncthreads();
    cur ^= 1;
  }

#undef LDS_A
#undef LDS_B
  // C/D layout of 16x16 MFMA: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = bn + wn * WN + j * 16 + (lane & 15);
      if (n >= a.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        if (m >= a.M) continue;
        const float v = acc[i][j][r] * a.alpha;
        if (a.splits > 1) a.ws[(((long)split * a.batch + b) * a.M + m) * a.N + n] = v;
        else epilogue_store<T>(a, b, m, n, v);
      }
    }
}

template <typename T>
__global__ void splitk_reduce_kernel(GemmArgs a) {
  const long total = (long)a.batch * a.M * a.N;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < a.splits; ++s) v += a.ws[s * total + idx];
    const int n = idx % a.N;
    const long bm = idx / a.N;
    const int m = bm % a.M, b = bm / a.M;
    epilogue_store<T>(a, b, m, n, v);
  }
}

template <typename T, int BM, int BN, int WM_, bool AK, bool BKC>
int launch_cfg(GemmArgs& a, bool ala, bool alb, hipStream_t s) {
  using GA = TileGeom<T, BM, AK>;
  using GB = TileGeom<T, BN, BKC>;
  const size_t lds = (size_t)2 * (GA::ELEMS + GB::ELEMS) * sizeof(T);
  dim3 grid(cdiv(a.M, BM), cdiv(a.N, BN), a.batch * a.splits);
#define DFM_GEMM_GO(X, Y)                                                                         \
  do {                                                                                            \
    static bool attr_set = false;                                                                 \
    if (!attr_set) {                                                                              \
      (void)hipFuncSetAttribute((const void*)gemm_kernel<T, BM, BN, WM_, AK, BKC, X, Y>,                \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                \
      attr_set = true;                                                                            \
    }                                                                                             \
    hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM_, AK, BKC, X, Y>), grid, dim3(256), lds, s, a); \
  } while (0)
  if (ala && alb) DFM_GEMM_GO(true, true);
  else if (ala) DFM_GEMM_GO(true, false);
  else if (alb) DFM_GEMM_GO(false, true);
  else DFM_GEMM_GO(false, false);
#undef DFM_GEMM_GO
  DFM_LAUNCH_CHECK();
  if (a.splits > 1) {
    const long total = (long)a.batch * a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(min(cdiv(total, 256), 4096u)), dim3(256), 0, s, a);
    DFM_LAUNCH_CHECK();
  }
  return DFM_OK;
}

template <typename T, int BM, int BN, int WM_>
int launch_layout(GemmArgs& a, bool ak, bool bk, bool ala, bool alb, hipStream_t s) {
  if (ak && bk) return launch_cfg<T, BM, BN, WM_, true, true>(a, ala, alb, s);
  if (ak && !bk) return launch_cfg<T, BM, BN, WM_, true, false>(a, ala, alb, s);
  if (!ak && bk) return launch_cfg<T, BM, BN, WM_, false, true>(a, ala, alb, s);
  return launch_cfg<T, BM, BN, WM_, false, false>(a, ala, alb, s);
}

int choose_splits(const DfmGemmDesc* d, int BM, int BN) {
  if (d->split_k >= 1) return d->split_k;
  const long tiles = (long)cdiv(d->M, BM) * cdiv(d->N, BN) * d->batch;
  if (tiles >= 256 || d->K < 2048) return 1;
  int s = (int)((512 + tiles - 1) / tiles);
  s = min(s, d->K / 1024);
  return max(1, min(s, 64));
}

template <typename T>
void pick_tile(const DfmGemmDesc* d, int& BM, int& BN) {
  if (d->N <= 32) { BM = 128; BN = 32; }
  else if (d->N <= 64) { BM = 128; BN = 64; }
  else { BM = 128; BN = 128; }
}

template <typename T>
int gemm_typed(const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws, hipStream_t s) {
  constexpr int VEC = Mf<T>::VEC;
  GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.ws = (float*)ws;
  a.M = d->M; a.N = d->N; a.K = d->K; a.batch = d->batch > 0 ? d->batch : 1;
  a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
  a.sa = d->stride_a; a.sb = d->stride_b; a.sc = d->stride_c;
  a.alpha = d->alpha; a.beta = d->beta; a.c_f32 = d->c_f32;
  a.bias = d->bias; a.act = d->act; a.preact = d->preact; a.ldpre = d->ldpre;
  a.mul = d->mul; a.ldmul = d->ldmul; a.res = d->res; a.ldres = d->ldres;
  a.colscale = d->colscale; a.rowscale = d->rowscale; a.act_col0 = d->act_col0; a.rps = d->rows_per_scale > 0 ? d->rows_per_scale : 1;
  int BM, BN;
  pick_tile<T>(d, BM, BN);
  a.splits = choose_splits(d, BM, BN);
  if (a.splits > 1) DFM_CHECK_ARG(ws != nullptr, "dfm_gemm: split-K needs a workspace");
  const bool ala = (d->lda % VEC == 0) && ((uintptr_t)A % 16 == 0) && (a.batch == 1 || d->stride_a % VEC == 0);
  const bool alb = (d->ldb % VEC == 0) && ((uintptr_t)B % 16 == 0) && (a.batch == 1 || d->stride_b % VEC == 0);
  const bool ak = d->a_kcontig, bk = d->b_kcontig;
  if (BN == 32) return launch_layout<T, 128, 32, 4>(a, ak, bk, ala, alb, s);
  if (BN == 64) return launch_layout<T, 128, 64, 2>(a, ak, bk, ala, alb, s);
  return launch_layout<T, 128, 128, 2>(a, ak, bk, ala, alb, s);
}

}  // namespace

extern "C" size_t dfm_gemm_workspace_size(const DfmGemmDesc* d) {
  int BM = 128, BN = d->N <= 32 ? 32 : (d->N <= 64 ? 64 : 128);
  const int s = choose_splits(d, BM, BN);
  if (s <= 1) return 0;
  return (size_t)s * (d->batch > 0 ? d->batch : 1) * d->M * d->N * sizeof(float);
}

extern "C" int dfm_gemm(int dtype, const DfmGemmDesc* d, const void* A, const void* B, void* C, void* ws,
                        dfm_stream_t stream) {
  DFM_CHECK_ARG(d && A && B && C, "dfm_gemm: null argument");
  DFM_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "dfm_gemm: negative size");
  if (d->M == 0 || d->N == 0) return DFM_OK;
  DFM_CHECK_ARG(d->a_kcontig ? d->lda >= d->K : d->lda >= d->M, "dfm_gemm: lda too small");
  DFM_CHECK_ARG(d->b_kcontig ? d->ldb >= d->K : d->ldb >= d->N, "dfm_gemm: ldb too small");
  DFM_CHECK_ARG(d->ldc >= d->N, "dfm_gemm: ldc too small");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DFM_BF16) return gemm_typed<bf16_t>(d, A, B, C, ws, s);
  if (dtype == DFM_F32) return gemm_typed<float>(d, A, B, C, ws, s);
  dfm_set_error("dfm_gemm: unsupported dtype %d", dtype);
  return DFM_ERR_DTYPE;
}
