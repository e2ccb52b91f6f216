// Short-K GEMM for tall operands (K <= 128, k-contiguous A, thousands of row tiles): the stage-0/1
// ConvFFN fc1 forward (M = 307,200 / 76,800 rows, K = C = 64 / 128, N = hidden = 512 / 1024), its fc2
// input gradient times GELU' (K = C, N = hidden) and the other short-K linears of those stages.
// Included by gemm_impl.h.
//
// These GEMMs do almost no arithmetic per byte: they are bound by writing (and, for the input
// gradient, reading the GELU' multiplier of) an M x N tensor of hundreds of MB. A block keeps the
// W slice of its 128 output columns in LDS for its whole life and walks row steps of 64 (16 rows per
// wave); every wave loads its A fragments straight from global memory (16 bytes per lane, the next
// step's in flight while this one multiplies), multiplies the W slice (MFMA A operand) by them, so
// a lane holds 4 consecutive output columns of one row, and writes the output through a wave-private
// LDS staging tile as whole 128-byte lines (16 bytes per lane, two 256-byte rows per instruction).
// The epilogue's tile operand (GELU' multiplier, residual or C) comes in the same way in reverse:
// coalesced 16-byte rows into a second staging tile, read back in the accumulator layout. No block
// barrier after the W slice is staged; the wave-private staging tiles only need the wave's own
// LDS ordering (an explicit lgkmcnt(0) wait + compiler fence between write and read-back).
#pragma once

constexpr int WIDE_NSL = 128;  // output columns per block
constexpr int WIDE_MS = 64;    // rows per block step (16 per wave)
constexpr int WIDE_D = 3;      // row steps of operands in flight per wave

template <int KD>
struct WideCfg {
  static constexpr int WP = KD + 8;                        // W image pitch (elements): conflict-free b128 fragments
  static constexpr int W_BYTES = WIDE_NSL * WP * 2;
  static constexpr int SP = WIDE_NSL + 8;                  // staging pitch (elements)
  static constexpr int S_BYTES = 16 * SP * 2;              // one wave's 16 x 128 tile
  static constexpr int LDS = W_BYTES + 4 * S_BYTES + 2 * WIDE_NSL * 4;
};

DFM_INLINE void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// 4 consecutive 16-bit elements (8 bytes) from floats
template <typename T> DFM_INLINE void wide_st4(T* p, const float* v) {
  const uint32_t w0 = (uint32_t)bits16<T>(v[0]) | ((uint32_t)bits16<T>(v[1]) << 16);
  const uint32_t w1 = (uint32_t)bits16<T>(v[2]) | ((uint32_t)bits16<T>(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(w0, w1);
}

// ekind: 0 none, 1 multiplier (GELU' of it with mul_gelu_grad), 2 residual (+ colscale * rowscale *
// branch), 3 beta * C. ep / lde: that operand.
template <typename T, int KD, bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_wide_kernel(GemmArgs a, const T* __restrict__ ep, long lde, int ekind,
                                                           int msteps) {
  using CF = WideCfg<KD>;
  constexpr int KS = KD / 32;             // MFMA k-steps of 32
  constexpr int NT = WIDE_NSL / 16;       // 16-column tiles per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* wimg = reinterpret_cast<bf16_t*>(smem);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // one staging tile per wave serves the operand coming in and the output going out: a lane reads
  // its operand piece and then writes its output piece at the same address
  T* stg = reinterpret_cast<T*>(smem + CF::W_BYTES + wid * CF::S_BYTES);
  float* vb = reinterpret_cast<float*>(smem + CF::W_BYTES + 4 * CF::S_BYTES);
  float* vc = vb + WIDE_NSL;

  const int lid = xcd_lid(blockIdx.x, gridDim.x);
  const int cn = lid % a.tiles_n, r0 = lid / a.tiles_n, R = gridDim.x / a.tiles_n;
  const int n0 = cn * WIDE_NSL;
  const T* Bp = (const T*)a.B;

  // ---- the block's W slice -> LDS as [n][k] (zero rows past N), bias / column scale
  // (K < KD, a multiple of 16: the image's columns / rows k >= K are zero, and so are the A fragments there)
  if constexpr (BKC) {  // W[n][k]: 16-byte k-vectors
    for (int e = threadIdx.x; e < WIDE_NSL * (KD / 8); e += 256) {
      const int nl = e / (KD / 8), kc = (e % (KD / 8)) * 8;
      const int n = n0 + nl;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < a.N && kc < a.K) v = *reinterpret_cast<const uint4*>(Bp + (long)n * a.ldb + kc);
      *reinterpret_cast<uint4*>(wimg + nl * CF::WP + kc) = v;
    }
  } else {  // W[k][n]: 16-byte n-vectors transposed into the [n][k] image
    for (int e = threadIdx.x; e < KD * (WIDE_NSL / 8); e += 256) {
      const int k = e / (WIDE_NSL / 8), nl = (e % (WIDE_NSL / 8)) * 8;
      const int n = n0 + nl;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < a.N && k < a.K) v = *reinterpret_cast<const uint4*>(Bp + (long)k * a.ldb + n);
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int i = 0; i < 8; ++i) reinterpret_cast<uint16_t*>(wimg)[(nl + i) * CF::WP + k] = h[i];
    }
  }
  for (int e = threadIdx.x; e < WIDE_NSL; e += 256) {
    const int n = n0 + e;
    vb[e] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
    vc[e] = (a.colscale && n < a.N) ? a.colscale[n] : 1.f;
  }
  __syncthreads();

  const T* A = (const T*)a.A;
  auto load_a = [&](int ms, bf16x8_t* af) {
    const int row = min(ms * WIDE_MS + wid * 16 + (lane & 15), a.M - 1);
    const T* p = A + (long)row * a.lda + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s < KS - 1 || a.K == KD) {
        af[s] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p + 32 * s));
      } else {  // the padded last k-step: lanes past K load their row's first vector and zero it
        const bool kin = 32 * s + 8 * (lane >> 4) < a.K;
        const uint4 v = *reinterpret_cast<const uint4*>(p + (kin ? 32 * s : 0));
        af[s] = __builtin_bit_cast(bf16x8_t, kin ? v : make_uint4(0, 0, 0, 0));
      }
    }
  };
  auto load_e = [&](int ms, uint4* ev) {  // epilogue operand rows, coalesced 16-byte chunks
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = i * 64 + lane, rr = q >> 4, c = (q & 15) * 8;
      const int m = ms * WIDE_MS + wid * 16 + rr, n = n0 + c;
      ev[i] = (m < a.M && n < a.N) ? *reinterpret_cast<const uint4*>(ep + (long)m * lde + n) : make_uint4(0, 0, 0, 0);
    }
  };

  // D row steps of operands in flight per wave (registers): a step's MFMAs and epilogue take far
  // less than one HBM round trip, so one step of look-ahead leaves the wave waiting on every load
  bf16x8_t af[WIDE_D][KS];
  uint4 ev[WIDE_D][4];
#pragma unroll
  for (int d = 0; d < WIDE_D; ++d) {
    const int ms = r0 + d * R;
    if (ms < msteps) {
      load_a(ms, af[d]);
      if (ekind) load_e(ms, ev[d]);
    }
  }
  for (int base = r0; base < msteps; base += WIDE_D * R) {
#pragma unroll
    for (int d = 0; d < WIDE_D; ++d) {
      const int ms = base + d * R;
      if (ms >= msteps) break;
      const int mw = ms * WIDE_MS + wid * 16;  // this wave's first row
      float4_t acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const bf16x8_t wf = __builtin_bit_cast(
              bf16x8_t, *reinterpret_cast<const uint4*>(wimg + (t * 16 + (lane & 15)) * CF::WP + 32 * s + 8 * (lane >> 4)));
          acc[t] = mma16<T>(wf, af[d][s], acc[t]);  // W as the A operand: lane holds 4 columns of one row
        }
      }
      if (ekind) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = i * 64 + lane, rr = q >> 4, c = (q & 15) * 8;
          *reinterpret_cast<uint4*>(stg + rr * CF::SP + c) = ev[d][i];
        }
        wave_lds_fence();
      }
      const int nx = ms + WIDE_D * R;  // refill this slot: D steps ahead
      if (nx < msteps) load_a(nx, af[d]);
      const int ml = lane & 15, m = mw + ml;
      const float rsv = (a.rowscale && m < a.M) ? a.rowscale[m / a.rps] : 1.0f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int nl = t * 16 + 4 * (lane >> 4), n = n0 + nl;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[t][r] * a.alpha;
        float e4[4] = {0.f, 0.f, 0.f, 0.f};
        if (ekind) {
          const uint2 u = *reinterpret_cast<const uint2*>(stg + ml * CF::SP + nl);
          const T* h = reinterpret_cast<const T*>(&u);
#pragma unroll
          for (int r = 0; r < 4; ++r) e4[r] = Num<T>::to_f(h[r]);
        }
        if (ekind == 3) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += a.beta * e4[r];
        }
        const float4 bv = *reinterpret_cast<const float4*>(vb + nl);
        v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
        if (n >= a.act_col0) {
          if (a.act == 3) {
            float dv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float cdf, pdf;
              normal_cdf_pdf(v[r], cdf, pdf);
              dv[r] = fmaf(v[r], pdf, cdf);
              v[r] *= cdf;
            }
            if (a.preact && m < a.M && n < a.N) wide_st4<T>((T*)a.preact + (long)m * a.ldpre + (n - a.act_col0), dv);
          } else {
            if (a.preact && m < a.M && n < a.N) wide_st4<T>((T*)a.preact + (long)m * a.ldpre + (n - a.act_col0), v);
            if (a.act == 1) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
            } else if (a.act == 2) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.0f);
            }
          }
        }
        if (ekind == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= a.mul_gelu_grad ? gelu_grad_f(e4[r]) : e4[r];
        } else if (ekind == 2) {
          const float4 cv = *reinterpret_cast<const float4*>(vc + nl);
          v[0] = e4[0] + cv.x * rsv * v[0];
          v[1] = e4[1] + cv.y * rsv * v[1];
          v[2] = e4[2] + cv.z * rsv * v[2];
          v[3] = e4[3] + cv.w * rsv * v[3];
        }
        wide_st4<T>(stg + ml * CF::SP + nl, v);  // the operand piece read above, same lane and address
      }
      if (ekind && nx < msteps) load_e(nx, ev[d]);
      wave_lds_fence();
      // staged output rows -> global, two 256-byte rows per instruction
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = i * 64 + lane, rr = q >> 4, c = (q & 15) * 8;
        const int mm = mw + rr, n = n0 + c;
        const uint4 o = *reinterpret_cast<const uint4*>(stg + rr * CF::SP + c);
        if (mm < a.M && n < a.N) *reinterpret_cast<uint4*>((T*)a.C + (long)mm * a.ldc + n) = o;
      }
      wave_lds_fence();  // the next step's operand staging overwrites this tile
    }
  }
}

template <typename T>
bool wide_eligible(const GemmArgs& a, const DfmGemmDesc* d) {
  if (sizeof(T) != 2) return false;
  if (!d->a_kcontig || a.splits != 1 || a.batch != 1 || d->colsum || d->c_f32 || d->out2 || !a.ala || !a.alb ||
      !a.vec_ok)
    return false;
  // K a multiple of 16 (48 / 80 / 112: DFormer-Large's stage-0 depth branch, C = 48) padded to the next 32
  if (d->K % 16 != 0 || d->K > 128 || d->K < 32 || d->N % 8 != 0 || d->M < 65536 || d->N < 144) return false;
  const int tiles = (d->mul != nullptr) + (d->res != nullptr) + (d->beta != 0.0f);
  if (tiles > 1) return false;
  if (d->mul && d->ldmul % 8 != 0) return false;
  if (d->res && d->ldres % 8 != 0) return false;
  return true;
}

template <typename T, int KD, bool BKC>
int wide_launch_cfg(GemmArgs& a, const DfmGemmDesc* d, hipStream_t s) {
  using CF = WideCfg<KD>;
  auto kern = gemm_wide_kernel<T, KD, BKC>;
  static int per_cu = -1;
  if (per_cu < 0) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kern, 256, CF::LDS) != hipSuccess || n < 1) n = 1;
    per_cu = n;
  }
  a.tiles_n = cdiv(a.N, WIDE_NSL);
  const int msteps = cdiv(a.M, WIDE_MS);
  const int R = std::max(1, std::min(msteps, 256 * per_cu / a.tiles_n));
  int ekind = 0;
  const void* ep = nullptr;
  long lde = 0;
  if (d->mul) { ekind = 1; ep = d->mul; lde = d->ldmul; }
  else if (d->res) { ekind = 2; ep = d->res; lde = d->ldres; }
  else if (d->beta != 0.0f) { ekind = 3; ep = a.C; lde = d->ldc; }
  DFM_LAUNCH(kern, dim3((unsigned)(R * a.tiles_n)), dim3(256), CF::LDS, s, a, (const T*)ep, lde, ekind, msteps);
  DFM_LAUNCH_CHECK();
  return DFM_OK;
}

template <typename T, bool BKC>
int wide_launch_k(GemmArgs& a, const DfmGemmDesc* d, hipStream_t s) {
  switch ((d->K + 31) / 32) {
    case 1: return wide_launch_cfg<T, 32, BKC>(a, d, s);
    case 2: return wide_launch_cfg<T, 64, BKC>(a, d, s);
    case 3: return wide_launch_cfg<T, 96, BKC>(a, d, s);
    default: return wide_launch_cfg<T, 128, BKC>(a, d, s);
  }
}

template <typename T>
int wide_launch(GemmArgs& a, const DfmGemmDesc* d, hipStream_t s) {
  return d->b_kcontig ? wide_launch_k<T, true>(a, d, s) : wide_launch_k<T, false>(a, d, s);
}
