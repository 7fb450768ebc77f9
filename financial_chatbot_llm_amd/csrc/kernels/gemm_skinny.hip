// Decode-time projection GEMMs (K3/K8/K9/K10/K11 at M <= 64 tokens): Y[M,N] = X[M,K] . W[N,K]^T.
//
// At decode batch sizes the op is a weight stream (W: 33-235 MB per projection, X: <= 512 KB and
// L2-resident), so the kernel is built around keeping HBM busy, not around MFMA throughput:
//   * each workgroup owns a 16*NTF-row slice of W and splits K over its NW waves (in-workgroup
//     split-K), so even N = 4096 launches >= 256 workgroups with no cross-workgroup reduction;
//   * W fragments stream straight into VGPRs (no LDS hop -- each byte is used once), U k-steps of
//     loads in flight per wave; X fragments come from L2;
//   * v_mfma_f32_16x16x32_bf16 computes Y^T tiles (W rows on the MFMA "row" side, tokens on the
//     16 columns), f32 accumulation; the NW partial tiles are summed through LDS and the
//     workgroup writes bf16 with 16-byte stores;
//   * fused epilogues: EPI_SILU -- W's gate/up rows are interleaved in 16-row groups
//     (gate 16i..16i+15 then up 16i..16i+15), so a workgroup holds matching gate/up rows and
//     writes silu(gate) * up directly ([M, F] output, no [M, 2F] round trip);
//     EPI_RESID -- adds a residual tensor (o/down projections) in the same pass.
#include "common.h"

#define EPI_NONE 0
#define EPI_SILU 1
#define EPI_RESID 2

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

union F8 {
  uint4 u;
  u32x4 n;
  bf16x8 v;
};

template <int MT, int NTF, int NW, int U, int EPI>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_kernel(const bf16* __restrict__ X, int ldx,
                                                              const bf16* __restrict__ W, int K,
                                                              bf16* __restrict__ Y, int ldy,
                                                              const bf16* __restrict__ R, int ldr, int M, int N) {
  constexpr int NR = 16 * NTF;  // W rows per workgroup
  constexpr int MC = 16 * MT;   // token columns
  extern __shared__ __attribute__((aligned(16))) float red[];  // [NW][NR][MC]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;
  const int n0 = blockIdx.x * NR;
  const int kper = K / NW;
  const int kb = w * kper;

  f32x4 acc[NTF][MT];
#pragma unroll
  for (int f = 0; f < NTF; ++f)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // W is pre-tiled (ops/gemm.py tile_weight): fragment (row group rg, k-step ks) is the 1 KiB at
  // ((rg*(K/32) + ks)*64 + lane)*16 B, so every wave-instruction reads 1 KiB contiguous and a
  // wave's consecutive k-steps are consecutive KiBs -- long sequential HBM bursts.
  const int ksteps = K / 32;
  const bf16* wrow[NTF];
#pragma unroll
  for (int f = 0; f < NTF; ++f) wrow[f] = W + ((long)(n0 / 16 + f) * ksteps + kb / 32) * 512 + lane * 8;
  const bf16* xrow[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int r = min(16 * m + col, M - 1);
    xrow[m] = X + (long)r * ldx + kb + 8 * g;
  }

  // Modulo-scheduled ring of DEPTH k-steps: step s's W and X fragments are issued DEPTH steps
  // before their MFMAs, into ring slot s % DEPTH (static after unrolling).  X is prefetched
  // together with W on purpose: vmcnt retires loads in issue order, so a late X load would make
  // every MFMA wait for all younger W prefetches too.
  constexpr int DEPTH = 4;
  const int nsteps = kper / 32;
  F8 wr[DEPTH][NTF], xr[DEPTH][MT];
  auto issue = [&](int slot_unused, int s, F8* wv, F8* xv) {
#pragma unroll
    for (int f = 0; f < NTF; ++f)
      wv[f].n = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow[f] + 512 * s));
#pragma unroll
    for (int m = 0; m < MT; ++m) xv[m].u = *reinterpret_cast<const uint4*>(xrow[m] + 32 * s);
  };
  auto mma = [&](const F8* wv, const F8* xv) {
#pragma unroll
    for (int f = 0; f < NTF; ++f)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[f][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[f].v, xv[m].v, acc[f][m], 0, 0, 0);
  };
  // nsteps is a multiple of DEPTH (host check), so the steady-state body is branch-free and the
  // waitcnt pass can leave the younger ring slots in flight (counted vmcnt, not vmcnt(0)).
#pragma unroll
  for (int j = 0; j < DEPTH; ++j) issue(j, j, wr[j], xr[j]);
  for (int base = 0; base < nsteps - DEPTH; base += DEPTH) {
#pragma unroll
    for (int j = 0; j < DEPTH; ++j) {
      mma(wr[j], xr[j]);
      issue(j, base + j + DEPTH, wr[j], xr[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < DEPTH; ++j) mma(wr[j], xr[j]);

  // partial tiles -> LDS: lane holds rows n = 16f + 4g + r, column m = 16mt + col
  float* mine = red + w * NR * MC;
#pragma unroll
  for (int f = 0; f < NTF; ++f)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) mine[(16 * f + 4 * g + r) * MC + 16 * m + col] = acc[f][m][r];
  __syncthreads();

  // reduce over waves + epilogue: each thread produces 8 consecutive outputs of one token row
  constexpr int OUTN = (EPI == EPI_SILU) ? NR / 2 : NR;
  for (int idx = threadIdx.x; idx < MC * (OUTN / 8); idx += NW * 64) {
    const int m = idx / (OUTN / 8);
    const int c8 = (idx % (OUTN / 8)) * 8;
    if (m >= M) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (EPI == EPI_SILU) {
        // output column c = 16*pair + jj -> gate row 32*pair + jj, up row 32*pair + 16 + jj
        const int c = c8 + j, pair = c >> 4, jj = c & 15;
        float gsum = 0.f, usum = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) {
          gsum += red[(ww * NR + 32 * pair + jj) * MC + m];
          usum += red[(ww * NR + 32 * pair + 16 + jj) * MC + m];
        }
        const float gb = (float)(bf16)gsum, ub = (float)(bf16)usum;  // match the unfused bf16 path
        o[j] = (float)(bf16)(gb / (1.f + __expf(-gb))) * ub;
      } else {
        float s = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) s += red[(ww * NR + c8 + j) * MC + m];
        o[j] = s;
      }
    }
    if (EPI == EPI_RESID) {
      float rr[8];
      unpack8(*reinterpret_cast<const uint4*>(R + (long)m * ldr + n0 + c8), rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (float)(bf16)o[j] + rr[j];
    }
    const int ncol = (EPI == EPI_SILU) ? (n0 / 2 + c8) : (n0 + c8);
    *reinterpret_cast<uint4*>(Y + (long)m * ldy + ncol) = pack8(o);
  }
}

template <int MT, int EPI>
static int launch_mt(const void* X, int ldx, const void* W, int K, void* Y, int ldy, const void* R, int ldr, int M,
                     int N, int ntf, int nw, hipStream_t s) {
#define LAUNCH_CFG(NTF_, NW_)                                                                                  \
  if (ntf == NTF_ && nw == NW_) {                                                                              \
    constexpr int U = 4; /* K granularity: ring depth x 32-wide k-steps per wave */                    \
    if (N % (16 * NTF_) || K % (NW_ * 32 * U)) return (int)hipErrorInvalidValue;                               \
    const size_t lds = (size_t)NW_ * 16 * NTF_ * 16 * MT * sizeof(float);                                     \
    hipLaunchKernelGGL((skinny_gemm_kernel<MT, NTF_, NW_, U, EPI>), dim3(N / (16 * NTF_)), dim3(NW_ * 64), lds, \
                       s, (const bf16*)X, ldx, (const bf16*)W, K, (bf16*)Y, ldy, (const bf16*)R, ldr, M, N);    \
    return (int)hipGetLastError();                                                                             \
  }
  LAUNCH_CFG(2, 4)
  LAUNCH_CFG(2, 8)
  LAUNCH_CFG(4, 4)
  LAUNCH_CFG(1, 8)
  LAUNCH_CFG(1, 4)
#undef LAUNCH_CFG
  return (int)hipErrorInvalidValue;
}

// epi: 0 none, 1 silu (W gate/up interleaved by 16 rows; Y is [M, N/2]), 2 residual add (R [M, N])
PENNY_API int penny_skinny_gemm(const void* X, int ldx, const void* W, int K, void* Y, int ldy, const void* R, int ldr,
                                int M, int N, int epi, int ntf, int nw, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || (epi == EPI_SILU && ntf % 2)) return (int)hipErrorInvalidValue;
  const int mt = (M + 15) / 16;
#define BY_EPI(MT_)                                                                                           \
  switch (epi) {                                                                                              \
    case EPI_NONE: return launch_mt<MT_, EPI_NONE>(X, ldx, W, K, Y, ldy, R, ldr, M, N, ntf, nw, stream);      \
    case EPI_SILU: return launch_mt<MT_, EPI_SILU>(X, ldx, W, K, Y, ldy, R, ldr, M, N, ntf, nw, stream);      \
    case EPI_RESID: return launch_mt<MT_, EPI_RESID>(X, ldx, W, K, Y, ldy, R, ldr, M, N, ntf, nw, stream);    \
    default: return (int)hipErrorInvalidValue;                                                               \
  }
  switch (mt) {
    case 1: BY_EPI(1)
    case 2: BY_EPI(2)
    case 3: BY_EPI(3)
    default: BY_EPI(4)
  }
#undef BY_EPI
}
