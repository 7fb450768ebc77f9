// Narrow-shard / small-M prefill projection GEMM (K3 QKV, K8 O, K9 gate|up, K10 down of the
// Llama-3-70B TP=8 per-rank shards):
//   Y[m, n] = sum_k X[m, k] * W[n, k]          X [M, K] bf16 (row stride ldx), W [N, K] bf16
//
// Why a second tile kernel: the 256 x 256 tile of gemm_prefill.hip runs these shapes at 5-32
// column tiles (N = 1280-8192) and 2-6 row tiles at the serving scheduler's 384-1536-row steps --
// 10-190 tiles for 256 CUs -- and its wave-quantisation tail pays a 256 KB f32 partial per split.
// Here a 128 x 128 tile (4x the tiles) with the K dimension split over the grid (S slices, f32
// slabs the consumer reduces: RoPE/KV write, add+RMSNorm, or penny_splitk_reduce{,_silu}) fills
// the chip at those sizes.
//
// Structure (gfx950): 256 threads = 4 waves as 2 (W rows) x 2 (tokens), each wave a 64 x 64
// (n x token) sub-tile of 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators (MFMA A = W: a lane's 4
// accumulator registers are 4 consecutive output columns, as in gemm_prefill.hip).  Both operands
// are staged by LDS-DMA (global_load_lds_dwordx4, 1-KiB lane-linear pieces) with an XOR chunk
// swizzle on the source address and on the fragment read (conflict-free ds_read_b128 phases), in a
// ring of stages (mid_variant below): one wait + barrier per stage, the next stages' DMA in flight
// while the current one is on the MFMAs, and LDS sized so two or three workgroups share a CU and
// one's MFMAs cover the others' barriers.  Workgroup ids are remapped bijectively over the 8 XCDs with
// the token tile fastest: an XCD's concurrent workgroups share W panels in its L2.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int MT = 128;                 // token rows per tile
constexpr int NT_ = 128;                // W rows (output columns) per tile
enum { MEPI_BF16 = 0, MEPI_SILU = 1, MEPI_SLAB = 2, MEPI_RESID = 3 };

union Frag {
  uint4 u;
  bf16x8 v;
};
union Pack8 {
  uint4 u;
  bf16 e[8];
};

// lo = columns 16f + 4g .. +3 and hi = 16(f+1) + 4g .. +3 of lane row g -> 8 consecutive columns
// 8*(g>>1) + 16*(g&1) .. +7 of this lane (v_permlane16_swap: one 16-B store instead of two 8-B ones)
__device__ __forceinline__ uint4 pair16(bf16x4 lo, bf16x4 hi) {
  union {
    bf16x4 v;
    uint2 u;
  } a, b;
  a.v = lo;
  b.v = hi;
  const auto x = __builtin_amdgcn_permlane16_swap(a.u.x, b.u.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.u.y, b.u.y, false, false);
  return make_uint4(x[0], y[0], x[1], y[1]);
}

// Staging geometry: RB bytes of K per row per stage (128: BK = 64, two MFMA k-steps; 64: BK = 32, one
// k-step), NST stages in the LDS ring (NST = 2: one vmcnt(0) + barrier per stage; NST >= 3: the
// counted wait of prefill2 -- stage t+NST-1 streams in while stage t is on the MFMAs).
// Chunk swizzles, conflict-free over the four 16-lane phases of the fragment ds_read_b128 (lanes of
// a phase read rows l & 15 at chunk 4kk + (l >> 4)): 128-B rows (2 per bank row) chunk ^ ((r >> 1) & 7)
// as gemm_prefill.hip; 64-B rows (4 per bank row) chunk ^ {0, 2, 3, 1}[(r >> 2) & 3] (checked by hand
// over the phases: the four rows r = a + 4i of a phase land on distinct 16-B slots).
template <int RB>
__device__ __forceinline__ int mswz(int r) { return RB == 128 ? (r >> 1) & 7 : (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int N_>
__device__ __forceinline__ void mid_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N_) : "memory");
}

template <int EPI, int RB, int NST>
__global__ void __launch_bounds__(256, (NST * 2 * 128 * RB <= 49152) ? 3 : (NST * 2 * 128 * RB <= 65536 ? 2 : 1))
gemm_mid_kernel(const bf16* __restrict__ X, int ldx, const bf16* __restrict__ W, int K, void* __restrict__ Y, int ldy,
                const bf16* __restrict__ R, int ldr, int M, int N, int S) {
  constexpr int OPB = 128 * RB;            // one operand's stage image
  constexpr int STG = 2 * OPB;             // W image, then X image
  constexpr int CPR = RB / 16;             // 16-B chunks per row
  constexpr int RPP = 1024 / RB;           // rows per 1-KiB DMA piece
  constexpr int PPW = 128 / RPP / 4;       // pieces per operand per wave
  constexpr int LPS = 2 * PPW;             // DMA instructions per wave per stage
  constexpr int KS = RB / 64;              // MFMA k-steps per stage
  constexpr int BKE = RB / 2;              // K elements per stage
  __shared__ __attribute__((aligned(1024))) char smem[NST * STG];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wa = w >> 1, wb = w & 1;     // wave grid 2 (W rows) x 2 (tokens)
  const int g = lane >> 4, col = lane & 15;

  // ---- workgroup -> (slice, column tile, token tile): bijective XCD remap, token tile fastest ----
  const int Mt = (M + MT - 1) / MT, Nt = N / NT_, nwg = Mt * Nt * S;
  int id = blockIdx.x;
  {
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int tm = id % Mt, rest = id / Mt, tn = rest % Nt, s = rest / Nt;
  const int m0 = tm * MT, n0 = tn * NT_;
  const int kc = K / S, k0 = s * kc, nt = kc / BKE;
  PENNY_DASSERT(N % NT_ == 0 && K % (64 * S) == 0 && nt >= 1 && s < S);

  // ---- LDS-DMA sources: wave w owns pieces w*PPW .. of the W image and of the X image ----
  // piece p = image rows RPP*p ..; lane l -> row RPP*p + l / CPR, LDS slot l % CPR = logical chunk
  // (l % CPR) ^ mswz(row) of the row's RB-byte K slice
  const char* src[2 * PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int r = RPP * (w * PPW + i) + lane / CPR;
    const int c = (lane % CPR) ^ mswz<RB>(r);
    src[i] = reinterpret_cast<const char*>(W + (long)(n0 + r) * K + k0) + 16 * c;
    const int m = min(m0 + r, M - 1);
    src[PPW + i] = reinterpret_cast<const char*>(X + (long)m * ldx + k0) + 16 * c;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  // inline-asm DMA: invisible to hipcc's waitcnt pass, so the fragment ds_reads of the current
  // stage are not held behind a vmcnt(0) for the next stages' DMA (the explicit waits are the only
  // ones); M0 is set and restored inside the statement
  auto stage = [&](int t) {
    const unsigned buf = lds0 + (t % NST) * STG;
#pragma unroll
    for (int i = 0; i < 2 * PPW; ++i) {
      const unsigned dst = buf + (i < PPW ? 0 : OPB) + RPP * (w * PPW + (i % PPW)) * RB;
      const char* gp = src[i] + (long)t * RB;
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(gp), "s"(dst)
                   : "memory");
    }
  };

  // fragment chunk offsets of this lane's row (lane & 15): k-step kk reads logical chunk 4kk + g
  const int rowoff = col * RB;
  int choff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) choff[kk] = ((4 * kk + g) ^ mswz<RB>(col)) << 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nt) stage(t);
  for (int t = 0; t < nt; ++t) {
    // this wave's pieces of stage t landed (younger stages may stay in flight), then publish it; the
    // barrier also retires every wave's reads of the buffer restaged next (read at t - 1)
    if (NST >= 3 && t + NST - 2 < nt) mid_wait_barrier<(NST >= 3 ? (NST - 2) * LPS : 0)>();
    else mid_wait_barrier<0>();
    if (t + NST - 1 < nt) stage(t + NST - 1);
    const char* wi = smem + (t % NST) * STG + (wa * 64) * RB + rowoff;
    const char* xi = smem + (t % NST) * STG + OPB + (wb * 64) * RB + rowoff;
    Frag a[4][KS], b[4][KS];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        a[f][kk].u = *reinterpret_cast<const uint4*>(wi + f * 16 * RB + choff[kk]);
        b[f][kk].u = *reinterpret_cast<const uint4*>(xi + f * 16 * RB + choff[kk]);
      }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[f][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f][kk].v, b[u][kk].v, acc[f][u], 0, 0, 0);
  }

  // ---- epilogue: lane holds Y[m0 + wb*64 + 16u + col][n0 + wa*64 + 16f + 4g + r], r = 0..3 ----
  const int lane_off = 8 * (g >> 1) + 16 * (g & 1);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int m = m0 + wb * 64 + u * 16 + col;
    if (m >= M) continue;
    if constexpr (EPI == MEPI_SLAB) {
      float* P = static_cast<float*>(Y) + ((long)s * M + m) * N + n0 + wa * 64 + 4 * g;
#pragma unroll
      for (int f = 0; f < 4; ++f) *reinterpret_cast<f32x4*>(P + 16 * f) = acc[f][u];
    } else if constexpr (EPI == MEPI_SILU) {
      // row group G (16 W rows): gate (G even) / up (G odd) of output columns 16*(G/2) .. +15 -- the
      // wave's 4 groups are 2 output groups of 16 columns
      bf16x4 o[2];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // the roundings of GEMM -> bf16 gate|up -> silu_mul
          const float gt = (float)(bf16)acc[2 * q][u][r], up = (float)(bf16)acc[2 * q + 1][u][r];
          o[q][r] = (bf16)((float)(bf16)(gt / (1.f + __expf(-gt))) * up);
        }
      bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + ((n0 + wa * 64) >> 5) * 16 + lane_off;
      *reinterpret_cast<uint4*>(y) = pair16(o[0], o[1]);
    } else {
      bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + n0 + wa * 64 + lane_off;
#pragma unroll
      for (int f = 0; f < 4; f += 2) {
        bf16x4 lo, hi;
#pragma unroll
        for (int r = 0; r < 4; ++r) lo[r] = (bf16)acc[f][u][r], hi[r] = (bf16)acc[f + 1][u][r];
        Pack8 v;
        v.u = pair16(lo, hi);
        if constexpr (EPI == MEPI_RESID) {
          Pack8 rr;
          rr.u = *reinterpret_cast<const uint4*>(R + (long)m * ldr + n0 + wa * 64 + lane_off + 16 * f);
#pragma unroll
          for (int j = 0; j < 8; ++j) v.e[j] = (bf16)((float)v.e[j] + (float)rr.e[j]);
        }
        *reinterpret_cast<uint4*>(y + 16 * f) = v.u;
      }
    }
  }
}

}  // namespace

// Staging variant (PENNY_MID_VARIANT, or penny_gemm_mid_variant for in-process A/B): 0 = BK 64, 2-stage
// ring (64 KiB, 2 workgroups per CU), 1 = BK 64, 3-stage counted ring (96 KiB, 1 per CU), 2 = BK 32,
// 3-stage counted ring (48 KiB, 3 per CU)
static int g_mid_variant = -1;
static int mid_variant() {
  if (g_mid_variant < 0) {
    const char* v = getenv("PENNY_MID_VARIANT");
    g_mid_variant = v ? atoi(v) : 0;
  }
  return g_mid_variant;
}
PENNY_API int penny_gemm_mid_variant(int v) {
  const int old = mid_variant();
  if (v >= 0 && v <= 2) g_mid_variant = v;
  return old;
}

// Contract (checked): N % 128 == 0, K % (64 * S) == 0, ldx % 8 == 0, 16-B aligned rows; epi 0 bf16
// [M, N] (row stride ldy), 1 SiLU(gate)*up of the interleave16 gate|up weight -> bf16 [M, N/2], 2 f32
// split-K slabs P [S, M, N] (ldy unused), 3 bf16 + R (row stride ldr); epilogues other than 2 need S = 1.
PENNY_API int penny_gemm_mid(const void* X, int ldx, const void* W, int K, void* Y, int ldy, const void* R, int ldr,
                             int M, int N, int S, int epi, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % NT_ || S < 1 || K % (64 * S) || ldx % 8 || (epi != MEPI_SLAB && S != 1) || epi < 0 || epi > 3 ||
      (epi == MEPI_RESID && (!R || ldr % 8)) || (epi != MEPI_SLAB && ldy % 8))
    return (int)hipErrorInvalidValue;
  const long nwg = (long)((M + MT - 1) / MT) * (N / NT_) * S;
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)nwg);
  const int var = mid_variant();
  if (var == 2 && (K / S) % 32) return (int)hipErrorInvalidValue;
#define MID_LAUNCH(E)                                                                                                \
  if (var == 1)                                                                                                      \
    hipLaunchKernelGGL((gemm_mid_kernel<E, 128, 3>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, (const bf16*)W, \
                       K, Y, ldy, (const bf16*)R, ldr, M, N, S);                                                      \
  else if (var == 2)                                                                                                 \
    hipLaunchKernelGGL((gemm_mid_kernel<E, 64, 3>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, (const bf16*)W,  \
                       K, Y, ldy, (const bf16*)R, ldr, M, N, S);                                                      \
  else                                                                                                               \
    hipLaunchKernelGGL((gemm_mid_kernel<E, 128, 2>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, (const bf16*)W, \
                       K, Y, ldy, (const bf16*)R, ldr, M, N, S)
  switch (epi) {
    case MEPI_BF16: MID_LAUNCH(MEPI_BF16); break;
    case MEPI_SILU: MID_LAUNCH(MEPI_SILU); break;
    case MEPI_SLAB: MID_LAUNCH(MEPI_SLAB); break;
    default: MID_LAUNCH(MEPI_RESID); break;
  }
#undef MID_LAUNCH
  PENNY_RETURN_LAUNCH();
}
