// Mid-batch decode projection GEMM (K3/K8/K10 at 32 < M <= 256 tokens): f32 split-K slabs
//   P[s, m, n] = sum_{k in slice s} X[m, k] * W[n, k]        (Y = sum_s P[s] is reduced by the consumer)
//
// Why not hipBLASLt here: at M = 64..256 the QKV / O / down projections are still weight streams
// (33-117 MB of W against <= 7 MB of X) but the library runs them at 1.7-2.6 TB/s -- its tiles
// leave most CUs idle at N = 4096-6144 or re-read X per narrow tile.  This kernel is shaped for
// the stream instead:
//   * one workgroup = 4 waves owns BN = 16*NF rows of W and one K slice (split-K over the grid, S
//     slices) so N = 4096 still launches >= 256 workgroups; slice s = blockIdx.x % S keeps each
//     XCD on 8/S K slices, so X's L2 footprint per XCD is X/S (down-proj X is 7 MB at M = 256);
//   * BOTH operands stream into LDS with global_load_lds (16 B per lane, 1-KiB lane-linear pieces):
//     W from its MFMA-fragment-tiled copy (ops/gemm.py tile_weight -- each piece IS one A
//     fragment), X in full 128-B lines (8 token rows x 64 k per piece) with an XOR-swizzled image
//     chosen on the SOURCE address so the 16-lane phases of the fragment reads are conflict-free;
//     X is fetched once per workgroup and shared by its 4 waves (X/W on-chip traffic = M/BN);
//   * NBUF-deep ring (3-8, what fits in LDS) of BK = 64 stages, counted `s_waitcnt vmcnt` + one raw s_barrier per stage (no
//     vmcnt(0) drain in the steady state, no VGPR-destination loads in the loop at all);
//   * waves split the (W rows x tokens) tile WA x WB; v_mfma_f32_16x16x32_bf16, f32 accumulate;
//   * the epilogue writes the f32 partial tile (16-B stores); no in-launch reduction -- the next
//     kernel that reads Y anyway (residual-add+RMSNorm, RoPE/KV-write, or penny_splitk_reduce)
//     sums the S slabs, which costs S*4 B per output instead of a 1.5-2 us kernel boundary.
#include "common.h"

#include <utility>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

namespace {

template <int N>
__device__ __forceinline__ void vmcnt_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

union Frag {
  uint4 u;
  bf16x8 v;
};

// epilogues of splitk_gemm_kernel
enum { SK_SLAB = 0, SK_SILU = 1, SK_BF16 = 2, SK_SAMPLE = 3 };

// SK_SAMPLE (the streaming LM head + K12 sampler): per-row temperature (<= 0: greedy) and seed;
// pv / pi [M, pstride] partial (best score, token) per (row, workgroup tile, wave row).  Token
// ids are voff + local row; local rows >= vvalid (a vocab shard's padding) never win.
struct SkSample {
  const float* temps;
  const unsigned long long* seeds;
  float* pv;
  int* pi;
  int pstride, voff, vvalid;
};

// X image: token row r of a stage lives at byte r*128; its logical 16-B chunk c (k = 8c..8c+7) at
// physical chunk c ^ (r & 7) ^ ((r >> 3) & 1).  A fragment read (16 consecutive rows, one logical
// chunk) then touches 16 distinct (row parity, chunk) bank groups per 16-lane phase.
__device__ __forceinline__ int xswz(int r, int c) { return c ^ (r & 7) ^ ((r >> 3) & 1); }

// stage ring depth: as many BK=64 stages as fit in ~150 KB of LDS (one workgroup per CU), capped
// at 8 -- a CU must keep ~50-70 KB of W in flight to stream its 1/256 share of HBM bandwidth
// MAXB: ring depth cap -- 8 by default; 16 for the narrow configs (NF = 2-4 rows groups: 4-8 KiB of
// W per stage) whose 8-stage ring keeps only 28-56 KiB in flight per CU.  Also capped so the counted
// vmcnt ((NBUF - 2) * loads per stage) fits the 6-bit counter.
// BKM: BK=64 stages issued (and waited for) in pairs -- a ring slot then holds BKM stages, so each
// W row's consecutive 128-B chunks leave the CU back to back (row-major W: 256 contiguous bytes per
// row per issue instead of 128 B one stage period apart)
template <int NF, int MT, int KB = 150, int MAXB = 8, int BKM = 1>
struct Ring {
  static constexpr int SBYTES = (NF + MT) * 2 * 1024 * BKM;
  static constexpr int LOADS = (2 * NF + 2 * MT) / 4 * BKM;
  static constexpr int BY_LDS = KB * 1024 / SBYTES;
  static constexpr int BY_VM = 63 / LOADS + 2;
  static constexpr int CAP = MAXB / BKM > 3 ? MAXB / BKM : 3;
  static constexpr int NBUF = BY_LDS < CAP ? (BY_LDS < BY_VM ? BY_LDS : BY_VM) : (CAP < BY_VM ? CAP : BY_VM);
};

// compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>)
template <class F, int... U>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, U...>) {
  (f(std::integral_constant<int, U>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// wait until at most `younger` stages of this wave's glds are still in flight, then barrier
template <int LOADS, int MAXY>
__device__ __forceinline__ void wait_stage(int younger) {
  if constexpr (MAXY <= 0) {
    vmcnt_barrier<0>();
  } else {
    if (younger >= MAXY) vmcnt_barrier<MAXY * LOADS>();
    else wait_stage<LOADS, MAXY - 1>(younger);
  }
}

// MFMAs of one BK=64 stage.  `base` is __restrict__ ON PURPOSE: inlined, it gives the ds_reads
// alias-scope metadata, which is what lets hipcc's waitcnt pass leave the younger stages' LDS-DMA
// in flight -- without it the pass cannot tell them apart from this stage and drains vmcnt(0)
// before the first ds_read of every stage (measured: the ring then degenerates to one stage).
template <int FW, int TW, int WBYTES, bool WROW>
__device__ __forceinline__ void stage_mma(const char* __restrict__ base, f32x4 (&acc)[FW][TW], int wa, int wb,
                                          int lane, int g, int col) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    Frag wf[FW], xf[TW];
#pragma unroll
    for (int f = 0; f < FW; ++f) {
      if constexpr (WROW) {   // row-major W staged like X: row r at r*128, swizzled 16-B chunks
        const int r = (wa * FW + f) * 16 + col;
        wf[f].u = *reinterpret_cast<const uint4*>(base + r * 128 + xswz(r, 4 * kk + g) * 16);
      } else {
        wf[f].u = *reinterpret_cast<const uint4*>(base + ((wa * FW + f) * 2 + kk) * 1024 + lane * 16);
      }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int r = (wb * TW + t) * 16 + col;
      xf[t].u = *reinterpret_cast<const uint4*>(base + WBYTES + r * 128 + xswz(r, 4 * kk + g) * 16);
    }
#pragma unroll
    for (int f = 0; f < FW; ++f)
#pragma unroll
      for (int t = 0; t < TW; ++t)
        acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[f].v, xf[t].v, acc[f][t], 0, 0, 0);
  }
}

// Epilogues (EPI):
//   SK_SLAB   f32 partial slabs P [S, M, N] (reduced by the consumer's row pass);
//   SK_SILU   W is the 16-row-interleaved gate|up weight (ops/gemm.py interleave16) and S == 1: the
//             epilogue writes Y[m, f] = silu(gate) * up as bf16 [M, N/2] (ldy) instead of f32 slabs --
//             each wave owns whole (gate, up) row-group pairs, so the pair meets in one lane's registers;
//   SK_BF16   S == 1, Y bf16 [M, N] (ldy): a row-parallel TP shard whose output goes straight into the
//             all-reduce (no slab round trip, no reduce launch);
//   SK_SAMPLE S == 1, W = the [V, K] vocabulary projection (or a TP rank's padded shard): no logits
//             reach HBM -- each lane Gumbel-max-scores its bf16-rounded logits (sampler.hip's noise of
//             (row seed, global token id)) and each wave leaves one (score, token) pair per token row,
//             reduced per row by lm_sample_final_kernel (gemm_prefill.hip).  The weight-streaming LM
//             head for decode batches (M <= 128), where the 256x256 tile kernel is MFMA-bound on
//             padding rows.
// WROW: W is the plain row-major [N, K] weight (no fragment-tiled copy): its stage pieces are
// 8 rows x 128 B with the same source-side XOR swizzle as X, so every glds instruction still reads
// whole 128-B lines and the fragment reads stay conflict-free.
// RKB: LDS ring budget in KiB (150: one workgroup per CU; ~72: two co-resident workgroups, so one's
// pipeline ramp overlaps the other's stream when a CU runs several tiles in sequence).
template <int NF, int MT, int WA, int EPI = SK_SLAB, bool WROW = false, int RKB = 150, int MAXB = 8, int BKM = 1>
__global__ void __launch_bounds__(256, 1) splitk_gemm_kernel(const bf16* __restrict__ X, int ldx,
                                                             const bf16* __restrict__ Wt, int K,
                                                             float* __restrict__ P, int M, int N, int S,
                                                             bf16* __restrict__ Y = nullptr, int ldy = 0,
                                                             SkSample sa = SkSample{}) {
  constexpr bool SILU = EPI == SK_SILU;
  constexpr int WB = 4 / WA;
  constexpr int FW = NF / WA;   // W row groups per wave
  constexpr int TW = MT / WB;   // token tiles per wave
  static_assert(NF % WA == 0 && MT % WB == 0, "wave split");
  static_assert(!SILU || FW % 2 == 0, "SiLU epilogue needs (gate, up) row-group pairs per wave");
  constexpr int NBUF = Ring<NF, MT, RKB, MAXB, BKM>::NBUF;   // ring slots of BKM stages each
  static_assert(NBUF >= 3, "ring too shallow");
  constexpr int WBYTES = NF * 2 * 1024;        // W pieces of one BK=64 stage
  constexpr int XBYTES = MT * 2 * 1024;        // X pieces (16*MT rows x 128 B)
  constexpr int SBYTES = WBYTES + XBYTES;
  constexpr int PIECES = (2 * NF + 2 * MT);     // 1-KiB pieces per stage
  static_assert(PIECES % 4 == 0, "pieces must split evenly over 4 waves");
  constexpr int LOADS = PIECES / 4;             // glds per wave per stage
  constexpr int SLOT = BKM * SBYTES;
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * SLOT];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;
  const int s = blockIdx.x % S, tile = blockIdx.x / S;
  // token chunks (blockIdx.y): rows m0 .. m0 + 16*MT - 1 of X / Y / the slabs; one chunk for decode
  // batches, ceil(M / (16*MT)) for the small prefill steps of narrow TP shards
  const int Mtot = M, m0 = blockIdx.y * 16 * MT;
  M = min(Mtot - m0, 16 * MT);
  X += (long)m0 * ldx;
  if constexpr (EPI == SK_SILU || EPI == SK_BF16) Y += (long)m0 * ldy;
  PENNY_DASSERT(M > 0 && (EPI != SK_SAMPLE || gridDim.y == 1));
  PENNY_DASSERT((tile + 1) * 16 * NF <= N && K % (64 * BKM * S) == 0);
  const int n0 = tile * 16 * NF;
  const int kc = K / S, k0 = s * kc;
  const int nst = kc / (64 * BKM);              // ring slots to stream
  const int ksteps = K / 32;
  const int wa = w / WB, wb = w % WB;

  // per-lane glds source for each of this wave's pieces (fixed per kernel; advanced by k per stage)
  // piece id q = w*LOADS + i:  q < 2*NF -> W (row group q/2, k-step q%2), else X rows 8*(q-2NF)..
  const char* src[LOADS];
  int dst[LOADS];
  long step[LOADS];
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const int q = w * LOADS + i;
    if (q < 2 * NF && WROW) {
      const int r = q * 8 + (lane >> 3);                    // weight row within the tile
      const int c = xswz(r, lane & 7);
      src[i] = reinterpret_cast<const char*>(Wt + (long)(n0 + r) * K + k0 + 8 * c);
      step[i] = 128;       // 64 k per stage
      dst[i] = q * 1024;
    } else if (q < 2 * NF) {
      const int f = q >> 1, kk = q & 1;
      src[i] = reinterpret_cast<const char*>(Wt) +
               (((long)(n0 / 16 + f) * ksteps + k0 / 32 + kk) * 64 + lane) * 16;
      step[i] = 2 * 1024;  // two k-steps of one row group per stage
      dst[i] = (f * 2 + kk) * 1024;
    } else {
      const int xp = q - 2 * NF;
      const int r = xp * 8 + (lane >> 3);                 // token row within the tile
      const int c = xswz(r, lane & 7);                    // logical chunk this lane's slot holds
      const int row = min(r, M - 1);
      src[i] = reinterpret_cast<const char*>(X + (long)row * ldx + k0 + 8 * c);
      step[i] = 128;  // 64 bf16 per stage
      dst[i] = WBYTES + xp * 1024;
    }
  }
  auto stage = [&](int j) {
    char* base = smem + (j % NBUF) * SLOT;
    // default cache policy on W too: the nt hint measured 4-7 % slower at M >= 48 (2-3 % faster
    // only at M <= 32; profiles/r1_splitk_v5_qkv_nont.jsonl vs r1_splitk_v4_qkv.jsonl)
#pragma unroll
    for (int i = 0; i < LOADS; ++i)
#pragma unroll
      for (int u = 0; u < BKM; ++u)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src[i] + (j * BKM + u) * step[i]),
                                         (lds_void_t*)(base + u * SBYTES + dst[i]), 16, 0, 0);
  };

  f32x4 acc[FW][TW];
#pragma unroll
  for (int f = 0; f < FW; ++f)
#pragma unroll
    for (int t = 0; t < TW; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j)
    if (j < nst) stage(j);

  for (int j = 0; j < nst; ++j) {
    // stages j+1 .. min(j+NBUF-2, nst-1) may stay in flight
    wait_stage<LOADS * BKM, NBUF - 2>(min(NBUF - 2, nst - 1 - j));
    if (j + NBUF - 1 < nst) stage(j + NBUF - 1);
#pragma unroll
    for (int u = 0; u < BKM; ++u)
      stage_mma<FW, TW, WBYTES, WROW>(smem + (j % NBUF) * SLOT + u * SBYTES, acc, wa, wb, lane, g, col);
  }

  if constexpr (SILU) {
    // row group G = n0/16 + wa*FW + f is gate (G even) / up (G odd) of output cols 16*(G/2)..+15
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int m = (wb * TW + t) * 16 + col;
      if (m >= M) continue;
#pragma unroll
      for (int f = 0; f < FW; f += 2) {
        const int G = n0 / 16 + wa * FW + f;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // same roundings as GEMM -> bf16 gate|up -> silu_mul (HF: silu in the activation dtype)
          const float gt = (float)(bf16)acc[f][t][r], up = (float)(bf16)acc[f + 1][t][r];
          o[r] = (bf16)((float)(bf16)(gt / (1.f + __expf(-gt))) * up);
        }
        *reinterpret_cast<bf16x4*>(Y + (long)m * ldy + (G >> 1) * 16 + 4 * g) = o;
      }
    }
    return;
  }
  if constexpr (EPI == SK_BF16) {
    // lane holds W rows n = 16f + 4g + r (r = 0..3) for token 16t + col: one 8-B store per fragment
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int m = (wb * TW + t) * 16 + col;
      if (m >= M) continue;
#pragma unroll
      for (int f = 0; f < FW; ++f) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)acc[f][t][r];
        *reinterpret_cast<bf16x4*>(Y + (long)m * ldy + n0 + (wa * FW + f) * 16 + 4 * g) = o;
      }
    }
    return;
  }
  if constexpr (EPI == SK_SAMPLE) {
    // token row m's 16*FW columns of this wave sit in lanes col, col+16, col+32, col+48 (g = 0..3):
    // each scores its FW*4, two xor-shuffles inside that lane set (all active or all skipped: they
    // share m), and lane g == 0 leaves the wave's pair
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int m = (wb * TW + t) * 16 + col;
      if (m >= M) continue;
      const float temp = sa.temps[m];
      const bool greedy = !(temp > 0.f);
      const float inv_t = greedy ? 1.f : 1.f / temp;
      const unsigned long long seed = sa.seeds[m];
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int f = 0; f < FW; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int loc = n0 + (wa * FW + f) * 16 + 4 * g + r, idx = sa.voff + loc;
          float v = (float)(bf16)acc[f][t][r];   // the bf16 logit the unfused path samples
          if (!greedy) v = v * inv_t + gumbel_noise(seed, idx);
          if (loc >= sa.vvalid) v = -INFINITY;
          better(bv, bi, v, idx);
        }
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        better(bv, bi, ov, oi);
      }
      if (g == 0) {
        const long slot = (long)m * sa.pstride + tile * WA + wa;
        sa.pv[slot] = bv;
        sa.pi[slot] = bi;
      }
    }
    return;
  }
  // lane holds W rows n = 16f + 4g + r (r = 0..3) for token 16t + col: one 16-B store per tile
  float* ps = P + (long)s * Mtot * N + (long)m0 * N;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int m = (wb * TW + t) * 16 + col;
    if (m >= M) continue;
#pragma unroll
    for (int f = 0; f < FW; ++f) {
      const int n = n0 + (wa * FW + f) * 16 + 4 * g;
      *reinterpret_cast<f32x4*>(ps + (long)m * N + n) = acc[f][t];
    }
  }
}

// Y[m, n] = bf16(sum_s P[s, m, n]) (+ R[m, n], rounded like the unfused GEMM-then-add path)
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ P, int S, int M, int N,
                                                            bf16* __restrict__ Y, int ldy,
                                                            const bf16* __restrict__ R, int ldr) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;  // index of 8 outputs
  const long total8 = (long)M * N / 8;
  if (i8 >= total8) return;
  const int m = (int)(i8 / (N / 8));
  const int n = (int)(i8 % (N / 8)) * 8;
  float o[8];
  {
    const f32x4* p = reinterpret_cast<const f32x4*>(P + (long)m * N + n);
    const f32x4 a = p[0], b = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = a[j], o[4 + j] = b[j];
  }
  for (int s = 1; s < S; ++s) {
    const f32x4* p = reinterpret_cast<const f32x4*>(P + ((long)s * M + m) * N + n);
    const f32x4 a = p[0], b = p[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] += a[j], o[4 + j] += b[j];
  }
  if (R) {
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>(R + (long)m * ldr + n), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)(bf16)o[j] + r[j];
  }
  *reinterpret_cast<uint4*>(Y + (long)m * ldy + n) = pack8(o);
}

// wrow bit 0: W is the row-major [N, K] weight (else tile_weight's fragment-tiled copy); bit 1: BK=64
// stages issued in pairs (BKM = 2) -- taken where the ring still holds >= 3 slots and each K slice
// is a multiple of 128, else single stages.  (A double-buffered pair ring -- two slots, for the
// widest tiles at M 97-256 -- measured 3-14 % slower than single stages:
// profiles/r5_decode_gemm_pair_double_buffer_rejected.jsonl.)
template <int NF, int MT, int RKB, int MAXB>
constexpr bool pair_fits() {
  return Ring<NF, MT, RKB, MAXB, 2>::NBUF >= 3;
}

// one launch of splitk_gemm_kernel<NF, MT, WA, EPI, *, 150, MAXB, *> with the W layout / stage pairing
// of wrow (runtime) mapped onto the template arguments
template <int NF, int MT, int WA, int EPI, int MAXB, class... A>
int launch_any(int wrow, bool pair_ok, dim3 grid, hipStream_t st, A... args) {
  const bool rm = wrow & 1;
  if constexpr (pair_fits<NF, MT, 150, MAXB>()) {
    if ((wrow & 2) && pair_ok) {
      if (rm) hipLaunchKernelGGL((splitk_gemm_kernel<NF, MT, WA, EPI, true, 150, MAXB, 2>), grid, dim3(256), 0, st, args...);
      else hipLaunchKernelGGL((splitk_gemm_kernel<NF, MT, WA, EPI, false, 150, MAXB, 2>), grid, dim3(256), 0, st, args...);
      return (int)hipGetLastError();
    }
  }
  if (rm) hipLaunchKernelGGL((splitk_gemm_kernel<NF, MT, WA, EPI, true, 150, MAXB>), grid, dim3(256), 0, st, args...);
  else hipLaunchKernelGGL((splitk_gemm_kernel<NF, MT, WA, EPI, false, 150, MAXB>), grid, dim3(256), 0, st, args...);
  return (int)hipGetLastError();
}

template <int NF, int MT, int WA>
int launch(const void* X, int ldx, const void* Wt, int K, float* P, int M, int N, int S, int wrow, hipStream_t st) {
  return launch_any<NF, MT, WA, SK_SLAB, 8>(wrow, (K / S) % 128 == 0, dim3((N / (16 * NF)) * S, (M + 16 * MT - 1) / (16 * MT)), st, (const bf16*)X,
                                            ldx, (const bf16*)Wt, K, P, M, N, S, (bf16*)nullptr, 0, SkSample{});
}

template <int NF, int MT, int WA>
int launch_silu(const void* X, int ldx, const void* Wt, int K, void* Y, int ldy, int M, int N, int wrow,
                hipStream_t st) {
  return launch_any<NF, MT, WA, SK_SILU, NF == 2 ? 16 : 8>(wrow, K % 128 == 0, dim3(N / (16 * NF), (M + 16 * MT - 1) / (16 * MT)), st, (const bf16*)X,
                                                          ldx, (const bf16*)Wt, K, (float*)nullptr, M, N, 1, (bf16*)Y,
                                                          ldy, SkSample{});
}

template <int NF, int MT, int WA>
int launch_bf16(const void* X, int ldx, const void* Wt, int K, void* Y, int ldy, int M, int N, int wrow,
                hipStream_t st) {
  return launch_any<NF, MT, WA, SK_BF16, 16>(wrow, K % 128 == 0, dim3(N / (16 * NF), (M + 16 * MT - 1) / (16 * MT)), st, (const bf16*)X, ldx,
                                             (const bf16*)Wt, K, (float*)nullptr, M, N, 1, (bf16*)Y, ldy, SkSample{});
}

// the streaming LM head: row-major W (wrow) or its fragment-tiled copy; ring budget 150 KiB (one
// workgroup per CU) or 72 KiB (two)
template <int NF, int MT, int WA>
int launch_sample(const void* X, int ldx, const void* Wt, int K, int M, int N, int wrow, int ring2, const SkSample& sa,
                  hipStream_t st) {
  const dim3 grid(N / (16 * NF)), block(256);
#define SK_SAMPLE_LAUNCH(WROW_, KB_)                                                                               \
  hipLaunchKernelGGL((splitk_gemm_kernel<NF, MT, WA, SK_SAMPLE, WROW_, KB_, 16>), grid, block, 0, st, (const bf16*)X, ldx, \
                     (const bf16*)Wt, K, (float*)nullptr, M, N, 1, (bf16*)nullptr, 0, sa)
  // the 72-KiB ring only where it still holds >= 3 stages (else the 150-KiB one)
  constexpr bool R2 = Ring<NF, MT, 72, 16>::NBUF >= 3;
  if constexpr (R2) {
    if (ring2) {
      if (wrow & 1) SK_SAMPLE_LAUNCH(true, 72);
      else SK_SAMPLE_LAUNCH(false, 72);
      return (int)hipGetLastError();
    }
  }
  if (wrow & 1) SK_SAMPLE_LAUNCH(true, 150);
  else SK_SAMPLE_LAUNCH(false, 150);
#undef SK_SAMPLE_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace

// lm_sample_final_kernel's launcher (gemm_prefill.hip): per row, the best of P (score, token) pairs
extern "C" int penny_lm_sample_final(const float* pv, const int* pi, int P, int M, int* out, int* pairs,
                                     hipStream_t stream);

// Fused gate|up + SiLU*up for 16 < M <= 256 (K9 at mid-batch decode): W = tile_weight(interleave16
// gate|up) [N = 2F rows], Y [M, F] bf16 with row stride ldy.  No split-K: N = 28672 already gives
// N/(16*nf) = 224 (nf 8) or 448 (nf 4) workgroups.  M > 256: 256-row token chunks side by side on
// grid y.  Contract (checked): N % (16*nf) == 0, nf in {2, 4, 8}, K % 64 == 0, ldx % 8 == 0, ldy % 4 == 0.
PENNY_API int penny_gateup_silu_gemm(const void* X, int ldx, const void* Wt, int K, void* Y, int ldy, int M, int N,
                                     int nf, int wrow, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > (1 << 20) || K % 64 || ldx % 8 || ldy % 4 || (nf != 2 && nf != 4 && nf != 8) || N % (16 * nf))
    return (int)hipErrorInvalidValue;
  const int mt = min((M + 15) / 16, 16);   // > 256 rows: 256-row token chunks on grid y
  // nf = 2 (one (gate, up) pair per workgroup, WA = 1): twice the workgroups of nf = 4 for narrow
  // TP shards (Llama-3-70B TP=8 gate|up: N = 7168 -> 224 workgroups)
  if (nf == 2) {   // WA = 1 -> 4 token-tile wave columns: token tiles rounded up to a multiple of 4
    if (mt <= 4) return launch_silu<2, 4, 1>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);
    if (mt <= 8) return launch_silu<2, 8, 1>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);
    if (mt <= 12) return launch_silu<2, 12, 1>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);
    return launch_silu<2, 16, 1>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);
  }
#define GU_CASE(MT_, WA4_, WA8_)                                                          \
  if (mt <= MT_) {                                                                      \
    if (nf == 4) return launch_silu<4, MT_, WA4_>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream); \
    return launch_silu<8, MT_, WA8_>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);              \
  }
  GU_CASE(2, 2, 2)
  GU_CASE(4, 1, 2)
  GU_CASE(6, 2, 2)
  GU_CASE(8, 1, 2)
  GU_CASE(12, 1, 2)
  GU_CASE(16, 1, 2)
#undef GU_CASE
  return (int)hipErrorInvalidValue;
}

// Shape contract (checked): N % (16*NF) == 0, K % (64*S) == 0, X rows 16-B
// aligned (ldx % 8 == 0).  wrow: bit 0 row-major W instead of tile_weight's copy, bit 1 paired stages.  nf: W row groups per workgroup (2, 4, 6 or 8;
// 6 = 96 rows puts N = 6144 on exactly 64 tiles, i.e. 256 workgroups at S = 4; 16 -- half the X
// bytes per W byte -- measured 5-53 % slower at M = 32-128 on every 8B / TP=8 shape: too few
// workgroups, profiles/r5_decode_gemm_nf16_rejected.jsonl).  P is [S, M, N] f32.
// M > 256: 256-row token chunks side by side on grid y (small prefill steps of narrow TP shards).
PENNY_API int penny_splitk_gemm(const void* X, int ldx, const void* Wt, int K, void* P, int M, int N, int S, int nf,
                                int wrow, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > (1 << 20) || S < 1 || K % (64 * S) || ldx % 8 || (nf != 2 && nf != 4 && nf != 6 && nf != 8) || N % (16 * nf))
    return (int)hipErrorInvalidValue;
  const int mt = min((M + 15) / 16, 16);   // > 256 rows: 256-row token chunks on grid y
  float* p = static_cast<float*>(P);
#define SK_CASE(MT_, WA2_, WA4_, WA8_)                                                 \
  if (mt <= MT_) {                                                                     \
    if (nf == 2) return launch<2, MT_, WA2_>(X, ldx, Wt, K, p, M, N, S, wrow, stream); \
    if (nf == 4) return launch<4, MT_, WA4_>(X, ldx, Wt, K, p, M, N, S, wrow, stream); \
    if (nf == 6) return launch<6, MT_, 2>(X, ldx, Wt, K, p, M, N, S, wrow, stream);    \
    return launch<8, MT_, WA8_>(X, ldx, Wt, K, p, M, N, S, wrow, stream);              \
  }
  // (NF + MT) even; wave split picked to minimise fragment reads per wave (NF/WA + MT/WB)
  SK_CASE(2, 2, 2, 2)
  SK_CASE(4, 1, 1, 2)
  SK_CASE(6, 2, 2, 2)
  SK_CASE(8, 1, 1, 2)
  SK_CASE(12, 1, 1, 2)
  SK_CASE(16, 1, 1, 2)
#undef SK_CASE
  return (int)hipErrorInvalidValue;
}

// Split-K gate|up: P [S, M, N] f32 slabs of the interleave16 gate|up projection (row group 2j = gate
// features 16j..16j+15, 2j+1 = their up rows) -> Y [M, N/2] bf16 = silu(gate) * up with the SK_SILU
// epilogue's roundings.  For gate|up shapes whose column tiles alone underfill the chip (Llama-3-70B
// TP=8 shard: 7168 rows = 112 tiles at nf = 4) or whose weights stream row-major (70B TP=1: no tiled
// copy), the K split fills the CUs and this pass adds S*8 B per output.  One thread per 8 outputs.
__global__ void __launch_bounds__(256) splitk_reduce_silu_kernel(const float* __restrict__ P, int S, int M, int N,
                                                                 bf16* __restrict__ Y, int ldy) {
  const int F = N / 2;
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;  // index of 8 outputs
  const long total8 = (long)M * F / 8;
  if (i8 >= total8) return;
  const int m = (int)(i8 / (F / 8));
  const int f = (int)(i8 % (F / 8)) * 8;                 // 8 features of one 16-feature group
  const int ng = (f >> 4) * 32 + (f & 15);               // gate column; up = ng + 16
  float gt[8], up[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) gt[j] = up[j] = 0.f;
  for (int s = 0; s < S; ++s) {
    const f32x4* pg = reinterpret_cast<const f32x4*>(P + ((long)s * M + m) * N + ng);
    const f32x4* pu = reinterpret_cast<const f32x4*>(P + ((long)s * M + m) * N + ng + 16);
    const f32x4 g0 = pg[0], g1 = pg[1], u0 = pu[0], u1 = pu[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) gt[j] += g0[j], gt[4 + j] += g1[j], up[j] += u0[j], up[4 + j] += u1[j];
  }
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gb = (float)(bf16)gt[j], ub = (float)(bf16)up[j];
    o[j] = (float)(bf16)(gb / (1.f + __expf(-gb))) * ub;
  }
  *reinterpret_cast<uint4*>(Y + (long)m * ldy + f) = pack8(o);
}

PENNY_API int penny_splitk_reduce_silu(const void* P, int S, int M, int N, void* Y, int ldy, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 32 || ldy % 8 || S < 1) return (int)hipErrorInvalidValue;
  const long total8 = (long)M * (N / 2) / 8;
  hipLaunchKernelGGL(splitk_reduce_silu_kernel, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, stream,
                     (const float*)P, S, M, N, (bf16*)Y, ldy);
  return (int)hipGetLastError();
}

PENNY_API int penny_splitk_reduce(const void* P, int S, int M, int N, void* Y, int ldy, const void* R, int ldr,
                                  hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 8 || ldy % 8 || (R && ldr % 8)) return (int)hipErrorInvalidValue;
  const long total8 = (long)M * N / 8;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, stream,
                     (const float*)P, S, M, N, (bf16*)Y, ldy, (const bf16*)R, ldr);
  return (int)hipGetLastError();
}

// Row-parallel decode projection with a bf16 output (no split-K): Y [M, N] (row stride ldy) =
// X [M, K] x W [N, K]^T, one workgroup per 16*nf W rows -- the TP shards of O / down whose output
// feeds the all-reduce directly (Llama-3-70B TP=8: N = 8192 -> 256 workgroups at nf = 2).
// Contract (checked): N % (16*nf) == 0, nf in {2, 4, 8}, K % 64 == 0, ldx % 8 == 0, ldy % 4 == 0,
// M >= 1 (> 256: 256-row token chunks on grid y).
PENNY_API int penny_splitk_gemm_bf16(const void* X, int ldx, const void* Wt, int K, void* Y, int ldy, int M, int N,
                                     int nf, int wrow, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > (1 << 20) || K % 64 || ldx % 8 || ldy % 4 || (nf != 2 && nf != 4 && nf != 8) || N % (16 * nf))
    return (int)hipErrorInvalidValue;
  const int mt = min((M + 15) / 16, 16);   // > 256 rows: 256-row token chunks on grid y
#define BF_CASE(MT_, WA2_, WA4_, WA8_)                                                          \
  if (mt <= MT_) {                                                                            \
    if (nf == 2) return launch_bf16<2, MT_, WA2_>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);  \
    if (nf == 4) return launch_bf16<4, MT_, WA4_>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);  \
    return launch_bf16<8, MT_, WA8_>(X, ldx, Wt, K, Y, ldy, M, N, wrow, stream);               \
  }
  BF_CASE(2, 2, 2, 2)
  BF_CASE(4, 1, 1, 2)
  BF_CASE(6, 2, 2, 2)
  BF_CASE(8, 1, 1, 2)
  BF_CASE(12, 1, 1, 2)
  BF_CASE(16, 1, 1, 2)
#undef BF_CASE
  return (int)hipErrorInvalidValue;
}

// Weight-streaming LM head + sampler (K11 + K12) for decode batches, full vocabulary or a TP rank's
// padded shard: W [Vpad, K] (row-major with wrow = 1, else tile_weight's copy) holds global rows
// voff .. voff + vvalid - 1 then padding; per row m the Gumbel-max (temps[m] > 0) / argmax sample.
// out [M] int32 (the token) and/or pairs [M, 2] int32 (score bits, global id: the shard's candidate).
// workspace >= 2 * M * (Vpad / (16*nf)) * 2 floats.  ring2: the 72-KiB ring (two workgroups per CU).
// Contract (checked): 1 <= M <= 128, Vpad % (16*nf) == 0, nf in {4, 8}, 0 < vvalid <= Vpad,
// K % 64 == 0, ldx % 8 == 0.
PENNY_API int penny_lm_head_stream_sample(const void* X, int ldx, const void* W, int K, int M, int Vpad, int vvalid,
                                          int voff, const float* temps, const unsigned long long* seeds,
                                          void* workspace, int* out, int* pairs, int nf, int wrow, int ring2,
                                          hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 128 || (nf != 4 && nf != 8) || Vpad % (16 * nf) || vvalid <= 0 || vvalid > Vpad || voff < 0 || K % 64 ||
      ldx % 8 || !temps || !seeds || !workspace || (!out && !pairs))
    return (int)hipErrorInvalidValue;
  const int tiles = Vpad / (16 * nf), mt = (M + 15) / 16;
  // wave split per (nf, token tiles): as penny_splitk_gemm's table
  const int wa = nf == 8 ? 2 : (mt <= 2 || (mt > 4 && mt <= 6) ? 2 : 1);
  const int pstride = tiles * wa;
  float* pv = static_cast<float*>(workspace);
  int* pi = reinterpret_cast<int*>(pv + (long)M * pstride);
  const SkSample sa{temps, seeds, pv, pi, pstride, voff, vvalid};
  int rc;
#define LS_CASE(MT_, WA4_)                                                                                      \
  if (mt <= MT_) {                                                                                              \
    if (nf == 4) rc = launch_sample<4, MT_, WA4_>(X, ldx, W, K, M, Vpad, wrow, ring2, sa, stream);              \
    else rc = launch_sample<8, MT_, 2>(X, ldx, W, K, M, Vpad, wrow, ring2, sa, stream);                          \
  } else
  LS_CASE(2, 2)
  LS_CASE(4, 1)
  LS_CASE(6, 2)
  LS_CASE(8, 1)
  return (int)hipErrorInvalidValue;
#undef LS_CASE
  if (rc) return rc;
  return penny_lm_sample_final(pv, pi, pstride, M, out, pairs, stream);
}
