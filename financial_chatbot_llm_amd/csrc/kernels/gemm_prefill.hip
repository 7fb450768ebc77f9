// Prefill projection GEMM (K3 QKV, K8 O, K9 gate|up, K10 down at M = 256..4096+ token rows):
//   Y[m, n] = sum_k X[m, k] * W[n, k]          X [M, K] bf16 (row stride ldx), W [N, K] bf16
// with the epilogue fused into the tile:
//   EPI_BF16  Y bf16 [M, N] (row stride ldy)
//   EPI_SILU  W is the 16-row-interleaved gate|up weight (ops/gemm.py interleave16):
//             Y[m, f] = silu(gate) * up, bf16 [M, N/2] -- no [M, N] gate|up intermediate in HBM
//   EPI_SLAB  split-K: P[s, m, n] f32 partial sums over K slice s (S slices), reduced by the
//             consumer's own row pass (residual-add + RMSNorm, RoPE + KV write) -- fills the
//             256 CUs at small M without an extra reduce launch
//   EPI_RESID Y bf16 = bf16(acc) + R (residual add fused, rounded like GEMM-then-add)
//   EPI_BIAS / EPI_BIAS_GELU  Y bf16 = bf16(acc + bias[n]) [-> exact-erf GELU], R = the bias: the
//             bge encoder's QKV / O / fc2 and its GELU-MLP fc1 (no separate GELU pass)
//   EPI_SAMPLE the LM head fused with the K12 sampler: W = the [V, K] vocabulary projection, and
//             no logits reach HBM -- each lane scores its bf16-rounded logits (greedy, or
//             logit / T + Gumbel noise of (row seed, token id), sampler.hip's draw) and the
//             workgroup leaves one (best score, token) pair per (token row, 128-column wave half);
//             lm_sample_final_kernel reduces the V / 128 pairs of a row to the sampled token
//   EPI_ROPE  the fused QKV projection (K3+K4+K5): a wave's 128 output columns are exactly one
//             head, so the rotate-half RoPE pair (d, d+64) sits in one lane (accumulators f, f+4);
//             q heads -> rotated q [M, Hq, 128]; k heads -> rotated, v heads -> as is, both
//             scattered into the paged fragment-native KV cache (kv_layout.h).  Replaces the
//             [M, (Hq+2Hkv)*128] QKV activation round trip and the rope_kv pass.
//
// Why a hand-written kernel: hipBLASLt runs these shapes at 0.59-1.5 PF/s at the M the serving
// scheduler emits (profiles/r2_gemm_prefill_tunableop_sweep.jsonl), its best case is 256x256
// tiles launched with no K split (48 of 256 CUs busy for QKV at M = 512), and its epilogues
// (SiLU, residual) are separate passes over HBM.
//
// Structure (gfx950, one 512-thread workgroup per CU, 256 x 256 output tile, BK = 64):
//   * 8 waves as 2 (W rows) x 4 (tokens); each wave owns a 128 x 64 (n x token) sub-tile as
//     8 x 4 v_mfma_f32_16x16x32_bf16 accumulators.  MFMA A = W (so a lane's 4 accumulator
//     registers are 4 CONSECUTIVE output columns n -> vector stores, and a head's 128 dims sit in
//     one wave), MFMA B = X.
//   * both operands are staged into LDS by global_load_lds (16 B/lane, 1 KiB lane-linear pieces
//     of 8 rows x 128 B); the XOR swizzle phys_chunk = chunk ^ ((row >> 1) & 7) is applied on the
//     per-lane SOURCE address and on the fragment read, which makes every 16-lane phase of the
//     ds_read_b128 fragment reads bank-conflict free (2 rows share a 256-B bank row).
//   * LDS = 2 K-tiles x 4 half-tiles of 16 KiB, ordered by the phase that reads them:
//     W_q0 (W rows of quadrant-row 0 of both wave rows), X_q0, X_q1, W_q1.
//   * each K-tile runs as 4 phases {fragment ds_reads ; issue one half-tile of prefetch ;
//     s_barrier ; 16 MFMA ; s_barrier}.  A half-tile is restaged one phase after its last read,
//     so 3 half-tiles (6 loads per wave) stay in flight across every barrier: the only vmcnt wait
//     is a COUNTED vmcnt(6) once per K-tile (never 0 in the steady state).
//   * blockIdx is remapped bijectively so each XCD owns a contiguous range of tiles, grouped
//     4 token-tiles x N so the XCD's 32 concurrent tiles share X and W panels in its L2.
//   * wave quantisation (TailArgs): when the tile count T is not a multiple of the CU count C, the
//     first T - L tiles (L = T mod C) run whole, one per workgroup, and each of the L tail tiles is
//     split over s = C / L workgroups along K -- the last partial round costs 1/s of a tile
//     instead of a whole one (at M = 512 the QKV GEMM's 48 tiles become 240 workgroups).  Each
//     split stores its f32 accumulators, releases them (agent fence) and draws a ticket from the
//     tile's counter; the workgroup drawing s - 1 acquires, adds the other splits' partials into
//     its registers (in split order: bitwise repeatable), resets the counter and runs the tile's
//     ordinary epilogue.  No workgroup ever waits on another.
#include "common.h"
#include "kv_layout.h"

#include <type_traits>

namespace {

constexpr int TN = 256;              // W rows (output columns) per tile
constexpr int TM = 256;              // token rows per tile
constexpr int BK = 64;               // K per stage
constexpr int HALF = 128 * 128;      // half-tile: 128 rows x 64 bf16 = 16 KiB
constexpr int BUF = 4 * HALF;        // one K-tile (both operands)
constexpr int GM = 4;                // token tiles per L2 group (r5 sweep of 1-16 on the 8B prefill
                                     // projections: 4 within ~1 % of the best everywhere,
                                     // profiles/r5_tile_gemm_l2_group_sweep.jsonl)
enum { H_W0 = 0, H_X0 = 1, H_X1 = 2, H_W1 = 3 };
enum { EPI_BF16 = 0, EPI_SILU = 1, EPI_SLAB = 2, EPI_RESID = 3, EPI_ROPE = 4, EPI_BIAS = 5, EPI_BIAS_GELU = 6,
       EPI_MOE_SILU = 7, EPI_MOE_ROUTE = 8, EPI_SAMPLE = 9, EPI_MOE_SILU_MX = 10, EPI_MOE_ROUTE_MX = 11 };

// Grouped fp8 MoE GEMM (penny_moe_gemm_prefill_fp8): rows sorted by expert, bucket bounds on the
// DEVICE (offsets [E+1]), so tiles are found without a host round trip.
struct MoeArgs {
  const int* offsets;     // [E+1] sorted-row bucket bounds per expert
  const int* rows;        // [P] token row of each sorted row in X (GEMM1 gather), null: X is sorted
  const float* xs;        // per-row activation scale: xs[rows[p]] (GEMM1) / xs[p] (GEMM2)
  const float* ws;        // [E, N] per-output-row weight scales
  const float* route_w;   // [P] routing weight of each sorted row (EPI_MOE_ROUTE)
  int E;
  // MX hand-off between the two grouped GEMMs (EPI_MOE_SILU_MX writes, EPI_MOE_ROUTE_MX reads):
  // E8M0 scales of the fp8 intermediate, one per 32-element k-block, [tile][K-tile][1 KiB] where
  // "tile" is the 256-row token tile of the bucket walk (both GEMMs walk the same buckets) and a
  // K-tile's KiB is [row group wb 4][row col 16][k-block 4] dwords whose 4 bytes are the rows
  // wb*64 + 16j + col, j = 0..3: exactly the scale operand one lane of GEMM2 needs per K-tile
  // (byte j selected by the MFMA's op_sel).
  unsigned* mxs;
  int nkt;                // K-tiles of GEMM2 (F / 128)
};

// EPI_SAMPLE: per-row temperature (<= 0: greedy) and seed; pv / pi [M, 2 * N / 256] partial bests.
// Vocabulary-parallel (a TP rank's shard): token ids are voff + local row, and local rows >= vvalid
// (the shard's padding up to a multiple of 256) never win.
struct SampleArgs {
  const float* temps;
  const unsigned long long* seeds;
  float* pv;
  int* pi;
  int voff, vvalid;
};

// wave-quantisation tail (above): dpn whole tiles, then L tail tiles x s K-splits; part =
// [L, s, 256*256] f32, cnt = [L] zero-initialised tickets (self-resetting); s <= 1: no tail
struct TailArgs {
  int dpn, L, s;
  float* part;
  int* cnt;
  int gm = 0;             // token tiles per L2 group (0: GM); penny_gemm_prefill_set_group (A/B)
};

struct RopeArgs {
  const int* positions;   // [M]
  const float* cos_sin;   // [max_pos, 128]: cos of the 64 frequencies, then sin
  const int* slots;       // [M] paged-KV slot (block * 64 + offset), < 0 = do not store
  bf16* q_out;            // [M, Hq, 128]
  bf16* k_cache;          // [num_blocks, Hkv, 64 * 128]
  bf16* v_cache;
  int Hq, Hkv;
  // rotated q is stored as bf16(q * qscale): with qscale = softmax scale * log2(e) the attention
  // kernels take q prescaled at its one rounding (no second bf16 rounding of q * c)
  float qscale = 1.f;
};

// LDS row swizzle of 16-B chunks, per fragment-read pattern (ds_read_b128 16-lane phases, 2 rows
// per 256-B bank row): bf16 fragments read chunk 4kk + g, fp8 (16x16x128) fragments chunks 2g and
// 2g + 1 -- (r >> 1) & 7 and (r >> 1) & 5 make those conflict-free (exhaustive check over the
// linear XOR maps); rocprofv3 counts SQ_LDS_BANK_CONFLICT = 0 for the bf16 and fp8 variants
// (profiles/r3_gemm_prefill_lds_bank_conflicts_pmc.txt).
template <bool FP8>
__device__ __forceinline__ int swz(int r) { return FP8 ? ((r >> 1) & 5) : ((r >> 1) & 7); }

union Frag {
  uint4 u;
  bf16x8 v;
};
typedef int i32x8 __attribute__((ext_vector_type(8)));
// the two 16-B chunks a lane reads per fragment row: two bf16 k-steps, or ONE fp8 16x16x128 operand
union FragPair {
  Frag f[2];
  i32x8 v;
};

// Two 4-column groups of bf16 accumulators, lo = columns 16f + 4g .. +3 and hi = 16(f+1) + 4g .. +3
// in lane row g (= lane >> 4) -> the 8 CONSECUTIVE columns 16f + 8*(g>>1) + 16*(g&1) .. +7 of this
// lane, via v_permlane16_swap (odd lane rows of vdst <-> even lane rows of vsrc): one 16-B store
// instead of two 8-B ones (the epilogue store tail is issue-bound).
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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() { __builtin_amdgcn_s_barrier(); }

// Fragment reads.  Row r of a half-tile is at r*128; this lane's row within a 16-row fragment is
// (lane & 15), whose swizzle (lane >> 1) & 7 is folded into choff[kk].
__device__ __forceinline__ void read_w(const char* __restrict__ h, FragPair (&a)[4], int wa, int rowoff,
                                       const int (&choff)[2]) {
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      a[f].f[kk].u = *reinterpret_cast<const uint4*>(h + (wa * 64 + f * 16) * 128 + rowoff + choff[kk]);
}

// WT (fragment-tiled W, ops/gemm.py tile_weight): a half-tile's row group rgi (16 rows) and k-step kk
// is the lane-linear 1 KiB piece rgi * 2 + kk -- conflict-free by construction
__device__ __forceinline__ void read_w_tiled(const char* __restrict__ h, FragPair (&a)[4], int wa, int lane) {
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      a[f].f[kk].u = *reinterpret_cast<const uint4*>(h + ((wa * 4 + f) * 2 + kk) * 1024 + lane * 16);
}

__device__ __forceinline__ void read_x(const char* __restrict__ h, FragPair (&b)[2], int wb, int rowoff,
                                       const int (&choff)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      b[t].f[kk].u = *reinterpret_cast<const uint4*>(h + (wb * 32 + t * 16) * 128 + rowoff + choff[kk]);
}

// bf16: 2 k-steps of v_mfma_f32_16x16x32_bf16 per fragment pair.  fp8 (OCP e4m3): the whole
// 128-byte K-tile row in ONE v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair, unit block
// scales (E8M0 127 = 2^0) -- 2x the bf16 MFMA rate; lane (row l & 15) feeds its 32 bytes k-block
// (l >> 4) of A and of B alike, so the k order inside a block is the same on both operands.
// MFMAs stay inside their phase (sched_barriers against the machine scheduler, an empty asm "use"
// of the fp8 results against IR sinking): without that, hipcc moved every v_mfma_scale (fp8) of a
// K-tile past the phase barriers into its last phase (1 + 31 MFMAs between barriers instead of 8
// per phase), so the partner wave's fragment reads never overlapped them and every fragment was
// live at once (the balanced schedule then spilled 250 VGPRs).  The bf16 v_mfma_f32_16x16x32
// stayed in place.  tests/test_vw_asm_hazards.py checks the phase layout of both.
template <int F0, int T0, bool FP8, bool MXI = false>
__device__ __forceinline__ void mma(f32x4 (&acc)[8][4], const FragPair (&a)[4], const FragPair (&b)[2],
                                    unsigned sc = 0) {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
  if constexpr (FP8 && MXI) {
    // block-scaled X: byte T0 + t of this lane's scale word is the E8M0 scale of its token row
    // (fragment T0 + t) and k-block (lane >> 4); W keeps the unit scale (its row scales stay in
    // the epilogue)
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      acc[F0 + f][T0] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[f].v, b[0].v, acc[F0 + f][T0], 0, 0, 0,
                                                                         127, T0, (int)sc);
      acc[F0 + f][T0 + 1] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[f].v, b[1].v, acc[F0 + f][T0 + 1], 0, 0,
                                                                             0, 127, T0 + 1, (int)sc);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(acc[F0 + f][T0 + t]));
  } else if constexpr (FP8) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        acc[F0 + f][T0 + t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            a[f].v, b[t].v, acc[F0 + f][T0 + t], 0, 0, 0, 127, 0, 127);
    // the results "used" here, in place: an IR pass otherwise sank every fp8 MFMA of the K-tile
    // into its last phase (the intrinsic is pure; sched_barrier alone does not stop IR motion)
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(acc[F0 + f][T0 + t]));
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc[F0 + f][T0 + t] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f].f[kk].v, b[t].f[kk].v, acc[F0 + f][T0 + t], 0, 0, 0);
  }
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

// ABL (diagnostic builds only, penny_gemm_prefill_ablate): 1 = no LDS-DMA inside the K loop,
// 2 = no fragment ds_reads inside the K loop, 3 = LDS-DMA issued but never waited for in the
// steady state (wrong results; timing attribution only)
// BAL: balanced fragment-read schedule (below); 0 = the plain 12/4/8/0 schedule (A/B reference)
// FP8: X and W are OCP e4m3 bytes (K-tile = 128 elements), the grouped MoE form: W is [E, N, K],
// M counts sorted rows, the grid covers ceil(M/256) + E token tiles per column tile and the
// surplus workgroups exit before touching LDS.
// WT: W is the fragment-tiled copy (tile_weight) instead of the row-major [N, K] weight (bf16 only)
template <int EPI, int ABL = 0, int BAL = 1, bool FP8 = false, bool WT = false>
__global__ void __launch_bounds__(512) gemm_prefill_kernel(const void* __restrict__ Xv, int ldx,
                                                           const void* __restrict__ Wv, int K,
                                                           void* __restrict__ Y, int ldy,
                                                           const bf16* __restrict__ R, int ldr,
                                                           int M, int N, int S, RopeArgs ra, MoeArgs ma,
                                                           SampleArgs sa, TailArgs ta) {
  static_assert(!(WT && FP8), "fragment-tiled W: bf16 only");
  constexpr int ESZ = FP8 ? 1 : 2;        // bytes per element
  constexpr int BKE = 128 / ESZ;          // elements per K-tile row (128 bytes)
  constexpr bool MXI = EPI == EPI_MOE_ROUTE_MX;   // X carries E8M0 block scales (GEMM2 of the MX hand-off)
  constexpr bool MXO = EPI == EPI_MOE_SILU_MX;    // the epilogue writes fp8 + block scales (GEMM1)
  static_assert(!(MXI || MXO) || (FP8 && BAL), "MX hand-off: fp8 tiles on the balanced schedule");
  // X0 half-tiles carry one more LDS-DMA per wave under MXI (the K-tile's 1 KiB of scales)
  constexpr int XL0 = MXI ? 3 : 2;
  const char* __restrict__ X = static_cast<const char*>(Xv);
  const char* __restrict__ W = static_cast<const char*>(Wv);
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF + (MXI ? 2048 : 0)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wa = w >> 2, wb = w & 3;  // wave grid 2 (W rows) x 4 (tokens)
  const int g = lane >> 4, col = lane & 15;

  // ---- tile of this workgroup: bijective XCD remap, then L2 groups of GM token tiles ----
  const int Mt = (M + TM - 1) / TM + (FP8 ? ma.E : 0), Nt = N / TN, tiles = Mt * Nt;
  const bool tail = !FP8 && ta.s > 1 && (int)blockIdx.x >= ta.dpn;   // workgroup-uniform
  int s = 0, tile, tu = 0, tj = 0;
  if (tail) {
    const int u = blockIdx.x - ta.dpn;        // tail workgroups are dispatched last, round robin
    tu = u % ta.L;
    tj = u / ta.L;
    tile = ta.dpn + tu;
  } else {
    const int nwg = ta.s > 1 ? ta.dpn : tiles * S;
    int id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
    s = id / tiles;
    tile = id - s * tiles;
  }
  const int GMr = ta.gm > 0 ? ta.gm : GM;
  const int grp = tile / (GMr * Nt), first = grp * GMr, gm = min(Mt - first, GMr);
  const int within = tile - grp * GMr * Nt;
  const int tm = first + within % gm, tn = within / gm;
  int m0 = tm * TM, mend = M, e = 0;
  const int n0 = tn * TN;
  if constexpr (FP8) {
    // token tile tm -> (expert e, its bucket's tile): walk the bucket sizes (E is small)
    int rem = tm;
    for (e = 0; e < ma.E; ++e) {
      const int lo = ma.offsets[e], hi = ma.offsets[e + 1], nte = (hi - lo + TM - 1) / TM;
      if (rem < nte) {
        m0 = lo + rem * TM;
        mend = hi;
        break;
      }
      rem -= nte;
    }
    if (e == ma.E) return;                 // surplus tile of the upper-bound grid: whole WG exits
    W += (long)e * N * K;
  }
  int k0, nt;
  if (tail) {                                 // K-tiles [tj * ntot / s, (tj + 1) * ntot / s)
    const int ntot = K / BKE, kb = tj * ntot / ta.s, ke = (tj + 1) * ntot / ta.s;
    k0 = kb * BKE;
    nt = ke - kb;
  } else {
    const int kc = K / S;
    k0 = s * kc;
    nt = kc / BKE;
  }
  PENNY_DASSERT(N % TN == 0 && nt >= 1 && tm < Mt && tn < Nt);

  // ---- per-lane LDS-DMA sources: half h, piece i -> LDS rows 16w + 8i .. +7 of that half ----
  // fp8 (grouped MoE): 32-bit byte offsets from the wave-uniform W / X bases (SGPRs), the saddr
  // form of the DMA -- half the VGPRs of 64-bit per-lane pointers (an expert's W is < 2 GiB and
  // so are the [P, K] activations), which the balanced schedule + MX scales need.
  const char* src[4][2];
  unsigned soff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = 16 * w + 8 * i + (lane >> 3);
      const int c = (lane & 7) ^ swz<FP8>(lr);            // logical 16-B chunk held by this slot
      if (h == H_W0 || h == H_W1) {
        const int n = n0 + (lr >> 6) * 128 + (h == H_W1 ? 64 : 0) + (lr & 63);
        if constexpr (FP8) soff[h][i] = (unsigned)(((long)n * K + k0) + 16 * c);
        else if constexpr (WT) {
          // piece (w, i) of the half = row group rgi = w, k-step i: global row group G
          const int G = n0 / 16 + (w >> 2) * 8 + (w & 3) + (h == H_W1 ? 4 : 0);
          src[h][i] = W + (((long)G * (K / 32) + k0 / 32 + i) * 64 + lane) * 16;
        } else src[h][i] = W + ((long)n * K + k0) * ESZ + 16 * c;
      } else {
        int m = min(m0 + (lr >> 5) * 64 + (h == H_X1 ? 32 : 0) + (lr & 31), mend - 1);
        if (FP8 && ma.rows) m = ma.rows[m];              // GEMM1 gathers the routed token rows
        if constexpr (FP8) soff[h][i] = (unsigned)(((long)m * ldx + k0) + 16 * c);
        else src[h][i] = X + ((long)m * ldx + k0) * ESZ + 16 * c;
      }
    }
  // The LDS-DMA is issued from inline asm, invisible to hipcc's waitcnt pass: with the builtin,
  // hipcc cannot prove the fragment ds_reads do not alias the in-flight DMA and drains vmcnt(0)
  // before every phase.  The counted vmcnt(6) below is then the only wait on these loads (the
  // loop issues no other vector-memory instruction), and M0 is set and restored in the statement.
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  // MXI: the K-tile's scale KiB lands next to the two K-tile buffers, each wave 128 B of it (lanes
  // 0-31, 4 B each); issued with the X_q0 half, so it is retired by that half's wait
  // (wave-uniform base: kept in SGPRs; the lane offset is added at issue -- a per-lane pointer held
  // across the loop cost the two VGPRs that made the GEMM2 loop spill)
  const char* mxbase = nullptr;
  if constexpr (MXI) mxbase = reinterpret_cast<const char*>(ma.mxs) + ((long)tm * ma.nkt + k0 / BKE) * 1024 + w * 128;
  auto stage = [&](int h, int t, unsigned buf) {
    if (ABL == 1 && t > 1) return;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned dst = buf + h * HALF + (16 * w + 8 * i) * 128;
      unsigned keep;
      if constexpr (FP8) {
        const unsigned vo = soff[h][i] + (unsigned)t * 128;
        const char* base = (h == H_W0 || h == H_W1) ? W : X;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(vo), "s"(dst), "s"(base)
                     : "memory");
      } else {
        // one K-tile = 128 B of a row-major row, or two 1-KiB k-step pieces of a tiled row group
        const char* gp = src[h][i] + (long)t * ((WT && (h == H_W0 || h == H_W1)) ? 2048 : 128);
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gp), "s"(dst)
                     : "memory");
      }
    }
    if constexpr (MXI) {
      if (h == H_X0) {
        const char* gp = mxbase + (long)t * 1024 + lane * 4;
        const unsigned dst = lds0 + 2 * BUF + (t & 1) * 1024 + w * 128;
        unsigned keep;
        if (lane < 32)
          asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep)
                       : "v"(gp), "s"(dst)
                       : "memory");
      }
    }
  };
  // this lane's scale word of K-tile t (byte j: token row wb*64 + 16j + col, k-block g)
  auto read_sc = [&](int t) -> unsigned {
    if constexpr (MXI)
      return *reinterpret_cast<const unsigned*>(smem + 2 * BUF + (t & 1) * 1024 + wb * 256 + col * 16 + g * 4);
    else
      return 0u;
  };

  const int rowoff = col * 128;
  // fragment chunks of this lane: bf16 {g, 4 + g} (one per 32-k MFMA step), fp8 {2g, 2g + 1} (the
  // 32-byte k-block of the 16x16x128 MFMA); row (lane & 15)'s swizzle folded in
  const int choff[2] = {((FP8 ? 2 * g : g) ^ swz<FP8>(col)) << 4, ((FP8 ? 2 * g + 1 : 4 + g) ^ swz<FP8>(col)) << 4};

  f32x4 acc[8][4];
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  FragPair a[4], b0[2], b1[2];
#define READ_W(half_)                                              \
  do {                                                             \
    if constexpr (WT) read_w_tiled((half_), a, wa, lane);         \
    else read_w((half_), a, wa, rowoff, choff);                   \
  } while (0)

  // ---- prologue: K-tile 0 whole, K-tile 1 halves W0, X0, X1 ----
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(h, 0, lds0);
  if (nt > 1) {
#pragma unroll
    for (int h = 0; h < 3; ++h) stage(h, 1, lds0 + BUF);
    wait_vm<4 + XL0>();
  } else {
    wait_vm<0>();
  }
  bar();
  // Stagger: waves 4-7 (wave row wa = 1; SIMD s hosts waves s and s+4, one of each row) pass one
  // extra barrier here, so barrier instance i is phase-body i of one row and i-1 of the other:
  // each SIMD alternates one wave's fragment ds_reads with its partner's 16 MFMAs.  Hazards with
  // the offset: a W half-tile is restaged only by the wave row that reads it (rows 64*wa..), and
  // an X half-tile is restaged by the other row >= 1 barrier instance after this row's reads of
  // it retired (lgkmcnt(0) before the row's next barrier); the vmcnt(6) wait of phase 4 precedes
  // that row's barrier instance 8t+7 (row 0) / 8t+8 (row 1) and the next tile's first read
  // follows instance 8t+8 / 8t+9.  Row 0 passes one extra barrier after the loop to balance.
  if (wa == 1) bar();

  // one phase: [fragment reads + DMA issued by the caller] barrier lgkmcnt(0) 16 MFMAs barrier
  auto phase = [&](auto F0c, auto T0c, const FragPair (&aa)[4], const FragPair (&bb)[2], unsigned sc = 0) {
    constexpr int F0 = decltype(F0c)::value, T0 = decltype(T0c)::value;
    bar();
    wait_lgkm0();
    mma<F0, T0, FP8, MXI>(acc, aa, bb, sc);
    bar();
  };
  using I0 = std::integral_constant<int, 0>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;

  if constexpr (BAL) {
    // Balanced read schedule: the next K-tile's X_q0 fragments (B0) are read in phase 4, which
    // reads nothing otherwise, so each phase moves 8 / 4 / 8 / 4 fragments per wave instead of
    // 12 / 4 / 8 / 0 (phase 1's 48 KB of reads + 16 KB of landing DMA filled its whole MFMA
    // window on the LDS).  The extra wait: vmcnt(8) in phase 3 retires X_q0 (and W_q0) of t+1
    // (4 younger half-tiles may stay in flight), a phase before it is read.
    // MXI: a K-tile's scale word is read with its W_q0 fragments (phase 1; it landed with X_q0,
    // retired by the phase-3 wait of the tile before) and held through the tile -- its buffer is
    // restaged with X_q0 of t+2 in phase 3, two phases later
    FragPair c0[2];
    unsigned sc = 0;
    auto tile = [&](int t, FragPair (&bc)[2], FragPair (&bn)[2]) {
      const char* cur = smem + (t & 1) * BUF;
      const char* nx = smem + ((t + 1) & 1) * BUF;
      const unsigned lcur = lds0 + (t & 1) * BUF, lnxt = lds0 + ((t + 1) & 1) * BUF;
      const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
      if (ABL != 2 || t == 0) READ_W(cur + H_W0 * HALF);
      sc = read_sc(t);
      if (more1) stage(H_W1, t + 1, lnxt);
      phase(I0{}, I0{}, a, bc, sc);
      if (ABL != 2 || t == 0) read_x(cur + H_X1 * HALF, b1, wb, rowoff, choff);
      if (more2) stage(H_W0, t + 2, lcur);
      phase(I0{}, I2{}, a, b1, sc);
      if (ABL != 2 || t == 0) READ_W(cur + H_W1 * HALF);
      if (more2) {
        stage(H_X0, t + 2, lcur);
        if (ABL != 3) wait_vm<6 + XL0>();
      } else {
        wait_vm<0>();
      }
      phase(I4{}, I2{}, a, b1, sc);
      if (more1 && (ABL != 2 || t == 0)) read_x(nx + H_X0 * HALF, bn, wb, rowoff, choff);
      if (more2) {
        stage(H_X1, t + 2, lcur);
        if (ABL != 3) wait_vm<4 + XL0>();
      } else {
        wait_vm<0>();
      }
      phase(I4{}, I0{}, a, bc, sc);
    };
    read_x(smem + H_X0 * HALF, b0, wb, rowoff, choff);
    int t = 0;
    for (; t + 1 < nt; t += 2) {
      tile(t, b0, c0);
      tile(t + 1, c0, b0);
    }
    if (t < nt) tile(t, b0, c0);
  } else {
    for (int t = 0; t < nt; ++t) {
      const char* cur = smem + (t & 1) * BUF;
      const unsigned lcur = lds0 + (t & 1) * BUF, lnxt = lds0 + ((t + 1) & 1) * BUF;
      const bool more1 = t + 1 < nt, more2 = t + 2 < nt;
      // phase 1: W_q0 x X_q0          restage: W_q1 of tile t+1 (read last in phase 3 of t-1)
      if (ABL != 2 || t == 0) {
        READ_W(cur + H_W0 * HALF);
        read_x(cur + H_X0 * HALF, b0, wb, rowoff, choff);
      }
      if (more1) stage(H_W1, t + 1, lnxt);
      phase(I0{}, I0{}, a, b0);
      // phase 2: W_q0 x X_q1          restage: W_q0 of tile t+2 (read in phase 1)
      if (ABL != 2 || t == 0) read_x(cur + H_X1 * HALF, b1, wb, rowoff, choff);
      if (more2) stage(H_W0, t + 2, lcur);
      phase(I0{}, I2{}, a, b1);
      // phase 3: W_q1 x X_q1          restage: X_q0 of tile t+2 (read in phase 1)
      if (ABL != 2 || t == 0) READ_W(cur + H_W1 * HALF);
      if (more2) stage(H_X0, t + 2, lcur);
      phase(I4{}, I2{}, a, b1);
      // phase 4: W_q1 x X_q0          restage: X_q1 of tile t+2 (read in phase 2); retire tile t+1
      // (the 3 younger half-tiles of t+2 may stay in flight)
      if (more2) {
        stage(H_X1, t + 2, lcur);
        if (ABL != 3) wait_vm<6>();
      } else {
        wait_vm<0>();
      }
      phase(I4{}, I0{}, a, b0);
    }
  }
  if (wa == 0) bar();

  if (!FP8 && tail) {
    // ---- wave-quantisation tail: publish this K-split's accumulators; the last split combines ----
    // partial layout [wave][f][t][lane] f32x4: every store / load instruction moves 1 KiB contiguous
    float* mine = ta.part + ((long)tu * ta.s + tj) * (TM * TN);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<f32x4*>(mine + ((((w * 8 + f) * 4 + t) * 64 + lane) << 2)) = acc[f][t];
    wait_vm<0>();
    __syncthreads();                          // every wave's stores issued and retired
    int* flag = reinterpret_cast<int*>(smem); // LDS is free: the K loop is over for all waves
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      wait_vm<0>();
      const int old = __hip_atomic_fetch_add(&ta.cnt[tu], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == ta.s - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        wait_vm<0>();
        __hip_atomic_store(&ta.cnt[tu], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
      }
      *reinterpret_cast<volatile int*>(flag) = last;
    }
    __syncthreads();
    if (!*reinterpret_cast<volatile int*>(flag)) return;
    // sum every split (its own included, re-read) in split order whichever drew the last ticket, so
    // the result is bitwise repeatable; each pass issues its 32 independent 16-B loads at once
    const float* base = ta.part + (long)tu * ta.s * (TM * TN) + ((w * 32 * 64 + lane) << 2);
    for (int j = 0; j < ta.s; ++j) {
      const float* pj = base + (long)j * (TM * TN);
#pragma unroll
      for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(pj + ((f * 4 + t) * 64 << 2));
          acc[f][t] = j == 0 ? v : acc[f][t] + v;
        }
    }
  }

  // ---- epilogue: lane holds Y[m0 + wb*64 + 16t + col][n0 + wa*128 + 16f + 4g + r], r = 0..3 ----
  // bf16 outputs leave as 16-B stores: pair16 swaps 8-B halves between lane rows g and g^1 (same
  // token row m, so a lane masked off by m >= M always has a masked swap partner), after which a
  // lane holds 8 consecutive columns at lane_off + 16*(group pair index)
  const int lane_off = 8 * (g >> 1) + 16 * (g & 1);
  if constexpr (MXO) {
    // GEMM1 of the MX hand-off: SiLU(gate) * up with EPI_MOE_SILU's roundings, then per (row,
    // 32-column block) an E8M0 scale 2^X, X = ceil(log2(amax / 448)) (no saturation), and the
    // block's e4m3 bytes of value / 2^X -- the intermediate leaves as fp8 (half the bytes of bf16)
    // and GEMM2 reads it without a per-row quantisation pass.
    // The blocks are the ones the block-scaled MFMA scales together with the fragment layout of
    // GEMM2 (lane group g holds 16-B chunks 2g, 2g+1 of the 128-B K-tile row): measured
    // (tests/test_kernels_gpu.py test_mfma_scale_operand_map_dump), the scale of lane group g'
    // covers chunks {0,2}, {4,6}, {1,3}, {5,7} for g' = 0..3 -- i.e. in this
    // wave's 4 column groups q (16 columns each; wave wa holds chunks 4wa..4wa+3) block bb takes
    // q = bb and bb + 2, and its scale is k-block g' = wa + 2bb.  A block's 32 columns are lanes
    // g = 0..3 (4 each) x the two q: amax is two xor-shuffles over g.
    const float* wsc = ma.ws + (long)e * N + n0 + wa * 128;
    unsigned char* yq = static_cast<unsigned char*>(Y);
    const int ocol = ((n0 + wa * 128) >> 1) + 4 * g;        // this lane's first output column
    unsigned word[2] = {0u, 0u};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = m0 + wb * 64 + t * 16 + col;
      const bool valid = m < mend;                        // uniform over the 4 lanes of row m
      const int mr = min(m, mend - 1);
      const float sx = ma.xs[ma.rows ? ma.rows[mr] : mr];
      float o[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 sg = *reinterpret_cast<const f32x4*>(wsc + 32 * q + 4 * g);
        const f32x4 su = *reinterpret_cast<const f32x4*>(wsc + 32 * q + 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gv = (float)(bf16)(acc[2 * q][t][r] * sx * sg[r]);
          const float uv = (float)(bf16)(acc[2 * q + 1][t][r] * sx * su[r]);
          o[q][r] = (float)(bf16)((float)(bf16)(gv / (1.f + __expf(-gv))) * uv);
        }
      }
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {
        float amax = 0.f;
#pragma unroll
        for (int q = bb; q < 4; q += 2)
#pragma unroll
          for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(o[q][r]));
        amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
        const unsigned bits = __float_as_uint(amax * (1.f / 448.f));
        const int ex = (int)((bits >> 23) & 0xff);
        int X = ex == 0 ? -127 : ex - 127 + ((bits & 0x7fffff) != 0);
        X = max(-127, min(X, 126));
        word[bb] |= (unsigned)(X + 127) << (8 * t);
        const float inv = __uint_as_float((unsigned)(127 - X) << 23);   // 2^-X, exact
        if (valid) {
#pragma unroll
          for (int q = bb; q < 4; q += 2) {
            uint32_t pk = 0;
            pk = __builtin_amdgcn_cvt_pk_fp8_f32(o[q][0] * inv, o[q][1] * inv, pk, false);
            pk = __builtin_amdgcn_cvt_pk_fp8_f32(o[q][2] * inv, o[q][3] * inv, pk, true);
            *reinterpret_cast<uint32_t*>(yq + (long)m * ldy + ocol + 16 * q) = pk;
          }
        }
      }
    }
    // lane g < 2 stores block g's scale word: rows wb*64 + 16j + col (byte j), k-block wa + 2g of
    // GEMM2's K-tile n0 / 256
    if (g < 2)
      ma.mxs[((long)tm * ma.nkt + n0 / 256) * 256 + wb * 64 + col * 4 + wa + 2 * g] = g == 0 ? word[0] : word[1];
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int m = m0 + wb * 64 + t * 16 + col;
    if (m >= mend) continue;
    if constexpr (EPI == EPI_MOE_SILU || EPI == EPI_MOE_ROUTE || EPI == EPI_MOE_ROUTE_MX) {
      // dequantise (activation row scale x weight row scale), then the decode pipeline's epilogue
      // roundings (moe.hip moe_gemm_kernel): SiLU(gate) * up, or x routing weight.  MX input: the
      // activation's block scales were applied inside the MFMA
      const float sx = MXI ? 1.f : ma.xs[ma.rows ? ma.rows[m] : m];
      const float* wsc = ma.ws + (long)e * N + n0 + wa * 128;
      if constexpr (EPI == EPI_MOE_SILU) {
        bf16x4 o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 sg = *reinterpret_cast<const f32x4*>(wsc + 32 * q + 4 * g);
          const f32x4 su = *reinterpret_cast<const f32x4*>(wsc + 32 * q + 16 + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gv = (float)(bf16)(acc[2 * q][t][r] * sx * sg[r]);
            const float uv = (float)(bf16)(acc[2 * q + 1][t][r] * sx * su[r]);
            o[q][r] = (bf16)((float)(bf16)(gv / (1.f + __expf(-gv))) * uv);
          }
        }
        bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + ((n0 + wa * 128) >> 5) * 16 + lane_off;
#pragma unroll
        for (int q = 0; q < 4; q += 2) *reinterpret_cast<uint4*>(y + 16 * q) = pair16(o[q], o[q + 1]);
      } else {
        const float rw = sx * ma.route_w[m];
        bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + n0 + wa * 128 + lane_off;
#pragma unroll
        for (int f = 0; f < 8; f += 2) {
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(wsc + 16 * f + 4 * g);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(wsc + 16 * f + 16 + 4 * g);
          bf16x4 lo, hi;
#pragma unroll
          for (int r = 0; r < 4; ++r) lo[r] = (bf16)(acc[f][t][r] * s0[r] * rw), hi[r] = (bf16)(acc[f + 1][t][r] * s1[r] * rw);
          *reinterpret_cast<uint4*>(y + 16 * f) = pair16(lo, hi);
        }
      }
    } else if constexpr (EPI == EPI_SAMPLE) {
      // lanes col, col + 16, col + 32, col + 48 hold this row's 128 columns of the wave: each scores
      // its 32, then two xor-shuffles inside the same-row lane set (all active or all skipped)
      const float temp = sa.temps[m];
      const bool greedy = !(temp > 0.f);
      const float inv_t = greedy ? 1.f : 1.f / temp;
      const unsigned long long seed = sa.seeds[m];
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int loc = n0 + wa * 128 + f * 16 + 4 * g + r, idx = sa.voff + loc;
          float v = (float)(bf16)acc[f][t][r];          // the bf16 logit the unfused path samples
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
        const long slot = (long)m * (2 * Nt) + 2 * tn + wa;
        sa.pv[slot] = bv;
        sa.pi[slot] = bi;
      }
    } else if constexpr (EPI == EPI_ROPE) {
      constexpr int D = 128;
      const int hd = (n0 + wa * 128) >> 7;     // this wave's head (q heads, then k, then v)
      const int slot = ra.slots[m];
      if (hd >= ra.Hq && slot < 0) continue;
      const long blk = slot >= 0 ? slot / KV_BS : 0;
      const int off = slot >= 0 ? slot % KV_BS : 0;
      if (hd < ra.Hq + ra.Hkv) {
        const float* cs = ra.cos_sin + (long)ra.positions[m] * D;
        const float qs = hd < ra.Hq ? ra.qscale : 1.f;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const int d = f * 16 + 4 * g;       // this lane's dims d..d+3 and d+64..d+67
          const f32x4 co = *reinterpret_cast<const f32x4*>(cs + d), si = *reinterpret_cast<const f32x4*>(cs + 64 + d);
          bf16x4 o1, o2;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // GEMM output rounded to bf16 first, as the unfused GEMM -> rope_kv path does
            const float x1 = (float)(bf16)acc[f][t][r], x2 = (float)(bf16)acc[f + 4][t][r];
            o1[r] = (bf16)((x1 * co[r] - x2 * si[r]) * qs);
            o2[r] = (bf16)((x2 * co[r] + x1 * si[r]) * qs);
          }
          if (hd < ra.Hq) {
            bf16* q = ra.q_out + ((long)m * ra.Hq + hd) * D;
            *reinterpret_cast<bf16x4*>(q + d) = o1;
            *reinterpret_cast<bf16x4*>(q + 64 + d) = o2;
          } else {
            bf16* kb = ra.k_cache + (blk * ra.Hkv + (hd - ra.Hq)) * (long)(KV_BS * D);
            *reinterpret_cast<bf16x4*>(kb + k_index(off, d, D)) = o1;
            *reinterpret_cast<bf16x4*>(kb + k_index(off, 64 + d, D)) = o2;
          }
        }
      } else {
        bf16* vb = ra.v_cache + (blk * ra.Hkv + (hd - ra.Hq - ra.Hkv)) * (long)(KV_BS * D);
#pragma unroll
        for (int f = 0; f < 8; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r) vb[v_index(off, f * 16 + 4 * g + r, D)] = (bf16)acc[f][t][r];
      }
    } else if constexpr (EPI == EPI_SILU) {
      // row group G (16 W rows) is gate (G even) / up (G odd) of output columns 16*(G/2)..+15: the
      // wave's 8 groups give 4 output groups of 16 columns, col0 + 16p
      const int col0 = ((n0 + wa * 128) >> 5) * 16;
      bf16x4 o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // same roundings as GEMM -> bf16 gate|up -> silu_mul (HF: silu in the activation dtype)
          const float gt = (float)(bf16)acc[2 * q][t][r], up = (float)(bf16)acc[2 * q + 1][t][r];
          o[q][r] = (bf16)((float)(bf16)(gt / (1.f + __expf(-gt))) * up);
        }
      bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + col0 + lane_off;
#pragma unroll
      for (int q = 0; q < 4; q += 2) *reinterpret_cast<uint4*>(y + 16 * q) = pair16(o[q], o[q + 1]);
    } else if constexpr (EPI == EPI_SLAB) {
      float* P = static_cast<float*>(Y) + (long)s * M * N + (long)m * N;
#pragma unroll
      for (int f = 0; f < 8; ++f) *reinterpret_cast<f32x4*>(P + n0 + wa * 128 + f * 16 + 4 * g) = acc[f][t];
    } else {
      bf16* y = static_cast<bf16*>(Y) + (long)m * ldy + n0 + wa * 128 + lane_off;
#pragma unroll
      for (int f = 0; f < 8; f += 2) {
        bf16x4 lo, hi;
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
          const int n = n0 + wa * 128 + f * 16 + 4 * g;
          const bf16x4 b0 = *reinterpret_cast<const bf16x4*>(R + n), b1 = *reinterpret_cast<const bf16x4*>(R + n + 16);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // rounded where GEMM-with-bias -> bf16 -> GELU rounds (F.linear(x, w, b) then gelu)
            float u0 = (float)(bf16)(acc[f][t][r] + (float)b0[r]), u1 = (float)(bf16)(acc[f + 1][t][r] + (float)b1[r]);
            if constexpr (EPI == EPI_BIAS_GELU) {
              u0 = 0.5f * u0 * (1.f + erff(u0 * 0.70710678118654752f));
              u1 = 0.5f * u1 * (1.f + erff(u1 * 0.70710678118654752f));
            }
            lo[r] = (bf16)u0, hi[r] = (bf16)u1;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) lo[r] = (bf16)acc[f][t][r], hi[r] = (bf16)acc[f + 1][t][r];
        }
        Pack8 v;
        v.u = pair16(lo, hi);
        if constexpr (EPI == EPI_RESID) {
          Pack8 rr;
          rr.u = *reinterpret_cast<const uint4*>(R + (long)m * ldr + n0 + wa * 128 + lane_off + 16 * f);
#pragma unroll
          for (int j = 0; j < 8; ++j) v.e[j] = (bf16)((float)v.e[j] + (float)rr.e[j]);
        }
        *reinterpret_cast<uint4*>(y + 16 * f) = v.u;
      }
    }
  }
}

}  // namespace

#undef READ_W

// token tiles per L2 group of the bf16 launches below (0: GM); an A/B knob (bench/kernels.py gemm_group)
static int g_group = 0;

template <int EPI, int ABL = 0, int BAL = 1, bool WT = false>
static void launch(dim3 grid, hipStream_t stream, const void* X, int ldx, const void* W, int K, void* Y, int ldy,
                   const void* R, int ldr, int M, int N, int S, const RopeArgs& ra, TailArgs ta = TailArgs{}) {
  ta.gm = g_group;
  hipLaunchKernelGGL((gemm_prefill_kernel<EPI, ABL, BAL, false, WT>), grid, dim3(512), 0, stream, X, ldx, W, K, Y,
                     ldy, (const bf16*)R, ldr, M, N, S, ra, MoeArgs{}, SampleArgs{}, ta);
}

static dim3 grid_for(int M, int N, int S) { return dim3((unsigned)(((M + TM - 1) / TM) * (N / TN) * S)); }

// Tail plan for T tiles on `cus` CUs (S == 1 launches): L = T mod cus tiles split s = cus / L ways
// (>= 2, each split >= 16 K-tiles), workspace permitting (ws_floats >= L * s * 256 * 256, ncnt >= L).
// Returns the grid; ta.s <= 1 means no tail.
static dim3 tail_plan(int M, int N, int K, int cus, float* ws, long ws_floats, int* cnt, int ncnt, TailArgs& ta) {
  ta = TailArgs{};
  const int T = ((M + TM - 1) / TM) * (N / TN);
  if (cus > 0 && ws && cnt) {
    const int L = T % cus, ntot = K / BK;
    int s = L ? cus / L : 0;
    s = min(s, ntot / 16);          // >= 16 K-tiles per split: the f32 partial store + combine of a
                                    // 256x256 tile costs ~ a few K-tiles' time (bench/kernels.py gemm_tail)
    if (L && s >= 2 && L <= ncnt && (long)L * s * TM * TN <= ws_floats) {
      ta = TailArgs{T - L, L, s, ws, cnt};
      return dim3((unsigned)(T - L + L * s));
    }
  }
  return dim3((unsigned)T);
}

PENNY_API int penny_gemm_prefill_set_group(int gm) {
  if (gm < 0 || gm > 64) return (int)hipErrorInvalidValue;
  g_group = gm;
  return 0;
}

// Contract (checked): N % 256 == 0, K % (64*S) == 0, ldx % 8 == 0, rows 16-B aligned; EPI_SILU
// needs S == 1 and ldy % 8 == 0 (Y is [M, N/2]); EPI_SLAB writes P [S, M, N] f32 (ldy unused);
// EPI_RESID needs R (row stride ldr, ldr % 8 == 0) and S == 1; EPI_BIAS(_GELU) take the bias [N]
// as R.
// tail_ws / tail_cnt / cus (optional, null / 0: off): the wave-quantisation tail's workspace (f32
// [tail_ws_floats]), its zero-initialised ticket counters [tail_ncnt] and the device's CU count;
// one workspace per stream (launches on one stream run in order, the counters reset themselves).
PENNY_API int penny_gemm_prefill(const void* X, int ldx, const void* W, int K, void* Y, int ldy, const void* R,
                                 int ldr, int M, int N, int S, int epi, float* tail_ws, long tail_ws_floats,
                                 int* tail_cnt, int tail_ncnt, int cus, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % TN || S < 1 || K % (BK * S) || ldx % 8 || epi < 0 || epi > 6 || epi == EPI_ROPE)
    return (int)hipErrorInvalidValue;
  if (epi != EPI_SLAB && (S != 1 || ldy % 8)) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID && (!R || ldr % 8)) return (int)hipErrorInvalidValue;
  if ((epi == EPI_BIAS || epi == EPI_BIAS_GELU) && !R) return (int)hipErrorInvalidValue;
  if ((long)((M + TM - 1) / TM) * (N / TN) * S > (1L << 30)) return (int)hipErrorInvalidValue;
  TailArgs ta{};
  const dim3 grid = S == 1 ? tail_plan(M, N, K, cus, tail_ws, tail_ws_floats, tail_cnt, tail_ncnt, ta)
                           : grid_for(M, N, S);
  const RopeArgs ra{};
  switch (epi) {
    case EPI_BF16: launch<EPI_BF16>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    case EPI_SILU: launch<EPI_SILU>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    case EPI_SLAB: launch<EPI_SLAB>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra); break;
    case EPI_BIAS: launch<EPI_BIAS>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    case EPI_BIAS_GELU: launch<EPI_BIAS_GELU>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    default: launch<EPI_RESID>(grid, stream, X, ldx, W, K, Y, ldy, R, ldr, M, N, S, ra, ta);
  }
  return (int)hipGetLastError();
}

// penny_gemm_prefill on the fragment-tiled weight (ops/gemm.py tile_weight: [N/16, K/32, 64, 8]) instead
// of the row-major one -- the layout the decode kernels stream, so a shape could keep ONE copy.
// Epilogues BF16 / SILU / SLAB / RESID; same contract otherwise.
PENNY_API int penny_gemm_prefill_wt(const void* X, int ldx, const void* Wt, int K, void* Y, int ldy, const void* R,
                                    int ldr, int M, int N, int S, int epi, float* tail_ws, long tail_ws_floats,
                                    int* tail_cnt, int tail_ncnt, int cus, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % TN || S < 1 || K % (BK * S) || ldx % 8 || (epi != EPI_BF16 && epi != EPI_SILU && epi != EPI_SLAB &&
                                                    epi != EPI_RESID))
    return (int)hipErrorInvalidValue;
  if (epi != EPI_SLAB && (S != 1 || ldy % 8)) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID && (!R || ldr % 8)) return (int)hipErrorInvalidValue;
  TailArgs ta{};
  const dim3 grid = S == 1 ? tail_plan(M, N, K, cus, tail_ws, tail_ws_floats, tail_cnt, tail_ncnt, ta)
                           : grid_for(M, N, S);
  const RopeArgs ra{};
  switch (epi) {
    case EPI_BF16: launch<EPI_BF16, 0, 1, true>(grid, stream, X, ldx, Wt, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    case EPI_SILU: launch<EPI_SILU, 0, 1, true>(grid, stream, X, ldx, Wt, K, Y, ldy, R, ldr, M, N, S, ra, ta); break;
    case EPI_SLAB: launch<EPI_SLAB, 0, 1, true>(grid, stream, X, ldx, Wt, K, Y, ldy, R, ldr, M, N, S, ra); break;
    default: launch<EPI_RESID, 0, 1, true>(grid, stream, X, ldx, Wt, K, Y, ldy, R, ldr, M, N, S, ra, ta);
  }
  return (int)hipGetLastError();
}

// Fused QKV projection + RoPE + paged KV write (head dim 128): W [(Hq + 2*Hkv)*128, K] (q heads,
// k heads, v heads), positions / slots [M] int32, cos_sin [max_pos, 128] f32, q_out [M, Hq, 128].
// Contract (checked): N == (Hq + 2*Hkv)*128, N % 256 == 0, K % 64 == 0, ldx % 8 == 0.
PENNY_API int penny_gemm_prefill_qkv_rope(const void* X, int ldx, const void* W, int K, int M, const int* positions,
                                          const float* cos_sin, const int* slots, void* q_out, void* k_cache,
                                          void* v_cache, int Hq, int Hkv, float qscale, float* tail_ws,
                                          long tail_ws_floats,
                                          int* tail_cnt, int tail_ncnt, int cus, hipStream_t stream) {
  if (M <= 0) return 0;
  const int N = (Hq + 2 * Hkv) * 128;
  if (Hq <= 0 || Hkv <= 0 || N % TN || K % BK || ldx % 8 || !positions || !cos_sin || !slots || !q_out)
    return (int)hipErrorInvalidValue;
  const RopeArgs ra{positions, cos_sin, slots, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, Hq, Hkv, qscale};
  TailArgs ta{};
  const dim3 grid = tail_plan(M, N, K, cus, tail_ws, tail_ws_floats, tail_cnt, tail_ncnt, ta);
  launch<EPI_ROPE>(grid, stream, X, ldx, W, K, nullptr, 0, nullptr, 0, M, N, 1, ra, ta);
  return (int)hipGetLastError();
}

// Diagnostic: bf16-epilogue GEMM with part of the K loop removed (ablate 1: LDS-DMA, 2: fragment
// reads).  Results are WRONG by construction; bench/kernels.py gemm_ablate uses the timings only.
PENNY_API int penny_gemm_prefill_ablate(const void* X, int ldx, const void* W, int K, void* Y, int ldy, int M, int N,
                                        int ablate, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % TN || K % BK || ldx % 8 || ldy % 4) return (int)hipErrorInvalidValue;
  const RopeArgs ra{};
  if (ablate == 1) launch<EPI_BF16, 1>(grid_for(M, N, 1), stream, X, ldx, W, K, Y, ldy, nullptr, 0, M, N, 1, ra);
  else if (ablate == 10) launch<EPI_BF16, 0, 0>(grid_for(M, N, 1), stream, X, ldx, W, K, Y, ldy, nullptr, 0, M, N, 1, ra);
  else if (ablate == 3) launch<EPI_BF16, 3>(grid_for(M, N, 1), stream, X, ldx, W, K, Y, ldy, nullptr, 0, M, N, 1, ra);
  else if (ablate == 2) launch<EPI_BF16, 2>(grid_for(M, N, 1), stream, X, ldx, W, K, Y, ldy, nullptr, 0, M, N, 1, ra);
  else launch<EPI_BF16, 0>(grid_for(M, N, 1), stream, X, ldx, W, K, Y, ldy, nullptr, 0, M, N, 1, ra);
  return (int)hipGetLastError();
}

// Grouped fp8 x fp8 MoE GEMM over expert buckets at prefill sizes (K13), no host round trip:
//   epi 7 (GEMM1): Y[p, N/2] = silu(gate) * up of X[rows[p]] (fp8 [T, K], row scales xs[token]) x
//                  W13_e (fp8 [E, N, K] row-major, 16-row gate|up interleave, row scales ws [E, N])
//   epi 8 (GEMM2): Y[p, N] = X[p] (fp8 [P, K], scales xs[p]) x W2_e * route_w[p]
// offsets [E+1] int32 on the device (bucket bounds of the P sorted rows).  Grid: (ceil(P/256) + E)
// token tiles x N/256 -- an upper bound of the per-expert tile counts; surplus workgroups exit.
// Contract (checked): N % 256 == 0, K % 128 == 0, ldx % 16 == 0, ldy % 8 == 0.
PENNY_API int penny_moe_gemm_prefill_fp8(const void* X, int ldx, const int* rows, const float* xs, const int* offsets,
                                         const void* W, const float* ws, const float* route_w, void* Y, int ldy,
                                         int P, int E, int N, int K, int epi, hipStream_t stream) {
  if (P <= 0) return 0;
  // epi + 16: the plain 12/4/8/0 fragment-read schedule (A/B reference) instead of the balanced one
  const bool plain = epi >= 16;
  epi &= 15;
  if (N % TN || K % 128 || ldx % 16 || ldy % 8 || E <= 0 || E > 256 || !offsets || !xs || !ws)
    return (int)hipErrorInvalidValue;
  if ((epi != EPI_MOE_SILU && epi != EPI_MOE_ROUTE) || (epi == EPI_MOE_ROUTE && !route_w)) return (int)hipErrorInvalidValue;
  const MoeArgs ma{offsets, rows, xs, ws, route_w, E, nullptr, 0};
  const dim3 grid((unsigned)(((P + TM - 1) / TM + E) * (N / TN)));
#define MOE_TILE(EPI_, BAL_)                                                                                    \
  hipLaunchKernelGGL((gemm_prefill_kernel<EPI_, 0, BAL_, true>), grid, dim3(512), 0, stream, X, ldx, W, K, Y, ldy, \
                     (const bf16*)nullptr, 0, P, N, 1, RopeArgs{}, ma, SampleArgs{}, TailArgs{})
  if (plain) {
    if (epi == EPI_MOE_SILU) MOE_TILE(EPI_MOE_SILU, 0);
    else MOE_TILE(EPI_MOE_ROUTE, 0);
  } else {
    if (epi == EPI_MOE_SILU) MOE_TILE(EPI_MOE_SILU, 1);
    else MOE_TILE(EPI_MOE_ROUTE, 1);
  }
#undef MOE_TILE
  return (int)hipGetLastError();
}

// The MX hand-off between the two grouped GEMMs of an fp8 MoE layer (no per-row quantisation pass
// between them):
//   epi 10 (GEMM1): X = routed token rows (fp8, row scales xs, gathered by rows), W = W13 [E, 2F, H];
//                   Y = the SiLU(gate) * up intermediate as e4m3 bytes [P, F] (ldy = F) and its
//                   E8M0 block scales into mxs (one per 32 columns; layout: MoeArgs::mxs);
//   epi 11 (GEMM2): X = that intermediate [P, F] (ldx = F) with mxs, W = W2 [E, H, F];
//                   Y[p, H] bf16 = (X x W2_e) * ws2 * route_w[p].
// mxs holds ((P + 255) / 256 + E) * (F / 128) KiB; nkt = F / 128.  Contract as above.
PENNY_API int penny_moe_gemm_prefill_fp8_mx(const void* X, int ldx, const int* rows, const float* xs,
                                            const int* offsets, const void* W, const float* ws, const float* route_w,
                                            void* Y, int ldy, int P, int E, int N, int K, int epi, unsigned* mxs,
                                            int nkt, hipStream_t stream) {
  if (P <= 0) return 0;
  if (N % TN || K % 128 || ldx % 16 || ldy % 8 || E <= 0 || E > 256 || !offsets || !ws || !mxs || nkt <= 0)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_MOE_SILU_MX) {
    if (!xs || nkt != N / 256) return (int)hipErrorInvalidValue;
  } else if (epi == EPI_MOE_ROUTE_MX) {
    if (!route_w || nkt != K / 128) return (int)hipErrorInvalidValue;
  } else {
    return (int)hipErrorInvalidValue;
  }
  MoeArgs ma{offsets, rows, xs, ws, route_w, E, nullptr, 0};
  ma.mxs = mxs;
  ma.nkt = nkt;
  const dim3 grid((unsigned)(((P + TM - 1) / TM + E) * (N / TN)));
  if (epi == EPI_MOE_SILU_MX)
    hipLaunchKernelGGL((gemm_prefill_kernel<EPI_MOE_SILU_MX, 0, 1, true>), grid, dim3(512), 0, stream, X, ldx, W, K,
                       Y, ldy, (const bf16*)nullptr, 0, P, N, 1, RopeArgs{}, ma, SampleArgs{}, TailArgs{});
  else
    hipLaunchKernelGGL((gemm_prefill_kernel<EPI_MOE_ROUTE_MX, 0, 1, true>), grid, dim3(512), 0, stream, X, ldx, W, K,
                       Y, ldy, (const bf16*)nullptr, 0, P, N, 1, RopeArgs{}, ma, SampleArgs{}, TailArgs{});
  return (int)hipGetLastError();
}

// Probe of the block-scaled MFMA's scale operands (one wave, one v_mfma_scale_f32_16x16x128_f8f6f4):
// A, B: 64 lanes x 32 e4m3 bytes (lane l: row l & 15, k-block l >> 4), sa / sb: one 32-bit scale
// word per lane, out: the 64 x 4 accumulator.  tests/test_kernels_gpu.py pins the lane / byte
// semantics the MX hand-off relies on.
template <int OPSEL>
__global__ void __launch_bounds__(64) mfma_scale_probe_kernel(const int* __restrict__ A, const int* __restrict__ B,
                                                               const int* __restrict__ sa, const int* __restrict__ sb,
                                                               float* __restrict__ out) {
  const int lane = threadIdx.x;
  i32x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = A[lane * 8 + i], b[i] = B[lane * 8 + i];
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa[lane], OPSEL, sb[lane]);
#pragma unroll
  for (int r = 0; r < 4; ++r) out[lane * 4 + r] = acc[r];
}

PENNY_API int penny_probe_mfma_scale(const int* A, const int* B, const int* sa, const int* sb, float* out, int opsel,
                                     hipStream_t stream) {
  switch (opsel) {
    case 0: hipLaunchKernelGGL(mfma_scale_probe_kernel<0>, dim3(1), dim3(64), 0, stream, A, B, sa, sb, out); break;
    case 1: hipLaunchKernelGGL(mfma_scale_probe_kernel<1>, dim3(1), dim3(64), 0, stream, A, B, sa, sb, out); break;
    case 2: hipLaunchKernelGGL(mfma_scale_probe_kernel<2>, dim3(1), dim3(64), 0, stream, A, B, sa, sb, out); break;
    case 3: hipLaunchKernelGGL(mfma_scale_probe_kernel<3>, dim3(1), dim3(64), 0, stream, A, B, sa, sb, out); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Reduce a row's (score, token) partials of the fused LM head (EPI_SAMPLE) to its sampled token:
// one 256-thread workgroup per row, ties to the smallest token id (sample_final_kernel's rule).
__global__ void __launch_bounds__(256) lm_sample_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                              int P, int* __restrict__ out, int* __restrict__ pairs) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = threadIdx.x; j < P; j += 256) better(bv, bi, pv[(long)row * P + j], pi[(long)row * P + j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sv[w] = bv;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) better(bv, bi, sv[k], si[k]);
    if (out) out[row] = bi;
    if (pairs) {   // (score bits, token id): a vocab shard's candidate for the cross-rank pick
      pairs[2 * row] = __float_as_int(bv);
      pairs[2 * row + 1] = bi;
    }
  }
}

PENNY_API int penny_lm_sample_final(const float* pv, const int* pi, int P, int M, int* out, int* pairs,
                                    hipStream_t stream) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(lm_sample_final_kernel, dim3(M), dim3(256), 0, stream, pv, pi, P, out, pairs);
  return (int)hipGetLastError();
}

// LM head + sampler fused (K11 + K12): out[m] = Gumbel-max / argmax sample of row m of
// X [M, K] bf16 x W [V, K]^T, temps [M] f32 (<= 0: greedy), seeds [M] u64 -- the [M, V] logits are
// never written.  workspace: M * 2 * (V / 256) floats, then as many ints.
// Contract (checked): V % 256 == 0, K % 64 == 0, ldx % 8 == 0, M >= 1.
PENNY_API int penny_lm_head_sample(const void* X, int ldx, const void* W, int K, int M, int V, const float* temps,
                                   const unsigned long long* seeds, void* workspace, int* out, hipStream_t stream) {
  if (M <= 0) return 0;
  if (V % TN || K % BK || ldx % 8 || !temps || !seeds || !workspace || !out) return (int)hipErrorInvalidValue;
  const int P = 2 * (V / TN);
  float* pv = static_cast<float*>(workspace);
  int* pi = reinterpret_cast<int*>(pv + (long)M * P);
  const SampleArgs sa{temps, seeds, pv, pi, 0, V};
  hipLaunchKernelGGL((gemm_prefill_kernel<EPI_SAMPLE>), grid_for(M, V, 1), dim3(512), 0, stream, X, ldx, W, K,
                     nullptr, 0, (const bf16*)nullptr, 0, M, V, 1, RopeArgs{}, MoeArgs{}, sa, TailArgs{});
  hipLaunchKernelGGL(lm_sample_final_kernel, dim3(M), dim3(256), 0, stream, pv, pi, P, out, (int*)nullptr);
  return (int)hipGetLastError();
}

// Vocabulary-parallel form (a TP rank's LM-head shard, SURVEY C2 "per-rank top-k then gather"):
// W [Vpad, K] holds vocabulary rows voff .. voff + vvalid - 1 (rows vvalid .. Vpad - 1 padding),
// and pairs [M, 2] int32 receives each row's best (score bits, GLOBAL token id) -- the noise is
// keyed by the global id, so the best pair over the shards is exactly the TP = 1 sample.
// Contract (checked): Vpad % 256 == 0, 0 < vvalid <= Vpad, K % 64 == 0, ldx % 8 == 0.
PENNY_API int penny_lm_head_sample_shard(const void* X, int ldx, const void* W, int K, int M, int Vpad, int vvalid,
                                         int voff, const float* temps, const unsigned long long* seeds,
                                         void* workspace, int* pairs, hipStream_t stream) {
  if (M <= 0) return 0;
  if (Vpad % TN || vvalid <= 0 || vvalid > Vpad || voff < 0 || K % BK || ldx % 8 || !temps || !seeds ||
      !workspace || !pairs)
    return (int)hipErrorInvalidValue;
  const int P = 2 * (Vpad / TN);
  float* pv = static_cast<float*>(workspace);
  int* pi = reinterpret_cast<int*>(pv + (long)M * P);
  const SampleArgs sa{temps, seeds, pv, pi, voff, vvalid};
  hipLaunchKernelGGL((gemm_prefill_kernel<EPI_SAMPLE>), grid_for(M, Vpad, 1), dim3(512), 0, stream, X, ldx, W, K,
                     nullptr, 0, (const bf16*)nullptr, 0, M, Vpad, 1, RopeArgs{}, MoeArgs{}, sa, TailArgs{});
  hipLaunchKernelGGL(lm_sample_final_kernel, dim3(M), dim3(256), 0, stream, pv, pi, P, (int*)nullptr, pairs);
  return (int)hipGetLastError();
}
