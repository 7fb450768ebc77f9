// K6 (paged prefill / varlen, causal or bidirectional) and K7 (paged split-K decode) attention
// for gfx950, on v_mfma_f32_16x16x32_bf16 with f32 online softmax.
//
// Orientation (see kv_layout.h): scores are computed TRANSPOSED, S^T = K . Q^T, so a lane holds
// one query column and 16 keys in registers; the P.V product is O^T = V^T . P^T and takes P
// straight from those registers (no LDS round trip for P).  The KV cache is stored in
// MFMA-fragment-native order, so every K/V operand fragment is one contiguous 16-B piece at
// (64*fragment + lane)*16 inside a block tile.
//
// GQA packing: the G = Hq/Hkv query heads that share a kv head are packed into the MFMA's 16
// query columns (decode) or into the 128 "rows" of a prefill tile (rows = token*G + head), so
// every K/V byte staged is used by all G heads.
//
// Prefill: one workgroup = 4 waves = 128 (token, head) rows of one sequence and one kv head.
// K and V blocks (64 keys) are staged into LDS with lane-linear global_load_lds (the tile is
// already in fragment order, so no swizzle and no staging registers), double-buffered: block
// j+1 is requested before block j's MFMAs, one barrier per block.  Fragment reads are
// consecutive-lane ds_read_b128 (conflict-free).  ~64 KiB LDS and <=256 VGPRs per wave let two
// workgroups share a CU, so one workgroup's softmax VALU overlaps the other's MFMAs.
//
// Decode: one workgroup = 4 waves = one (sequence, kv head, partition of PB blocks).  Each wave
// streams whole 64-key blocks straight into VGPRs with 1-KiB coalesced loads (decode is
// HBM-bound; an LDS hop is pure overhead: the 'GEMV / M <= 16' row of the guide), the 4 waves
// merge through LDS, and a second kernel merges partitions (flash-decoding split-K).  The grid
// runs the sequence index fastest so the workgroups that read the SAME shared-prefix blocks
// (every turn's system prompt is a prefix-cache hit) are in flight together and hit in L2/MALL.
#include "common.h"

#include <type_traits>

#include <cstdlib>
#include "kv_layout.h"

#define LOG2E 1.4426950408889634f

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

union Frag {
  uint4 u;
  bf16x8 v;
};

// Raw v_exp_f32: exp2f() wraps it in a denormal-range fix-up (cmp, 2x cndmask, ldexp) -- 5 VALU
// ops per score instead of 1.  Softmax terms below 2^-126 are irrelevant (they add to l and O
// below f32 resolution of the running max term), so the flush is harmless.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Reductions over the 4 lanes {l, l^16, l^32, l^48} (the 4 row groups of a 16x16 MFMA tile) on
// the gfx950 VALU lane swaps.  permlane16_swap(v, v) leaves rows (0,0,2,2) in one result and
// (1,1,3,3) in the other, so combining the two is the xor-16 step; permlane32_swap the xor-32
// one.  __shfl_xor compiles to ds_bpermute: an LDS round trip on the softmax's critical path.
__device__ __forceinline__ float rowgroup_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// rowgroup_max without the canonicalising v_max_f32 x, x, x hipcc puts in front of fmaxf on each
// permlane result (4 extra VALU per call): the operands are finite scores or -inf, never sNaN
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float rowgroup_max_raw(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax_raw(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_raw(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rowgroup_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// Prefill
// ------------------------------------------------------------------------------------------
// One 64-key block for a wave's 32 query rows (2 column tiles of 16): S^T = K.Q^T on MFMA,
// base-2 online softmax in registers, O^T += V^T.P^T with P straight from the S^T registers.
// kl / vl: the block's K and V tiles in LDS (fragment-native).  `full`: no key of the block needs
// masking (all < ctx and, if causal, <= every row's position).
// The masking is one wave-uniform branch around a select loop: a per-element `full || (...)`
// short-circuit compiles to 32 divergent branches per block on gfx950.
// MASK: 0 never, 1 always, 2 when the wave-uniform runtime flag `need_mask` is set.  Mode 2 keeps
// ONE copy of the MFMA code in the loop: with two inlined copies (one per mode, behind an if/else)
// the accumulators meet at a join point and hipcc materialises the merge as v_mov_b64 copies of
// MFMA results (each one waits for its MFMA to retire), ~64 per block.
template <int D, int MASK, bool PREF = false, bool SB = false>
__device__ __forceinline__ void attend_block(const uint4* __restrict__ kl, const uint4* __restrict__ vl,
                                             const Frag (&qf)[2][D / 32], f32x4 (&o)[2][D / 16], float (&m)[2],
                                             float (&l)[2], bool causal, int j, int ctx,
                                             const int (&qpos)[2], float scale_log2, int lane, int g,
                                             bool need_mask = false) {
  constexpr int KC = D / 32;
  constexpr int DT = D / 16;
  // ---- S^T = K . Q^T for 64 keys x 32 query rows -------------------------------------
  f32x4 sc[2][4];
  Frag kfa[PREF ? 4 * KC : 1], vfa[PREF ? 2 * DT : 1];
  if constexpr (PREF) {
#pragma unroll
    for (int f = 0; f < 4 * KC; ++f) kfa[f].u = kl[f * 64 + lane];
    // SB: pin the 16 reads ahead of the MFMAs -- hipcc otherwise sinks each pair next to its use
    // and waits for it (lgkmcnt(0) every 2-4 MFMAs: the LDS latency exposed 8 times per block)
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    sc[0][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    sc[1][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      Frag kf;
      if constexpr (PREF) kf = kfa[t * KC + c];
      else kf.u = kl[(t * KC + c) * 64 + lane];
      sc[0][t] = mfma16(kf.v, qf[0][c].v, sc[0][t]);
      sc[1][t] = mfma16(kf.v, qf[1][c].v, sc[1][t]);
    }
  }
  // PREF (the 8-wave kernel, 1 workgroup per CU: registers to spare): all 16 K fragments of the
  // block are read before the QK^T MFMAs and all 16 V fragments right after them, so the V reads
  // are in flight during the softmax instead of exposed in front of each P.V pair (+2-5 %,
  // profiles/r2_prefill_attn_kv_prefetch_ab.jsonl)
  if constexpr (PREF) {   // V fragments in flight while the softmax runs
#pragma unroll
    for (int f = 0; f < 2 * DT; ++f) vfa[f].u = vl[f * 64 + lane];
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  }

  // ---- online softmax (base-2) -------------------------------------------------------
  Frag pf[2][2];
  if (MASK == 1 || (MASK == 2 && need_mask)) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = j * KV_BS + 16 * t + 4 * g + r;
          const bool ok = (key < ctx) & ((!causal) | (key <= qpos[ct]));   // non-short-circuit: selects
          sc[ct][t][r] = ok ? sc[ct][t][r] : -INFINITY;
        }
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) mt = fmaxf(mt, sc[ct][t][r]);
    }
    mt = rowgroup_max(mt);
    mt *= scale_log2;   // max of the scaled scores (scale > 0) -- the 32 scores stay unscaled
    // Deferred rescale: the running max m only moves when a block raises it by more than 8
    // (log2 domain), so p <= 2^8 in between -- harmless for f32 l/O and bf16 P -- and the 64
    // multiplies of O (plus l) run on the rare blocks that need them, behind a wave-uniform branch.
    const bool grow = mt > m[ct] + 8.f;
    if (__any(grow)) {
      const float mn = grow ? mt : m[ct];
      const float alpha = grow ? fast_exp2(m[ct] - mn) : 1.f;
      l[ct] *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[ct][dt] *= alpha;
      m[ct] = mn;
    }
    const float mref = (m[ct] == -INFINITY) ? 0.f : m[ct];
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fast_exp2(fmaf(sc[ct][t][r], scale_log2, -mref));
        sc[ct][t][r] = p;
        ls += p;
      }
    }
    l[ct] += ls;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[ct][st].v[r] = (bf16)sc[ct][2 * st][r];
        pf[ct][st].v[4 + r] = (bf16)sc[ct][2 * st + 1][r];
      }
    }
  }

  // ---- O^T += V^T . P^T ---------------------------------------------------------------
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      Frag vf;
      if constexpr (PREF) vf = vfa[dt * 2 + st];
      else vf.u = vl[(dt * 2 + st) * 64 + lane];
      o[0][dt] = mfma16(vf.v, pf[0][st].v, o[0][dt]);
      o[1][dt] = mfma16(vf.v, pf[1][st].v, o[1][dt]);
    }
  }
}

// attend_block with the softmax's VALU work cut (prefill2 FOLD, the default big-tile path).  Per block
// and wave the plain form issues ~170 VALU instructions beside its 64 MFMAs (32 v_exp, 32 FMAs of
// scale-and-subtract, a 16-deep serial add chain per column tile for the row sums, 32 max) -- with
// two waves per SIMD the issue slots, not the matrix pipe, bound the loop
// (profiles/r4_prefill_attn_mfma_busy_pmc.md: 31 % MFMA-busy, 4.3 VALU per MFMA).  Here:
//   * Q arrives prescaled by scale*log2(e) (the caller's qf), and each S^T accumulator chain STARTS
//     at -m (the running max, log2 units), so the MFMAs leave s' = s*c - m ready for v_exp: no
//     per-score FMA.  A block whose max rises by more than 8 (or the row's first live block, m still
//     -inf: chains start at 0) takes the rare branch that moves m and subtracts the rise from its
//     scores (T13's defer-max, the decision taken BEFORE any of this block's P is formed, and O and
//     the row sums rescaled together);
//   * the row sums come out of the matrix pipe: one extra MFMA per (column tile, k-step) with an
//     all-ones A operand (16 identical rows of sum_k P[q][k]) accumulates l in f32x4 `la` -- of the
//     bf16-rounded P that the P.V product uses, so numerator and denominator see the same p;
//   * the 4 lanes of a row group hold the same l, so no cross-lane reduction at the end.
// 68 MFMAs and ~100 VALU per block and wave instead of 64 and ~170.
// QPRE = false keeps Q exact (no extra rounding of q*c): the chains start at 0 and each score takes
// one FMA (s*c - m) before its v_exp, as in attend_block; the row-sum MFMAs and the lean max / grow
// logic are the same.  QPRE = true is the prescaled-Q form above: ~32 fewer VALU per block, but
// bf16(q*c) perturbs each score by ~2^-9 of |s*c|, which shows on very peaky rows (scores of std
// ~17 log2 units: max error 0.08 vs the fp32 reference where the exact form holds 0.02) -- opt-in.
template <int D, int MASK, bool SB = false, bool QPRE = false>
__device__ __forceinline__ void attend_block_fold(const uint4* __restrict__ kl, const uint4* __restrict__ vl,
                                                  const Frag (&qf)[2][D / 32], f32x4 (&o)[2][D / 16],
                                                  float (&m)[2], f32x4 (&la)[2], bool causal, int j, int ctx,
                                                  const int (&qpos)[2], float scale_log2, int lane, int g,
                                                  bool need_mask = false) {
  constexpr int KC = D / 32;
  constexpr int DT = D / 16;
  Frag kfa[4 * KC], vfa[2 * DT];
#pragma unroll
  for (int f = 0; f < 4 * KC; ++f) kfa[f].u = kl[f * 64 + lane];
  if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  // chains start at -m: the MFMAs deliver s*c - m (m = -inf, a row's first live block: start at 0,
  // and any finite max is a "rise")
  float m0[2], thr[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const bool fresh = m[ct] == -INFINITY;
    m0[ct] = (fresh || !QPRE) ? 0.f : -m[ct];
    thr[ct] = fresh ? -INFINITY : 8.f;
  }
  f32x4 sc[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    sc[0][t] = f32x4{m0[0], m0[0], m0[0], m0[0]};
    sc[1][t] = f32x4{m0[1], m0[1], m0[1], m0[1]};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      sc[0][t] = mfma16(kfa[t * KC + c].v, qf[0][c].v, sc[0][t]);
      sc[1][t] = mfma16(kfa[t * KC + c].v, qf[1][c].v, sc[1][t]);
    }
  }
#pragma unroll
  for (int f = 0; f < 2 * DT; ++f) vfa[f].u = vl[f * 64 + lane];
  if constexpr (SB) __builtin_amdgcn_sched_barrier(0);

  if (MASK == 1 || (MASK == 2 && need_mask)) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = j * KV_BS + 16 * t + 4 * g + r;
          const bool ok = (key < ctx) & ((!causal) | (key <= qpos[ct]));
          sc[ct][t][r] = ok ? sc[ct][t][r] : -INFINITY;
        }
  }
  Frag pf[2][2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mt = fmaxf(mt, sc[ct][t][r]);
    mt = rowgroup_max_raw(mt);              // QPRE: max of s*c - m; else max of s
    if constexpr (!QPRE) mt = m[ct] == -INFINITY ? mt * scale_log2 : mt * scale_log2 - m[ct];
    const bool grow = mt > thr[ct];
    if (__any(grow)) {
      const bool first = m[ct] == -INFINITY;
      const float rise = grow ? mt : 0.f;
      if (grow) {
        const float alpha = first ? 1.f : fast_exp2(-rise);   // first: O and l are still 0
        la[ct] *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[ct][dt] *= alpha;
        m[ct] = first ? rise : m[ct] + rise;
      }
      if constexpr (QPRE) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) sc[ct][t][r] -= rise;
      }
    }
    if constexpr (QPRE) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[ct][t][r] = fast_exp2(sc[ct][t][r]);
    } else {
      const float mref = m[ct] == -INFINITY ? 0.f : m[ct];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[ct][t][r] = fast_exp2(fmaf(sc[ct][t][r], scale_log2, -mref));
    }
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[ct][st].v[r] = (bf16)sc[ct][2 * st][r];
        pf[ct][st].v[4 + r] = (bf16)sc[ct][2 * st + 1][r];
      }
  }
  // ---- O^T += V^T . P^T, and l += 1 . P^T on the matrix pipe --------------------------------
  Frag ones;
  ones.u = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);   // bf16 1.0 x 8
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      o[0][dt] = mfma16(vfa[dt * 2 + st].v, pf[0][st].v, o[0][dt]);
      o[1][dt] = mfma16(vfa[dt * 2 + st].v, pf[1][st].v, o[1][dt]);
    }
  }
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    la[0] = mfma16(ones.v, pf[0][st].v, la[0]);
    la[1] = mfma16(ones.v, pf[1][st].v, la[1]);
  }
}

template <int D>
constexpr int prefill_smem_bytes() { return 4 * KV_BS * D * 2; }

// One 128-row (token*G + head) tile of sequence `s`, kv head `h` (4 waves x 32 rows): the short-chunk
// prefill path (<= 128 rows per sequence and kv head).
template <int D>
__device__ __forceinline__ void attend_tile(char* smem, const bf16* __restrict__ q, const int* __restrict__ cu_q,
                                            const int* __restrict__ ctx_lens, const int* __restrict__ block_tables,
                                            const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
                                            bf16* __restrict__ out, float scale_log2, int Hq, int Hkv,
                                            int max_blocks, int causal_arg, int s, int h, int tile,
                                            float* __restrict__ lse = nullptr) {
  constexpr int KC = D / 32;                 // k-chunks of the QK^T product
  constexpr int DT = D / 16;                 // 16-row dim tiles of O^T
  constexpr int TILE = KV_BS * D * 2;        // bytes of one K (or V) block tile
  constexpr int PIECES = TILE / 1024 / 4;    // 1-KiB glds pieces per wave per tile
  const bool causal = causal_arg;

  const int G = Hq / Hkv;
  const int TQ = 128 / G;
  const int q0 = cu_q[s], qlen = cu_q[s + 1] - q0;
  const int tok0 = tile * TQ;
  if (tok0 >= qlen) return;
  const int ctx = ctx_lens[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;

  int tok[2], head[2], qpos[2];
  Frag qf[2][KC];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int r = w * 32 + ct * 16 + col;
    tok[ct] = tok0 + r / G;
    head[ct] = h * G + r % G;
    const bool valid = tok[ct] < qlen;
    qpos[ct] = valid ? ctx - qlen + tok[ct] : ctx - 1;
    const int qi = q0 + (valid ? tok[ct] : 0);
    const bf16* qrow = q + ((long)qi * Hq + head[ct]) * D;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      qf[ct][c].u = valid ? *reinterpret_cast<const uint4*>(qrow + c * 32 + g * 8) : make_uint4(0, 0, 0, 0);
  }

  const int last_tok = min(tok0 + TQ, qlen) - 1;
  const int kv_end = causal ? min(ctx, ctx - qlen + last_tok + 1) : ctx;
  const int nblk = (kv_end + KV_BS - 1) / KV_BS;
  const int jb = 0, je = nblk;
  const int* bt = block_tables + (long)s * max_blocks;

  f32x4 o[2][DT];
  float m[2], l[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    m[ct] = -INFINITY;
    l[ct] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[ct][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // lane-linear global -> LDS copy of block j's K and V tiles into buffer `buf`
  auto stage = [&](int j, int buf) {
    const long phys = bt[j];
    PENNY_DASSERT(phys >= 0);
    const char* kb = reinterpret_cast<const char*>(k_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    const char* vb = reinterpret_cast<const char*>(v_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    char* kl = smem + buf * 2 * TILE;
    char* vl = kl + TILE;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = w * PIECES + i;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(kb + piece * 1024 + lane * 16), (lds_void_t*)(kl + piece * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(vb + piece * 1024 + lane * 16), (lds_void_t*)(vl + piece * 1024),
                                       16, 0, 0);
    }
  };

  if (je > jb) stage(jb, 0);
  __syncthreads();

  for (int j = jb; j < je; ++j) {
    const int buf = (j - jb) & 1;
    if (j + 1 < je) stage(j + 1, buf ^ 1);
    const uint4* kl = reinterpret_cast<const uint4*>(smem + buf * 2 * TILE);
    const uint4* vl = reinterpret_cast<const uint4*>(smem + buf * 2 * TILE + TILE);

    const bool full = (j + 1) * KV_BS <= ctx && (!causal || (j + 1) * KV_BS - 1 <= ctx - qlen + tok0);
    attend_block<D, 2>(kl, vl, qf, o, m, l, causal, j, ctx, qpos, scale_log2, lane, g,
                       __builtin_amdgcn_readfirstlane((int)!full) != 0);
    __syncthreads();  // block j+1 landed (vmcnt drained) and everyone is done with buffer `buf`
  }

  // ---- epilogue: finish row sums across the 4 lane groups, normalise, store -----------
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    float lt = l[ct];
    lt = rowgroup_sum(lt);
    if (tok[ct] >= qlen) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16* orow = out + ((long)(q0 + tok[ct]) * Hq + head[ct]) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      bf16x4 v4;
#pragma unroll
      for (int r = 0; r < 4; ++r) v4[r] = (bf16)(o[ct][dt][r] * inv);
      *reinterpret_cast<bf16x4*>(orow + 16 * dt + 4 * g) = v4;
    }
    if (lse != nullptr && g == 0)   // natural-log sum-exp of the scaled scores (ring-attention merge)
      lse[(long)(q0 + tok[ct]) * Hq + head[ct]] = lt > 0.f ? (m[ct] + __log2f(lt)) * 0.6931471805599453f : -INFINITY;
  }
}

template <int D>
__global__ void __launch_bounds__(256, 2) prefill_kernel(
    const bf16* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ block_tables, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    bf16* __restrict__ out, float scale_log2, int Hq, int Hkv, int max_blocks, int causal,
    float* __restrict__ lse) {
  __shared__ __attribute__((aligned(16))) char smem[prefill_smem_bytes<D>()];  // [buf][K|V]
  attend_tile<D>(smem, q, cu_q, ctx_lens, block_tables, k_cache, v_cache, out, scale_log2, Hq, Hkv, max_blocks,
                 causal, blockIdx.z, blockIdx.y, blockIdx.x, lse);
}

// ------------------------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------------------------
// HEAD_FAST: grid (Hkv, B, nparts) -- the kv head is the fastest-varying workgroup index, so with
// round-robin dispatch over the 8 XCDs (Hkv == 8 for every model served here) each XCD owns ONE
// kv head for every sequence and its 4 MB L2 holds that head's shared-prefix blocks (~0.5 MB per
// head per layer for a 1k-token system prompt).  Otherwise grid (B, nparts, Hkv), sequence
// fastest: each XCD streams whole sequences, whose 8 heads of a KV block are contiguous.
template <int D, bool HEAD_FAST>
__global__ void __launch_bounds__(256) decode_kernel(
    const bf16* __restrict__ q, const int* __restrict__ ctx_lens, const int* __restrict__ block_tables,
    const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache, bf16* __restrict__ out,
    float* __restrict__ part_m, float* __restrict__ part_l, float* __restrict__ part_o, float scale_log2, int Hq,
    int Hkv, int max_blocks, int pb, int nparts, int part_stride) {
  constexpr int KC = D / 32, DT = D / 16;
  __shared__ float s_m[4][16], s_l[4][16];
  __shared__ float s_o[4][16][D + 4];

  const int b = HEAD_FAST ? blockIdx.y : blockIdx.x;
  const int p = HEAD_FAST ? blockIdx.z : blockIdx.y;
  const int h = HEAD_FAST ? blockIdx.x : blockIdx.z;
  const int ctx = ctx_lens[b];
  const int nblk = (ctx + KV_BS - 1) / KV_BS;
  const int blk0 = p * pb;
  if (blk0 >= nblk) return;
  const int blk1 = min(blk0 + pb, nblk);
  const int G = Hq / Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;
  const int* bt = block_tables + (long)b * max_blocks;

  Frag qf[KC];
  {
    const bool valid = col < G;
    const bf16* qrow = q + ((long)b * Hq + h * G + (valid ? col : 0)) * D;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      qf[c].u = valid ? *reinterpret_cast<const uint4*>(qrow + c * 32 + g * 8) : make_uint4(0, 0, 0, 0);
  }

  f32x4 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  // This wave's block ids are fetched up front, one per lane (64 iterations per fetch), and read
  // back with v_readlane: a load of bt[j] at the top of every iteration put a dependent
  // global-memory round trip in front of each block's K/V loads.
  const int nit = blk1 - blk0 - w > 0 ? (blk1 - blk0 - w + 3) / 4 : 0;
  int ids = 0;
  for (int it = 0; it < nit; ++it) {
    if ((it & 63) == 0) {
      const int jl = blk0 + w + 4 * (it + lane);
      ids = jl < blk1 ? bt[jl] : 0;
    }
    const int j = blk0 + w + 4 * it;
    const int id = __builtin_amdgcn_readlane(ids, it & 63);
    const long phys = id < 0 ? -(long)id - 1 : id;     // < 0: marked shared (decode_lean_kernel)
    const uint4* kb = reinterpret_cast<const uint4*>(k_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    const uint4* vb = reinterpret_cast<const uint4*>(v_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    Frag kf[4][KC], vf[DT][2];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int c = 0; c < KC; ++c) kf[t][c].u = kb[(t * KC + c) * 64 + lane];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int st = 0; st < 2; ++st) vf[dt][st].u = vb[(dt * 2 + st) * 64 + lane];

    f32x4 sc[4];
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KC; ++c) sc[t] = mfma16(kf[t][c].v, qf[c].v, sc[t]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = j * KV_BS + 16 * t + 4 * g + r;
        const float v = key < ctx ? sc[t][r] * scale_log2 : -INFINITY;
        sc[t][r] = v;
        mt = fmaxf(mt, v);
      }
    }
    mt = rowgroup_max(mt);
    // deferred rescale as in prefill: m moves only when a block raises it by more than 8 (log2),
    // so the 32 accumulator multiplies (AGPR read-modify-write) run on the rare growing blocks
    const bool grow = mt > m + 8.f;
    if (__any(grow)) {
      const float mn = grow ? mt : m;
      const float alpha = grow ? fast_exp2(m - mn) : 1.f;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      m = mn;
    }
    const float mref = (m == -INFINITY) ? 0.f : m;
    float ls = 0.f;
    Frag pf[2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = fast_exp2(sc[t][r] - mref);
        ls += pv;
        pf[t >> 1].v[4 * (t & 1) + r] = (bf16)pv;
      }
    }
    l += ls;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      o[dt] = mfma16(vf[dt][0].v, pf[0].v, o[dt]);
      o[dt] = mfma16(vf[dt][1].v, pf[1].v, o[dt]);
    }
  }

  // merge the 4 waves through LDS
  l = rowgroup_sum(l);
  if (g == 0) {
    s_m[w][col] = m;
    s_l[w][col] = l;
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[w][col][16 * dt + 4 * g + r] = o[dt][r];
  __syncthreads();

  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int qc = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, s_m[ww][qc]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = s_m[ww][qc] == -INFINITY ? 0.f : exp2f(s_m[ww][qc] - M);
      L += s_l[ww][qc] * f;
      O += s_o[ww][qc][d] * f;
    }
    const int hq = h * G + qc;
    if (nparts == 1) {
      out[((long)b * Hq + hq) * D + d] = (bf16)(O / L);
    } else {
      const long pi = ((long)b * Hq + hq) * part_stride + p;
      part_o[pi * D + d] = O;
      if (d == 0) {
        part_m[pi] = M;
        part_l[pi] = L;
      }
    }
  }
}

template <int D>
__global__ void decode_reduce_kernel(const int* __restrict__ ctx_lens, const float* __restrict__ part_m,
                                     const float* __restrict__ part_l, const float* __restrict__ part_o,
                                     bf16* __restrict__ out, int Hq, int pb, int nparts, int part_stride) {
  const int b = blockIdx.y, hq = blockIdx.x, d = threadIdx.x;
  const int nblk = (ctx_lens[b] + KV_BS - 1) / KV_BS;
  const int np = min(nparts, (nblk + pb - 1) / pb);
  const long base = ((long)b * Hq + hq) * part_stride;
  float M = -INFINITY;
  for (int i = 0; i < np; ++i) M = fmaxf(M, part_m[base + i]);
  float L = 0.f, O = 0.f;
  for (int i = 0; i < np; ++i) {
    const float f = exp2f(part_m[base + i] - M);
    L += part_l[base + i] * f;
    O += part_o[(base + i) * D + d] * f;
  }
  if (d < D) out[((long)b * Hq + hq) * D + d] = (bf16)(L > 0.f ? O / L : 0.f);
}

// ------------------------------------------------------------------------------------------
// Lean (work-balanced) split-K decode
// ------------------------------------------------------------------------------------------
// The partitioned kernel above gives every (row, kv head, partition) its own workgroup, so a
// batch whose contexts spread over 1.5-6.5k keys leaves long partitions running alone at the end
// (and short rows waste whole workgroups).  Here each kv head's (row, block) units of the batch's
// per-row KV blocks are flattened
// row-major into one range that is cut into equal contiguous pieces, one per WAVE of the head's
// share of a fixed grid sized to one round of the chip: every wave streams the same number of KV
// blocks and the whole grid drains together.  Workgroup i serves kv head i % Hkv, so with the
// round-robin workgroup dispatch over the 8 XCDs (Hkv == 8) each XCD streams ONE head and its 4 MB
// L2 keeps that head's shared-prefix blocks (0.5 MB per 1k tokens) hot for every row.  A wave
// writes one partial (m, l, unnormalised O) per row segment it touches, at slot (wave - first
// wave of the segment); a segment one wave covers entirely is normalised and written straight to
// `out` (no partial, no merge).  The plan (per-row prefix sums, units per wave) is recomputed by
// every workgroup from ctx_lens (device data: hipGraph-capturable), and workgroup 0
// publishes it in `meta` for the merge kernel.
constexpr int LEAN_MAX_B = 1024;

struct LeanPlan {
  int total;     // KV blocks over all rows (per kv head)
  int per_wave;  // units per wave
};

// s_pre[0..B]: exclusive prefix sums of the per-row block counts
__device__ __forceinline__ LeanPlan lean_plan(int* s_pre, int* s_w, const int* __restrict__ ctx_lens, int B,
                                              int nwaves, int nparts, int min_per_wave) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int c[4], sum = 0, mx = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = 4 * t + i;
    c[i] = b < B ? (ctx_lens[b] + KV_BS - 1) / KV_BS : 0;
    sum += c[i];
    mx = max(mx, c[i]);
  }
  int inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
  if (lane == 63) s_w[w] = inc;
  if (lane == 0) s_w[4 + w] = mx;
  __syncthreads();
  int excl = inc - sum, total = 0, maxn = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < w) excl += s_w[i];
    total += s_w[i];
    maxn = max(maxn, s_w[4 + i]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = 4 * t + i;
    if (b < B) s_pre[b] = excl;
    excl += c[i];
  }
  if (t == 0) s_pre[B] = total;
  __syncthreads();
  // a segment of n blocks meets at most ceil(n / per_wave) + 1 waves: keep that <= nparts slots
  const int want = (total + nwaves - 1) / nwaves;
  const int cap = (maxn + nparts - 2) / (nparts - 1);
  return LeanPlan{total, max(max(want, cap), min_per_wave)};
}

// grid (nwg), nwg % Hkv == 0: workgroup i serves kv head i % Hkv with 4 waves.  A head's units
// are cut into chunks of per_wave blocks and wave hw of the head owns chunk hw.  (A dynamic form --
// smaller chunks claimed from a per-head atomic counter, for workgroups that start late beside a
// concurrent prefill attention -- measured slower, the claim round trip costing more than it
// balanced: 185 vs 140 us at B = 64, profiles/r3_decode_lean_vs_partitioned.jsonl; removed in r5.)
constexpr int LEAN_META0 = 64;   // meta[LEAN_META0..]: the plan, published for the merge kernel

// K/V fragment load of the lean kernel: default cache policy, or (NT) non-temporal.  A row's own
// blocks are read once per step; blocks several rows of the step share (the common system prompt --
// marked in the decode block table as -id - 1 by the host, engine/model_runner.mark_shared_blocks)
// keep the default policy for their L2 / MALL reuse.  lean_flags bit 0: NT for unmarked blocks.
template <bool NT>
__device__ __forceinline__ uint4 kv_load(const uint4* p) {
  if constexpr (NT) {
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    return *p;
  }
}

template <int D, bool NT = false>
__global__ void __launch_bounds__(256) decode_lean_kernel(
    const bf16* __restrict__ q, const int* __restrict__ ctx_lens, const int* __restrict__ block_tables,
    const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache, bf16* __restrict__ out,
    float* __restrict__ part_m, float* __restrict__ part_l, float* __restrict__ part_o, int* __restrict__ meta,
    float scale_log2, int B, int Hq, int Hkv, int max_blocks, int nparts, int part_stride, int min_per_wave) {
  constexpr int KC = D / 32, DT = D / 16;
  __shared__ int s_pre[LEAN_MAX_B + 1];
  __shared__ int s_w[8];
  const LeanPlan pl = lean_plan(s_pre, s_w, ctx_lens, B, gridDim.x / Hkv * 4, nparts, min_per_wave);
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i <= B; i += 256) meta[LEAN_META0 + i] = s_pre[i];
    if (threadIdx.x == 0) meta[LEAN_META0 + B + 1] = pl.per_wave;
  }
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int h = blockIdx.x % Hkv;
  const int G = Hq / Hkv;
  const int nch = (pl.total + pl.per_wave - 1) / pl.per_wave;
  const int chunk = (blockIdx.x / Hkv) * 4 + (threadIdx.x >> 6);
  if (chunk < nch) {   // no barrier below this point
  int u = chunk * pl.per_wave;
  const int uend = min(pl.total, u + pl.per_wave);
  // row of unit u: the last b with s_pre[b] <= u (skips empty rows)
  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_pre[mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  int b = lo;

  while (u < uend) {
    const int seg0 = s_pre[b], n = s_pre[b + 1] - seg0;
    const int k0 = u - seg0, k1 = min(n, uend - seg0);
    const int ctx = ctx_lens[b];
    const int* bt = block_tables + (long)b * max_blocks;

    Frag qf[KC];
    {
      const bool valid = col < G;
      const bf16* qrow = q + ((long)b * Hq + h * G + (valid ? col : 0)) * D;
#pragma unroll
      for (int c = 0; c < KC; ++c)
        qf[c].u = valid ? *reinterpret_cast<const uint4*>(qrow + c * 32 + g * 8) : make_uint4(0, 0, 0, 0);
    }
    f32x4 o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    int ids = 0;
    for (int k = k0; k < k1; ++k) {
      const int it = k - k0;
      if ((it & 63) == 0) {
        const int kl = k + lane;
        ids = kl < k1 ? bt[kl] : 0;
      }
      const int id = __builtin_amdgcn_readlane(ids, it & 63);
      const bool shared = id < 0;                          // marked by the host: several rows read it
      const long phys = shared ? -(long)id - 1 : id;
      const uint4* kb = reinterpret_cast<const uint4*>(k_cache + (phys * Hkv + h) * (long)(KV_BS * D));
      const uint4* vb = reinterpret_cast<const uint4*>(v_cache + (phys * Hkv + h) * (long)(KV_BS * D));
      Frag kf[4][KC], vf[DT][2];
      auto load_kv = [&](auto ntc) {
        constexpr bool NTB = decltype(ntc)::value;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int c = 0; c < KC; ++c) kf[t][c].u = kv_load<NTB>(kb + (t * KC + c) * 64 + lane);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int st = 0; st < 2; ++st) vf[dt][st].u = kv_load<NTB>(vb + (dt * 2 + st) * 64 + lane);
      };
      if (NT && !shared) load_kv(std::true_type{});    // wave-uniform branch
      else load_kv(std::false_type{});
      const int j = k;
      f32x4 sc[4];
      float mt = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < KC; ++c) sc[t] = mfma16(kf[t][c].v, qf[c].v, sc[t]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = j * KV_BS + 16 * t + 4 * g + r;
          const float v = key < ctx ? sc[t][r] * scale_log2 : -INFINITY;
          sc[t][r] = v;
          mt = fmaxf(mt, v);
        }
      }
      mt = rowgroup_max(mt);
      const bool grow = mt > m + 8.f;
      if (__any(grow)) {
        const float mn = grow ? mt : m;
        const float alpha = grow ? fast_exp2(m - mn) : 1.f;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
        m = mn;
      }
      const float mref = (m == -INFINITY) ? 0.f : m;
      float ls = 0.f;
      Frag pf[2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fast_exp2(sc[t][r] - mref);
          ls += pv;
          pf[t >> 1].v[4 * (t & 1) + r] = (bf16)pv;
        }
      }
      l += ls;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        o[dt] = mfma16(vf[dt][0].v, pf[0].v, o[dt]);
        o[dt] = mfma16(vf[dt][1].v, pf[1].v, o[dt]);
      }
    }
    l = rowgroup_sum(l);
    if (col < G) {
      const int hq = h * G + col;
      if (k0 == 0 && k1 == n) {   // whole segment: final output
        const float inv = 1.f / l;
        bf16* orow = out + ((long)b * Hq + hq) * D;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(o[dt][r] * inv);
          *reinterpret_cast<bf16x4*>(orow + 16 * dt + 4 * g) = v;
        }
      } else {
        const long pi = ((long)b * Hq + hq) * part_stride + (chunk - seg0 / pl.per_wave);
        PENNY_DASSERT(chunk - seg0 / pl.per_wave < nparts);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) *reinterpret_cast<f32x4*>(part_o + pi * D + 16 * dt + 4 * g) = o[dt];
        if (g == 0) {
          part_m[pi] = m;
          part_l[pi] = l;
        }
      }
    }
    u = seg0 + k1;
    do {
      ++b;
    } while (b < B - 1 && s_pre[b + 1] == s_pre[b]);
  }
  }
}

// grid (Hq / HPW, B), HPW * D threads: merges row b's lean partials for HPW heads per workgroup,
// skipping rows one wave already finished (the decision depends on b only, so the whole workgroup
// returns).  HPW = 1 is the r3 form (one workgroup per (head, row)); HPW = 4 (lean_flags bit 1)
// quarters the workgroup count.  (One workgroup per row looping over all heads measured 24-178 us
// per call against 8-10: the passes serialise their dependent loads.)
template <int D, int HPW>
__global__ void __launch_bounds__(HPW * D) decode_lean_reduce_kernel(const int* __restrict__ meta,
                                                                     const float* __restrict__ part_m,
                                                                     const float* __restrict__ part_l,
                                                                     const float* __restrict__ part_o,
                                                                     bf16* __restrict__ out, int B, int Hq,
                                                                     int part_stride) {
  const int b = blockIdx.y, hq = blockIdx.x * HPW + threadIdx.x / D, d = threadIdx.x % D;
  if (hq >= Hq) return;
  const int pre = meta[LEAN_META0 + b], n = meta[LEAN_META0 + b + 1] - pre, pw = meta[LEAN_META0 + B + 1];
  int np = 0;
  if (n > 0) {
    const int fw = pre / pw, lw = (pre + n - 1) / pw;
    if (fw == lw) return;   // written by its one wave
    np = lw - fw + 1;
  }
  const long base = ((long)b * Hq + hq) * part_stride;
  float M = -INFINITY;
  for (int i = 0; i < np; ++i) M = fmaxf(M, part_m[base + i]);
  float L = 0.f, O = 0.f;
  for (int i = 0; i < np; ++i) {
    const float f = exp2f(part_m[base + i] - M);
    L += part_l[base + i] * f;
    O += part_o[(base + i) * D + d] * f;
  }
  out[((long)b * Hq + hq) * D + d] = (bf16)(L > 0.f ? O / L : 0.f);
}


// Pipelined prefill (the production prefill path for tiles of > 128 rows).
// One workgroup = NW waves x 32 rows = NW*32 (token*G + head) rows of one sequence and kv head:
// every staged K/V block is shared by NW waves (half the LDS fill traffic per row of the 4-wave
// tile) and the K/V ring is NBUF blocks deep, so block j+NBUF-1 streams in while block j is on
// the MFMAs.  Synchronisation follows the counted-vmcnt recipe: each wave waits only for ITS
// pieces of block j (`s_waitcnt vmcnt(LOADS)` while the next block's pieces stay in flight), one
// raw s_barrier publishes block j to all waves and retires everyone's reads of the buffer about
// to be refilled -- one barrier per block, never a vmcnt(0) drain in the steady state.  All LDS is
// one __shared__ array (a second one makes hipcc drain vmcnt before every ds_read).
template <int N>
__device__ __forceinline__ void wait_vmcnt_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Lean (KV-split) prefill work: a tile's KV walk can be cut into chunks run by different
// workgroups; a chunk writes flash-decoding partial state (its normalised O / l, running max m, row
// sum l) to slot `slot`, and prefill_merge_kernel combines a tile's slots in chunk order.  The
// partial O is bf16 (r6): half the f32 round trip through HBM and half the chunk's store tail; O / l
// is a convex combination of V rows, so the bf16 rounding is relative to |V| (the same as the
// unsplit kernel's own output rounding), and the merge weights l * 2^(m - M) stay f32.
struct PrefillLean {
  const int* items;     // [n, 6]: sequence, tile, first block, end block, slot (< 0: whole tile), 0
  bf16* part_o;         // [slots, Hkv, 256 rows, D] bf16: O / l (0 where l = 0)
  float* part_ml;       // [slots, Hkv, 256 rows, 2] f32: m (log2 units of the scaled scores), l
};

template <int D, int NW, int NBUF, bool HEAD_FAST, bool PREF = true, bool SB = false, int FOLD = 0>
__global__ void __launch_bounds__(NW * 64, 1) prefill2_kernel(
    const bf16* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ block_tables, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    bf16* __restrict__ out, float scale_log2, int Hq, int Hkv, int max_blocks, int causal,
    float* __restrict__ lse, const int* __restrict__ work, PrefillLean lean = PrefillLean{}) {
  constexpr int KC = D / 32, DT = D / 16;
  constexpr int TILE = KV_BS * D * 2;         // bytes of one K (or V) block tile
  constexpr int PIECES = TILE / 1024 / NW;    // 1-KiB glds pieces per wave per tile
  constexpr int LOADS = 2 * PIECES;           // glds per wave per staged block (K + V)
  static_assert(PIECES >= 1 && TILE % (1024 * NW) == 0, "tile must split evenly over the waves");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TILE];  // [buf][K|V]

  // causal tiles grow with their index: dispatch the longest first so they do not form the tail.
  // HEAD_FAST grid (Hkv, tiles, seqs): with round-robin dispatch over the 8 XCDs every tile of a
  // (sequence, kv head) lands on the same XCD, so its K/V blocks are fetched into one L2 and
  // re-read from there by the other tiles (grid (tiles, Hkv, seqs) spreads them over all 8 L2s)
  // `work` (host-built, ops.attention.prefill_work_list): the step's real (sequence, tile) pairs,
  // longest KV walk first across ALL sequences (LPT order: the short decide tiles fill the last
  // round instead of trailing it, and no workgroup is launched for a tile past a short sequence's
  // end).  Without it: grid (.., max tiles, sequences), each sequence's tiles longest first.
  const int item = HEAD_FAST ? blockIdx.y : blockIdx.x;
  const int* li = lean.items ? lean.items + 6 * item : nullptr;
  const int s = li ? li[0] : (work ? work[2 * item] : blockIdx.z);
  const int h = HEAD_FAST ? blockIdx.x : blockIdx.y;
  const int tile = li ? li[1] : (work ? work[2 * item + 1] : (HEAD_FAST ? gridDim.y : gridDim.x) - 1 - item);
  const int G = Hq / Hkv;
  const int TQ = NW * 32 / G;
  const int q0 = cu_q[s], qlen = cu_q[s + 1] - q0;
  const int tok0 = tile * TQ;
  if (tok0 >= qlen) return;
  const int ctx = ctx_lens[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;

  const int last_tok = min(tok0 + TQ, qlen) - 1;
  const int kv_end = causal ? min(ctx, ctx - qlen + last_tok + 1) : ctx;
  const int nblk_tile = (kv_end + KV_BS - 1) / KV_BS;
  // lean items: this workgroup's blocks [jb, jb + nblk) of the tile's walk, partial state to `slot`
  const int jb = li ? li[2] : 0;
  const int nblk = li ? min(li[3], nblk_tile) - jb : nblk_tile;
  const int slot = li ? li[4] : -1;
  const int* bt = block_tables + (long)s * max_blocks + jb;

  auto stage = [&](int j) {
    const long phys = bt[j];
    PENNY_DASSERT(phys >= 0);
    const char* kb = reinterpret_cast<const char*>(k_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    const char* vb = reinterpret_cast<const char*>(v_cache + (phys * Hkv + h) * (long)(KV_BS * D));
    char* kl = smem + (j % NBUF) * 2 * TILE;
    char* vl = kl + TILE;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = w * PIECES + i;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(kb + piece * 1024 + lane * 16), (lds_void_t*)(kl + piece * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(vb + piece * 1024 + lane * 16), (lds_void_t*)(vl + piece * 1024),
                                       16, 0, 0);
    }
  };
  // K/V prologue first: the Q loads below are younger, so the first counted wait covers them too
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j)
    if (j < nblk) stage(j);

  int tok[2], head[2], qpos[2];
  Frag qf[2][KC];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int r = w * 32 + ct * 16 + col;
    tok[ct] = tok0 + r / G;
    head[ct] = h * G + r % G;
    const bool valid = tok[ct] < qlen;
    qpos[ct] = valid ? ctx - qlen + tok[ct] : ctx - 1;
    const bf16* qrow = q + ((long)(q0 + (valid ? tok[ct] : 0)) * Hq + head[ct]) * D;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      qf[ct][c].u = valid ? *reinterpret_cast<const uint4*>(qrow + c * 32 + g * 8) : make_uint4(0, 0, 0, 0);
  }
  if constexpr (FOLD == 2) {
    // Q prescaled by scale * log2(e) once per tile (one bf16 rounding of q*c): the block loop's
    // scores then need no per-score multiply (attend_block_fold)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[ct][c].v[e] = (bf16)((float)qf[ct][c].v[e] * scale_log2);
  }
  // Retire the Q loads (and the prologue) with a wait the compiler's waitcnt pass can SEE: it
  // then knows qf is resident and does not re-insert a vmcnt(0) at every loop iteration (an
  // inline-asm wait is opaque to it).  vmcnt(0), expcnt/lgkmcnt untouched.
  __builtin_amdgcn_s_waitcnt(0x0F70);

  f32x4 o[2][DT];
  float m[2], l[2];
  f32x4 la[2];      // FOLD: row sums from the matrix pipe
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    m[ct] = -INFINITY;
    l[ct] = 0.f;
    la[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[ct][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // Waves whose 32 rows are all padding (the last tile of a short chunk, e.g. a decide prompt's
  // 200 new tokens behind 4.6k cached ones) and, under the causal mask, blocks entirely after a
  // wave's last row: the wave still stages its K/V pieces and meets every barrier, but skips the
  // MFMAs and the softmax, leaving its SIMD's issue slots to the live wave sharing it.
  const int wave_tok0 = tok0 + (w * 32) / G;
  const bool wave_live = wave_tok0 < qlen;
  const int wave_last = min(tok0 + (w * 32 + 31) / G, qlen - 1);
  const int wave_kv_end = causal ? ctx - qlen + wave_last + 1 : ctx;
  for (int j = 0; j < nblk; ++j) {           // local block j = absolute block jb + j
    // my pieces of block j landed (younger blocks j+1.. may stay in flight), then publish
    if (j + NBUF - 2 < nblk && NBUF >= 3) wait_vmcnt_barrier<(NBUF - 2) * LOADS>();
    else wait_vmcnt_barrier<0>();
    if (j + NBUF - 1 < nblk) stage(j + NBUF - 1);   // refills the buffer everyone finished at j-1
    const int ja = jb + j;
    if (!wave_live || ja * KV_BS >= wave_kv_end) continue;
    const uint4* kl = reinterpret_cast<const uint4*>(smem + (j % NBUF) * 2 * TILE);
    const uint4* vl = reinterpret_cast<const uint4*>(smem + (j % NBUF) * 2 * TILE + TILE);
    const bool full = (ja + 1) * KV_BS <= ctx && (!causal || (ja + 1) * KV_BS - 1 <= ctx - qlen + wave_tok0);
    if constexpr (FOLD != 0)
      attend_block_fold<D, 2, SB, FOLD == 2>(kl, vl, qf, o, m, la, causal, ja, ctx, qpos, scale_log2, lane, g,
                                             __builtin_amdgcn_readfirstlane((int)!full) != 0);
    else
      attend_block<D, 2, PREF, SB>(kl, vl, qf, o, m, l, causal, ja, ctx, qpos, scale_log2, lane, g,
                                   __builtin_amdgcn_readfirstlane((int)!full) != 0);
  }

#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const float lt = FOLD != 0 ? la[ct][0] : rowgroup_sum(l[ct]);
    if (slot >= 0) {                          // a chunk of a split walk: partial state for the merge
      const long pr = ((long)slot * Hkv + h) * 256 + w * 32 + ct * 16 + col;
      const float pinv = lt > 0.f ? 1.f / lt : 0.f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf16x4 v4;
#pragma unroll
        for (int r = 0; r < 4; ++r) v4[r] = (bf16)(o[ct][dt][r] * pinv);
        *reinterpret_cast<bf16x4*>(lean.part_o + pr * D + 16 * dt + 4 * g) = v4;
      }
      if (g == 0) {
        lean.part_ml[2 * pr] = m[ct];
        lean.part_ml[2 * pr + 1] = lt;
      }
      continue;
    }
    if (tok[ct] >= qlen) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16* orow = out + ((long)(q0 + tok[ct]) * Hq + head[ct]) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      bf16x4 v4;
#pragma unroll
      for (int r = 0; r < 4; ++r) v4[r] = (bf16)(o[ct][dt][r] * inv);
      *reinterpret_cast<bf16x4*>(orow + 16 * dt + 4 * g) = v4;
    }
    if (lse != nullptr && g == 0)
      lse[(long)(q0 + tok[ct]) * Hq + head[ct]] = lt > 0.f ? (m[ct] + __log2f(lt)) * 0.6931471805599453f : -INFINITY;
  }
}

// Merge the chunk partials of split tiles (lean prefill): grid (splits, Hkv, 256 / RPB), 256
// threads, one row per thread group: lanes 0-31 / 32-63 take two rows (D = 128), 4 dims per lane
// (f32x4), so every load is coalesced.  A single-tile step splits its walk into up to ~32 chunks;
// a row per thread group (instead of 32 rows looped per workgroup) keeps the slot loads
// independent and in flight together -- the looped form was latency-bound at 126 us per merge
// (profiles/r4_bench_kernel_stats_head.md).
// merge [n, 6]: sequence, tile, first slot, number of slots, 0, 0 (chunk order = slot order).
template <int D>
__global__ void __launch_bounds__(256) prefill_merge_kernel(const int* __restrict__ merge, const int* __restrict__ cu_q,
                                                            const bf16* __restrict__ part_o,
                                                            const float* __restrict__ part_ml, bf16* __restrict__ out,
                                                            float* __restrict__ lse, int Hq, int Hkv) {
  static_assert(D == 128 || D == 64, "head dim");
  constexpr int LPR = D / 4;                  // lanes per row
  constexpr int RPW = 64 / LPR;               // rows per wave instruction
  constexpr int RPB = 4 * RPW;                // rows per workgroup
  const int* mg = merge + 6 * blockIdx.x;
  const int s = mg[0], tile = mg[1], slot0 = mg[2], np = mg[3];
  const int h = blockIdx.y, G = Hq / Hkv, TQ = 256 / G;
  const int q0 = cu_q[s], qlen = cu_q[s + 1] - q0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane / LPR, d = (lane % LPR) * 4;
  const int r = blockIdx.z * RPB + w * RPW + sub;
  const int tok = tile * TQ + r / G;
  if (tok >= qlen) return;
  const long stride = (long)Hkv * 256;        // rows between consecutive slots
  const long pr0 = ((long)slot0 * Hkv + h) * 256 + r;
  float M = -INFINITY;
#pragma unroll 8
  for (int i = 0; i < np; ++i) M = fmaxf(M, part_ml[2 * (pr0 + i * stride)]);
  float L = 0.f;
  f32x4 O = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int i = 0; i < np; ++i) {
    const long pr = pr0 + i * stride;
    const float mi = part_ml[2 * pr];
    const float wl = mi == -INFINITY ? 0.f : part_ml[2 * pr + 1] * exp2f(mi - M);   // l_i 2^(m_i - M)
    L += wl;
    const bf16x4 p4 = *reinterpret_cast<const bf16x4*>(part_o + pr * D + d);       // O_i / l_i
#pragma unroll
    for (int k = 0; k < 4; ++k) O[k] += (float)p4[k] * wl;
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int head = h * G + r % G;
  bf16x4 v4;
#pragma unroll
  for (int k = 0; k < 4; ++k) v4[k] = (bf16)(O[k] * inv);
  *reinterpret_cast<bf16x4*>(out + ((long)(q0 + tok) * Hq + head) * D + d) = v4;
  if (lse != nullptr && d == 0)
    lse[(long)(q0 + tok) * Hq + head] = L > 0.f ? (M + __log2f(L)) * 0.6931471805599453f : -INFINITY;
}

// ------------------------------------------------------------------------------------------
// 32x32x16 prefill (variant 7): prefill2's staging pipeline with the block math on
// v_mfma_f32_32x32x16_bf16.  Each MFMA holds the SIMD's vector issue for 8 of its 32 cycles instead
// of 8 of 16 (16x16x32), so the softmax VALU (~100 instructions per block and wave, 32 of them
// 8-cycle v_exp) fits in the shadow of a block's 32 MFMAs instead of bounding the loop
// (MI355X_MICROARCH.md cycle constants: 'vector-instruction ISSUE cost').
//
// Orientation as in prefill2 (S^T = K.Q^T, O^T = V^T.P^T), one wave = 32 query rows = the 32 MFMA
// columns: lane (c = lane & 31, h = lane >> 5) holds query row c and, per 32-key S^T tile, keys of
// tile rows (reg & 3) + 8 (reg >> 2) + 4h.  Tile row rho of key tile T is key pi(32T + rho), pi
// swapping bits 3 and 4 of the row index: with that permutation
//   * the K fragment of (T, k-step c) is one 16-B piece of the fragment-native K block at
//     lane base + 8192 T + 512 c (kv_layout.h k_index), and
//   * the P^T operand of P.V k-step s is registers 8(s&1) .. +7 of S^T tile s >> 1 converted to
//     bf16 in place (cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand'),
//     whose keys are exactly the 8 keys the fragment-native V block holds in ONE 16-B piece for
//     lane group 2(s&1) + h: V fragment (dim tile dt, s) at lane base + 4096 dt + 512 s.
// Every fragment read is a ds_read_b128 with an immediate offset from one per-lane base, and both
// read patterns are bank-conflict free on the 16-lane phases (the stored KV layout is unchanged:
// decode, the KV writers and the 16x16 kernels read the same blocks).
// The row max is 31 v_max + one permlane32 swap (lane and lane ^ 32 hold the same query); the row
// sum stays a per-lane f32 partial, combined once at the end.  Softmax: base 2 with the deferred
// rescale (threshold 8) of attend_block_fold; QPRE = q arrives prescaled by scale * log2(e) and the
// S^T chains start at -m (no per-score FMA).
__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float lanepair_max(float v) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_raw(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float lanepair_sum(float v) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <bool QPRE>
__device__ __forceinline__ void attend_block32(const char* __restrict__ kl, const char* __restrict__ vl,
                                               const Frag (&qf)[8], f32x16 (&o)[4], float& m, float& l,
                                               f32x16& ms, bool causal, int j, int ctx, int qpos, float scale_log2,
                                               int h, bool need_mask) {
  Frag kf[2][8];
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int c = 0; c < 8; ++c) kf[T][c].u = *reinterpret_cast<const uint4*>(kl + 8192 * T + 512 * c);
  const bool fresh = m == -INFINITY;
  // each S^T chain starts at ms = -m (QPRE; 0 while fresh or exact-Q): its first MFMA reads the
  // persistent splat as C, so no per-block re-initialisation of the 32 accumulator registers
  f32x16 sc[2];
#pragma unroll
  for (int T = 0; T < 2; ++T) {
    sc[T] = mfma32(kf[T][0].v, qf[0].v, ms);
#pragma unroll
    for (int c = 1; c < 8; ++c) sc[T] = mfma32(kf[T][c].v, qf[c].v, sc[T]);
  }
  Frag vf[4][4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int st = 0; st < 4; ++st) vf[dt][st].u = *reinterpret_cast<const uint4*>(vl + 4096 * dt + 512 * st);

  if (need_mask) {
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = j * KV_BS + 32 * T + 16 * ((r >> 2) & 1) + 8 * (r >> 3) + 4 * h + (r & 3);
        const bool ok = (key < ctx) & ((!causal) | (key <= qpos));
        sc[T][r] = ok ? sc[T][r] : -INFINITY;
      }
  }
  // a max3 tree over the lane's 32 scores (depth 4, 16 instructions): a serial v_max chain is 32
  // dependent instructions on the wave's critical path between its QK^T and P.V MFMAs
  float m3[11];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int a = 3 * i, b = a + 1, c = a + 2;
    m3[i] = vmax3_raw(sc[a >> 4][a & 15], sc[b >> 4][b & 15], sc[c >> 4][c & 15]);
  }
  m3[10] = vmax_raw(sc[1][14], sc[1][15]);
  const float mt4[4] = {vmax3_raw(m3[0], m3[1], m3[2]), vmax3_raw(m3[3], m3[4], m3[5]),
                        vmax3_raw(m3[6], m3[7], m3[8]), vmax_raw(m3[9], m3[10])};
  float mt = vmax_raw(vmax_raw(mt4[0], mt4[1]), vmax_raw(mt4[2], mt4[3]));
  mt = lanepair_max(mt);                      // QPRE: max of s*c - m; else max of s
  if constexpr (!QPRE) mt = fresh ? mt * scale_log2 : mt * scale_log2 - m;
  const bool grow = mt > (fresh ? -INFINITY : 8.f);
  if (__any(grow)) {
    const float rise = grow ? mt : 0.f;
    if (grow) {
      const float alpha = fresh ? 1.f : fast_exp2(-rise);   // fresh: O and l are still 0
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
      m = fresh ? rise : m + rise;
    }
    if constexpr (QPRE) {
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[T][r] -= rise;
      const float mn = m == -INFINITY ? 0.f : -m;
#pragma unroll
      for (int r = 0; r < 16; ++r) ms[r] = mn;
    }
  }
  if constexpr (QPRE) {
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[T][r] = fast_exp2(sc[T][r]);
  } else {
    const float mref = m == -INFINITY ? 0.f : m;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[T][r] = fast_exp2(fmaf(sc[T][r], scale_log2, -mref));
  }
  // row-sum partial as a pairwise tree (hipcc keeps a written f32 add chain serial: 32 dependent adds)
  float s16[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) s16[r] = sc[0][r] + sc[1][r];
#pragma unroll
  for (int w2 = 8; w2 >= 1; w2 >>= 1)
#pragma unroll
    for (int r = 0; r < w2; ++r) s16[r] = s16[r] + s16[r + w2];
  l += s16[0];
  Frag pf[4];
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int e = 0; e < 8; ++e) pf[st].v[e] = (bf16)sc[st >> 1][8 * (st & 1) + e];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int st = 0; st < 4; ++st) o[dt] = mfma32(vf[dt][st].v, pf[st].v, o[dt]);
}

// prefill2_kernel's grid, work lists, lean slots and K/V staging ring with attend_block32 (D = 128)
template <int NBUF, bool QPRE>
__global__ void __launch_bounds__(512, 1) prefill3_kernel(
    const bf16* __restrict__ q, const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ block_tables, const bf16* __restrict__ k_cache, const bf16* __restrict__ v_cache,
    bf16* __restrict__ out, float scale_log2, int Hq, int Hkv, int max_blocks, int causal,
    float* __restrict__ lse, const int* __restrict__ work, PrefillLean lean = PrefillLean{}) {
  constexpr int D = 128, NW = 8;
  constexpr int TILE = KV_BS * D * 2;
  constexpr int PIECES = TILE / 1024 / NW;
  constexpr int LOADS = 2 * PIECES;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * TILE];

  const int item = blockIdx.y;
  const int* li = lean.items ? lean.items + 6 * item : nullptr;
  const int s = li ? li[0] : (work ? work[2 * item] : blockIdx.z);
  const int hk = blockIdx.x;
  const int tile = li ? li[1] : (work ? work[2 * item + 1] : gridDim.y - 1 - item);
  const int G = Hq / Hkv;
  const int TQ = NW * 32 / G;
  const int q0 = cu_q[s], qlen = cu_q[s + 1] - q0;
  const int tok0 = tile * TQ;
  if (tok0 >= qlen) return;
  const int ctx = ctx_lens[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;

  const int last_tok = min(tok0 + TQ, qlen) - 1;
  const int kv_end = causal ? min(ctx, ctx - qlen + last_tok + 1) : ctx;
  const int nblk_tile = (kv_end + KV_BS - 1) / KV_BS;
  const int jb = li ? li[2] : 0;
  const int nblk = li ? min(li[3], nblk_tile) - jb : nblk_tile;
  const int slot = li ? li[4] : -1;
  const int* bt = block_tables + (long)s * max_blocks + jb;

  auto stage = [&](int jj) {
    const long phys = bt[jj];
    PENNY_DASSERT(phys >= 0);
    const char* kb = reinterpret_cast<const char*>(k_cache + (phys * Hkv + hk) * (long)(KV_BS * D));
    const char* vb = reinterpret_cast<const char*>(v_cache + (phys * Hkv + hk) * (long)(KV_BS * D));
    char* kls = smem + (jj % NBUF) * 2 * TILE;
    char* vls = kls + TILE;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = w * PIECES + i;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(kb + piece * 1024 + lane * 16), (lds_void_t*)(kls + piece * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(vb + piece * 1024 + lane * 16), (lds_void_t*)(vls + piece * 1024),
                                       16, 0, 0);
    }
  };
#pragma unroll
  for (int jj = 0; jj < NBUF - 1; ++jj)
    if (jj < nblk) stage(jj);

  // this lane's query row and its 8 Q fragments (B operand: dims 16c' + 8h .. +7 of the row)
  const int r = w * 32 + c;
  const int tok = tok0 + r / G, head = hk * G + r % G;
  const bool valid = tok < qlen;
  const int qpos = valid ? ctx - qlen + tok : ctx - 1;
  Frag qf[8];
  {
    const bf16* qrow = q + ((long)(q0 + (valid ? tok : 0)) * Hq + head) * D;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
      qf[cc].u = valid ? *reinterpret_cast<const uint4*>(qrow + cc * 16 + h * 8) : make_uint4(0, 0, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);        // vmcnt(0): Q resident (a wait hipcc can see)

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[dt][e] = 0.f;
  float m = -INFINITY, l = 0.f;
  f32x16 ms;                                  // the S^T chains' start value (attend_block32)
#pragma unroll
  for (int e = 0; e < 16; ++e) ms[e] = 0.f;
  // per-lane fragment bases: K key-row pi(r) at 16 (256 r3 + 16 h + 8 r4 + (r & 7)); V dim row r at
  // 2048 (r >> 4) + 256 h + 16 (r & 15)
  const int kbase = 16 * (256 * ((c >> 3) & 1) + 16 * h + 8 * (c >> 4) + (c & 7));
  const int vbase = 2048 * (c >> 4) + 256 * h + 16 * (c & 15);

  const int wave_tok0 = tok0 + (w * 32) / G;
  const bool wave_live = wave_tok0 < qlen;
  const int wave_last = min(tok0 + (w * 32 + 31) / G, qlen - 1);
  const int wave_kv_end = causal ? ctx - qlen + wave_last + 1 : ctx;
  // static priority for the second-dispatched half (waves 4-7 lose VALU arbitration to their SIMD
  // partner on every segment otherwise; cdna_hip_programming.md T5 static form)
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  for (int jj = 0; jj < nblk; ++jj) {
    if (jj + NBUF - 2 < nblk && NBUF >= 3) wait_vmcnt_barrier<(NBUF - 2) * LOADS>();
    else wait_vmcnt_barrier<0>();
    if (jj + NBUF - 1 < nblk) stage(jj + NBUF - 1);
    const int ja = jb + jj;
    if (!wave_live || ja * KV_BS >= wave_kv_end) continue;
    const char* kls = smem + (jj % NBUF) * 2 * TILE;
    const bool full = (ja + 1) * KV_BS <= ctx && (!causal || (ja + 1) * KV_BS - 1 <= ctx - qlen + wave_tok0);
    attend_block32<QPRE>(kls + kbase, kls + TILE + vbase, qf, o, m, l, ms, causal, ja, ctx, qpos, scale_log2, h,
                         __builtin_amdgcn_readfirstlane((int)!full) != 0);
  }

  const float lt = lanepair_sum(l);
  long pr = 0;
  if (slot >= 0) {                            // a chunk of a split walk: partial state for the merge
    pr = ((long)slot * Hkv + hk) * 256 + r;
    if (h == 0) {
      lean.part_ml[2 * pr] = m;
      lean.part_ml[2 * pr + 1] = lt;
    }
  } else if (!valid) {
    return;                                   // lanes c and c + 32 share the row: swap partners stay paired
  }
  // O / l as bf16, into the output row or (split walk) the chunk's partial row: the same stores
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  bf16* orow = slot >= 0 ? lean.part_o + pr * D : out + ((long)(q0 + tok) * Hq + head) * D;
  // 16-B stores (cdna_hip_programming.md T21): lane half h holds dims 8rg + 4h .. +3 of each 8-dim
  // group rg; one permlane32 swap per dword of groups (rg, rg + 1) leaves lanes 0-31 the 8 dims of
  // group rg and lanes 32-63 those of group rg + 1
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int rg = 0; rg < 4; rg += 2) {
      union {
        bf16x4 v;
        uint2 u;
      } a, b;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a.v[e] = (bf16)(o[dt][4 * rg + e] * inv);
        b.v[e] = (bf16)(o[dt][4 * rg + 4 + e] * inv);
      }
      const auto x = __builtin_amdgcn_permlane32_swap(a.u.x, b.u.x, false, false);
      const auto y = __builtin_amdgcn_permlane32_swap(a.u.y, b.u.y, false, false);
      *reinterpret_cast<uint4*>(orow + 32 * dt + 8 * rg + 8 * h) = make_uint4(x[0], y[0], x[1], y[1]);
    }
  if (slot < 0 && lse != nullptr && h == 0)
    lse[(long)(q0 + tok) * Hq + head] = lt > 0.f ? (m + __log2f(lt)) * 0.6931471805599453f : -INFINITY;
}

static int prefill_variant();

// Lean big-tile prefill: items [nitems, 6] (see PrefillLean; LPT order), merge [nmerge, 6];
// part_o / part_ml sized for the slots the items use.  Runs prefill2 in the selected variant.
PENNY_API int penny_attention_prefill_lean(const void* q, const int* cu_q, const int* ctx_lens, const int* block_tables,
                                           const void* k_cache, const void* v_cache, void* out, int Hq, int Hkv,
                                           int D, int max_blocks, float scale, int causal, float* lse,
                                           const int* items, int nitems, const int* merge, int nmerge,
                                           void* part_o, float* part_ml, hipStream_t stream) {
  if (nitems <= 0) return 0;
  if (Hq % Hkv || (256 % (Hq / Hkv)) || !items || (nmerge > 0 && (!merge || !part_o || !part_ml)))
    return (int)hipErrorInvalidValue;
  // causal bit 1: q arrives prescaled by scale * log2(e) (penny_gemm_prefill_qkv_rope qscale)
  const bool qpre = causal & 2;
  causal &= 1;
  const float sl2 = qpre ? 1.f : scale * LOG2E;
  const PrefillLean lean{items, static_cast<bf16*>(part_o), part_ml};
  const int var = prefill_variant();
  const dim3 grid(Hkv, nitems, 1);
#define LEAN_LAUNCH(DD, PREF_, SB_, FOLD_)                                                                        \
  hipLaunchKernelGGL((prefill2_kernel<DD, 8, 3, true, PREF_, SB_, FOLD_>), grid, dim3(512), 0, stream,             \
                     (const bf16*)q, cu_q, ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache,       \
                     (bf16*)out, sl2, Hq, Hkv, max_blocks, causal, lse, (const int*)nullptr, lean)
#define LEAN_VARIANTS(DD)                                   \
  if (DD == 128 && var == 7) {                              \
    if (qpre)                                               \
      hipLaunchKernelGGL((prefill3_kernel<3, true>), grid, dim3(512), 0, stream, (const bf16*)q, cu_q, ctx_lens, \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, sl2, Hq, Hkv,   \
                         max_blocks, causal, lse, (const int*)nullptr, lean);                                  \
    else                                                    \
      hipLaunchKernelGGL((prefill3_kernel<3, false>), grid, dim3(512), 0, stream, (const bf16*)q, cu_q, ctx_lens, \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, sl2, Hq, Hkv,    \
                         max_blocks, causal, lse, (const int*)nullptr, lean);                                   \
  } else if (var == 6 || qpre) LEAN_LAUNCH(DD, true, true, 2); \
  else if (var == 4) LEAN_LAUNCH(DD, true, true, 0);        \
  else LEAN_LAUNCH(DD, true, true, 1);                      \
  if (nmerge > 0)                                           \
    hipLaunchKernelGGL(prefill_merge_kernel<DD>, dim3(nmerge, Hkv, 256 / (4 * (64 / (DD / 4)))), dim3(256), 0, stream, \
                       merge, cu_q, static_cast<const bf16*>(part_o), part_ml, (bf16*)out, lse, Hq, Hkv);
  if (D == 128) {
    LEAN_VARIANTS(128)
  } else if (D == 64) {
    LEAN_VARIANTS(64)
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef LEAN_VARIANTS
#undef LEAN_LAUNCH
  PENNY_RETURN_LAUNCH();
}

// Big-tile prefill variant (PENNY_PREFILL_PP, or penny_attention_prefill_variant for in-process A/B
// runs): 7 (default, r6) prefill3 -- the block math on v_mfma_f32_32x32x16_bf16 (head dim 128; 64
// takes 5): +3-5 % on the workload's mixed respond + decide / spec steps, -1-3 % on long single
// responds (the 32x32 loop holds a ~6 % lower clock), +0.3-0.7 % end to end in two same-box driver
// A/Bs (profiles/r6_prefill_attn_32x32_ab.jsonl, r6_bench_prefill_pp7_vs_pp5*.json); 5 prefill2 with
// the VALU-lean softmax (ones-MFMA row sums, lean max / grow logic, exact Q; attend_block_fold), 6 =
// 5 with Q prescaled by scale*log2(e) in-kernel (one extra bf16 rounding of q*c, opt-in), 4 prefill2
// with its K/V fragment prefetch pinned ahead of the MFMAs (kept as the fallback with its tests).  Removed
// in r5: the ping-pong prefill3 (r4 variants 1-3: 15-20 % slower on every mixed step,
// profiles/r4_prefill_attn_pingpong_lean_rejected.jsonl), the unpinned prefill2 (variant 0, 4-6 %
// slower than 4) and the tile-fastest grid order (PENNY_PREFILL_HEAD_FAST=0, 5-47 % slower).
static int g_prefill_variant = -1;
static int prefill_variant() {
  if (g_prefill_variant < 0) {
    const char* v = getenv("PENNY_PREFILL_PP");
    g_prefill_variant = v ? atoi(v) : 7;
  }
  return g_prefill_variant;
}
PENNY_API int penny_attention_prefill_variant(int v) {
  const int old = prefill_variant();
  if (v >= 0) g_prefill_variant = v;
  return old;
}

PENNY_API int penny_attention_prefill(const void* q, const int* cu_q, const int* ctx_lens, const int* block_tables,
                                      const void* k_cache, const void* v_cache, void* out, int num_seqs,
                                      int max_q_len, int Hq, int Hkv, int D, int max_blocks, float scale, int causal,
                                      float* lse, const int* work, int nwork, hipStream_t stream) {
  if (num_seqs <= 0 || max_q_len <= 0) return 0;
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv;
  if (G > 128 || (128 % G)) return (int)hipErrorInvalidValue;
  // causal bit 1: q arrives prescaled by scale * log2(e) at its one bf16 rounding (the fused QKV
  // epilogue's qscale): the big tiles then run the prescaled-Q fold (variant 6's loop without its
  // in-kernel re-rounding of q * c -- it multiplies by 1), the exact scores of variant 5
  const bool qpre = causal & 2;
  causal &= 1;
  const float sl2 = qpre ? 1.f : scale * LOG2E;
  // > 128 rows per (sequence, kv head): the 8-wave pipelined kernel; short chunks keep the
  // 4-wave tile (a 256-row tile would be mostly padding)
  const bool big = (long)max_q_len * G > 128;
  const int pp_env = prefill_variant();
  const int TQ = (big ? 256 : 128) / G;
  const int ntiles = (max_q_len + TQ - 1) / TQ;
  // grid (Hkv, tiles, seqs): the kv head is the fastest workgroup index, so with round-robin dispatch
  // over the 8 XCDs each XCD owns one kv head (+5-47 % TF/s over tile-fastest,
  // profiles/r1_prefill_head_fast.txt: 457 -> 672 at 4 x 2048 causal, 687 -> 905 at 1 x 8192)
  // work list (big tiles only): one workgroup per real (sequence, tile), LPT order
  const bool wl = big && work != nullptr && nwork > 0;
  const dim3 grid(ntiles, Hkv, num_seqs);
  const dim3 grid2 = wl ? dim3(Hkv, nwork, 1) : dim3(Hkv, ntiles, num_seqs);
  const int* wp = wl ? work : nullptr;
#define PREFILL_LAUNCH(DD)                                                                                       \
  if (big && DD == 128 && pp_env == 7) {                                                                         \
    if (qpre)                                                                                                    \
      hipLaunchKernelGGL((prefill3_kernel<3, true>), grid2, dim3(512), 0, stream, (const bf16*)q, cu_q, ctx_lens,  \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, sl2, Hq, Hkv,     \
                         max_blocks, causal, lse, wp);                                                           \
    else                                                                                                         \
      hipLaunchKernelGGL((prefill3_kernel<3, false>), grid2, dim3(512), 0, stream, (const bf16*)q, cu_q, ctx_lens, \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, sl2, Hq, Hkv,      \
                         max_blocks, causal, lse, wp);                                                            \
  } else if (big && (pp_env == 6 || qpre))                                                                       \
    hipLaunchKernelGGL((prefill2_kernel<DD, 8, 3, true, true, true, 2>), grid2, dim3(512), 0, stream,            \
                       (const bf16*)q, cu_q, ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache,   \
                       (bf16*)out, sl2, Hq, Hkv, max_blocks, causal, lse, wp);                                     \
  else if (big && pp_env == 4)                                                                                   \
    hipLaunchKernelGGL((prefill2_kernel<DD, 8, 3, true, true, true>), grid2, dim3(512), 0, stream,               \
                       (const bf16*)q, cu_q, ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache,   \
                       (bf16*)out, sl2, Hq, Hkv, max_blocks, causal, lse, wp);                                     \
  else if (big)                                                                                                  \
    hipLaunchKernelGGL((prefill2_kernel<DD, 8, 3, true, true, true, 1>), grid2, dim3(512), 0, stream,            \
                       (const bf16*)q, cu_q, ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache,   \
                       (bf16*)out, sl2, Hq, Hkv, max_blocks, causal, lse, wp);                                     \
  else                                                                                                           \
    hipLaunchKernelGGL(prefill_kernel<DD>, grid, dim3(256), 0, stream, (const bf16*)q, cu_q, ctx_lens,           \
                       block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, sl2, Hq, Hkv,         \
                       max_blocks, causal, lse);
  if (D == 128) {
    PREFILL_LAUNCH(128)
  } else if (D == 64) {
    PREFILL_LAUNCH(64)
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef PREFILL_LAUNCH
  PENNY_RETURN_LAUNCH();
}

PENNY_API int penny_attention_decode(const void* q, const int* ctx_lens, const int* block_tables, const void* k_cache,
                                     const void* v_cache, void* out, float* part_m, float* part_l, float* part_o,
                                     int B, int Hq, int Hkv, int D, int max_blocks, int pb, int nparts,
                                     int part_stride, float scale, int lean_grid, int* lean_meta,
                                     int lean_min_per_wave, int lean_flags, hipStream_t stream) {
  if (B <= 0) return 0;
  if (Hq % Hkv || Hq / Hkv > 16 || pb <= 0 || nparts <= 0 || part_stride < nparts) return (int)hipErrorInvalidValue;
  // lean_grid > 0: the work-balanced kernel (decode_lean_kernel) and its merge; otherwise the
  // per-(row, head, partition) kernel, kept as the fallback (PENNY_DECODE_LEAN=0)
  const bool lean = lean_grid > 0;
  if (lean && (B > LEAN_MAX_B || nparts < 2 || !lean_meta || lean_min_per_wave < 1 || lean_grid % Hkv ||
               Hkv > LEAN_META0))
    return (int)hipErrorInvalidValue;
  // measured (profiles/r1_decode_head_fast.txt): head-fastest wins at B <= 16 (18.5 vs 21.6 us at
  // ctx 2048 / 1024 shared), sequence-fastest at B >= 64 (a sequence's 8 heads of a KV block are
  // one contiguous 128 KB run, read by one XCD); PENNY_DECODE_HEAD_FAST=0/1 forces either
  static const int head_fast_env = [] {
    const char* v = getenv("PENNY_DECODE_HEAD_FAST");
    return v ? atoi(v) : -1;
  }();
  const bool head_fast = head_fast_env >= 0 ? head_fast_env != 0 : B <= 16;
  const dim3 grid = head_fast ? dim3(Hkv, B, nparts) : dim3(B, nparts, Hkv);
  const float sl2 = scale * LOG2E;
#define DECODE_LAUNCH(DD)                                                                                         \
  if (lean) {                                                                                                   \
    if (lean_flags & 1)                                                                                         \
      hipLaunchKernelGGL((decode_lean_kernel<DD, true>), dim3(lean_grid), dim3(256), 0, stream, (const bf16*)q,  \
                         ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, part_m,  \
                         part_l, part_o, lean_meta, sl2, B, Hq, Hkv, max_blocks, nparts, part_stride,            \
                         lean_min_per_wave);                                                                     \
    else                                                                                                        \
      hipLaunchKernelGGL((decode_lean_kernel<DD, false>), dim3(lean_grid), dim3(256), 0, stream, (const bf16*)q, \
                         ctx_lens, block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, part_m,  \
                         part_l, part_o, lean_meta, sl2, B, Hq, Hkv, max_blocks, nparts, part_stride,            \
                         lean_min_per_wave);                                                                     \
    if (lean_flags & 2)                                                                                         \
      hipLaunchKernelGGL((decode_lean_reduce_kernel<DD, 4>), dim3((Hq + 3) / 4, B), dim3(4 * DD), 0, stream,     \
                         lean_meta, part_m, part_l, part_o, (bf16*)out, B, Hq, part_stride);                      \
    else                                                                                                        \
      hipLaunchKernelGGL((decode_lean_reduce_kernel<DD, 1>), dim3(Hq, B), dim3(DD), 0, stream, lean_meta, part_m, \
                         part_l, part_o, (bf16*)out, B, Hq, part_stride);                                         \
  } else {                                                                                                      \
    if (head_fast)                                                                                              \
      hipLaunchKernelGGL((decode_kernel<DD, true>), grid, dim3(256), 0, stream, (const bf16*)q, ctx_lens,          \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, part_m, part_l,   \
                         part_o, sl2, Hq, Hkv, max_blocks, pb, nparts, part_stride);                              \
    else                                                                                                        \
      hipLaunchKernelGGL((decode_kernel<DD, false>), grid, dim3(256), 0, stream, (const bf16*)q, ctx_lens,         \
                         block_tables, (const bf16*)k_cache, (const bf16*)v_cache, (bf16*)out, part_m, part_l,   \
                         part_o, sl2, Hq, Hkv, max_blocks, pb, nparts, part_stride);                              \
    if (nparts > 1)                                                                                             \
      hipLaunchKernelGGL(decode_reduce_kernel<DD>, dim3(Hq, B), dim3(DD), 0, stream, ctx_lens, part_m, part_l,     \
                         part_o, (bf16*)out, Hq, pb, nparts, part_stride);                                        \
  }
  if (D == 128) {
    DECODE_LAUNCH(128)
  } else if (D == 64) {
    DECODE_LAUNCH(64)
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef DECODE_LAUNCH
  PENNY_RETURN_LAUNCH();
}
