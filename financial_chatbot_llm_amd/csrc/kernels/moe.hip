// K13: Mixtral-style sparse MoE on CDNA4 fp8 MFMA (OCP e4m3; v_mfma_f32_16x16x32_fp8_fp8).
//
// Decode-step pipeline (every launch graph-capturable; buffers sized for the max batch):
//   1. moe_route:   router logits [T, E] -> softmax (f32), top-K, renormalise (HF Mixtral),
//                   counting sort of the T*K (token, expert) pairs by expert ->
//                   sorted token ids / routing weights, expert offsets [E+1], inverse map.
//   2. quant_rows:  dynamic per-row fp8 quantisation of the activations (scale = amax / 448).
//   3. moe_gemm<SILU>: per (expert, 32-row weight slice) workgroup: gathered token rows x W13_e
//                   (fp8 x fp8 MFMA, f32 acc), dequantised by row scales x weight scales, fused
//                   SiLU(gate) * up (16-row interleaved W13) -> [P, F] bf16.
//   4. quant_rows on [P, F], then moe_gemm<SCALE_W>: x W2_e, output scaled by the routing weight.
//   5. moe_combine: out[t] = sum over its K pairs (inverse map, no atomics).
// Weights are pre-tiled (ops/moe.py tile_fp8_weight): fragment pair (row group, 2 k-steps) is
// 1 KiB contiguous -- lane 16g+r holds 16 contiguous k of row r, feeding both MFMAs of the pair --
// so each weight load is one coalesced 16-byte-per-lane instruction, and the activation operand
// (same k permutation) is one 16-byte load per token row too; fp8 halves the bytes streamed per
// decode step versus bf16 (the whole expert bank is touched at decode batch sizes).
#include "common.h"

#define FP8_MAX 448.0f

// ---------------------------------------------------------------------------------------------
// 1. routing (single workgroup; T*K <= MOE_ROUTE_CAP pairs, E <= 64: decode batches)
// ---------------------------------------------------------------------------------------------
#define MOE_ROUTE_CAP 4096

__global__ void __launch_bounds__(1024) moe_route_kernel(const bf16* __restrict__ logits, int T, int E, int K,
                                                         int* __restrict__ sorted_tok, float* __restrict__ sorted_w,
                                                         int* __restrict__ offsets, int* __restrict__ inv) {
  __shared__ int cnt[64], cur[64];
  __shared__ int pe[MOE_ROUTE_CAP];    // expert of pair (t, j)
  __shared__ float pw[MOE_ROUTE_CAP];  // renormalised routing weight of pair (t, j)
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // pass 1: softmax (f32) + top-K + renormalise per token; count pairs per expert
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    float p[64];
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) {
      p[e] = (float)logits[(long)t * E + e];
      mx = fmaxf(mx, p[e]);
    }
    for (int e = 0; e < E; ++e) p[e] = __expf(p[e] - mx);
    float ws = 0.f;
    for (int j = 0; j < K; ++j) {
      int best = 0;
      for (int e = 1; e < E; ++e)
        if (p[e] > p[best]) best = e;
      atomicAdd(&cnt[best], 1);
      pe[t * K + j] = best;
      pw[t * K + j] = p[best];
      ws += p[best];
      p[best] = -1.f;
    }
    for (int j = 0; j < K; ++j) pw[t * K + j] /= ws;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cur[e] = acc;
      acc += cnt[e];
    }
    offsets[E] = acc;
  }
  __syncthreads();
  // pass 2: scatter pairs into their expert buckets (order inside a bucket is irrelevant: every
  // pair's rows are computed independently)
  for (int i = threadIdx.x; i < T * K; i += blockDim.x) {
    const int pos = atomicAdd(&cur[pe[i]], 1);
    inv[i] = pos;
    sorted_tok[pos] = i / K;
    sorted_w[pos] = pw[i];
  }
}

// ---------------------------------------------------------------------------------------------
// 1b. prefill routing + activation quantisation (any T): two launches instead of the torch
//     softmax / top-k / renormalise / argsort / bincount / cumsum / gather chain plus quant_rows.
//   moe_route_quant: one workgroup per token. Wave 0 routes it (one expert per lane: f32 softmax
//     numerators, K rounds of wave arg-max -- ties to the smaller expert id -- renormalised over the
//     top K, as moe_route_kernel); all four waves quantise the token's hidden row to e4m3 with the
//     row held in registers between the amax and the convert sweeps (read from HBM once).
//   moe_bucket: one workgroup counts the T*K pairs per expert in LDS, scans the offsets and
//     scatters the pairs into their buckets (order inside a bucket is irrelevant -- rows are
//     computed independently -- so the result is deterministic per row).
// ---------------------------------------------------------------------------------------------
template <int CPT>
__global__ void __launch_bounds__(256) moe_route_quant_kernel(const bf16* __restrict__ x, int ldx, int H,
                                                              const bf16* __restrict__ logits, int E, int K,
                                                              unsigned char* __restrict__ q, float* __restrict__ scale,
                                                              int* __restrict__ pe, float* __restrict__ pw) {
  __shared__ float red[4];
  const long t = blockIdx.x;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    float l = lane < E ? (float)logits[t * E + lane] : -INFINITY;
    float mx = l;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float p = lane < E ? __expf(l - mx) : -1.f;
    float ws = 0.f, mine = 0.f;
    int myj = -1;
    for (int j = 0; j < K; ++j) {
      float bv = p;
      int bi = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      ws += bv;
      if (lane == bi) { mine = p; myj = j; p = -1.f; }
    }
    if (myj >= 0) {
      pe[t * K + myj] = lane;
      pw[t * K + myj] = mine / ws;
    }
  }
  const uint4* xr = reinterpret_cast<const uint4*>(x + t * ldx);
  const int nchunk = H >> 3;
  float a[CPT][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nchunk) {
      unpack8(xr[c], a[i]);
#pragma unroll
      for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(a[i][k]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if (lane == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = amax > 0.f ? amax / FP8_MAX : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) scale[t] = sc;
  uint2* qr = reinterpret_cast<uint2*>(q + t * (long)H);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nchunk) {
      uint32_t w0 = 0, w1 = 0;
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][0] * inv, a[i][1] * inv, w0, false);
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][2] * inv, a[i][3] * inv, w0, true);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][4] * inv, a[i][5] * inv, w1, false);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][6] * inv, a[i][7] * inv, w1, true);
      qr[c] = make_uint2(w0, w1);
    }
  }
}

__global__ void __launch_bounds__(1024) moe_bucket_kernel(const int* __restrict__ pe, const float* __restrict__ pw,
                                                          int P, int E, int K, int* __restrict__ sorted_tok,
                                                          float* __restrict__ sorted_w, int* __restrict__ offsets,
                                                          int* __restrict__ inv) {
  __shared__ int cnt[64], cur[64];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += blockDim.x) atomicAdd(&cnt[pe[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cur[e] = acc;
      acc += cnt[e];
    }
    offsets[E] = acc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const int pos = atomicAdd(&cur[pe[i]], 1);
    inv[i] = pos;
    sorted_tok[pos] = i / K;
    sorted_w[pos] = pw[i];
  }
}

// ---------------------------------------------------------------------------------------------
// 2. dynamic per-row fp8 quantisation (one workgroup per row; row length multiple of 8)
// ---------------------------------------------------------------------------------------------
__global__ void quant_rows_kernel(const bf16* __restrict__ x, int ld, int n, unsigned char* __restrict__ q,
                                  float* __restrict__ scale) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (long)row * ld);
  float amax = 0.f;
  for (int c = threadIdx.x; c < n / 8; c += blockDim.x) {
    float f[8];
    unpack8(xr[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(f[i]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) amax = fmaxf(amax, red[i]);
  const float s = amax > 0.f ? amax / FP8_MAX : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint2* qr = reinterpret_cast<uint2*>(q + (long)row * n);
  for (int c = threadIdx.x; c < n / 8; c += blockDim.x) {
    float f[8];
    unpack8(xr[c], f);
    uint32_t w0 = 0, w1 = 0;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[0] * inv, f[1] * inv, w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f[2] * inv, f[3] * inv, w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[4] * inv, f[5] * inv, w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f[6] * inv, f[7] * inv, w1, true);
    qr[c] = make_uint2(w0, w1);
  }
}

// 2b. prefill experts: SiLU(gate) * up of the 16-row-interleaved W13 GEMM output, quantised per row
//     to fp8 in the same pass (one workgroup per row, the row held in registers between the amax
//     and the quantise sweeps): the bf16 activation never round-trips through HBM.
template <int CPT>
__global__ void __launch_bounds__(256) silu_quant_rows_kernel(const bf16* __restrict__ gu, int F,
                                                              unsigned char* __restrict__ q,
                                                              float* __restrict__ scale) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const uint4* gr = reinterpret_cast<const uint4*>(gu + row * 2L * F);
  const int nchunk = F >> 3;   // 8 outputs per chunk: output cols 8c..8c+7 = pair c/2, half c&1
  float a[CPT][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nchunk) {
      float g[8], u[8];
      const int pair = c >> 1, half = c & 1;
      unpack8(gr[pair * 4 + half], g);
      unpack8(gr[pair * 4 + 2 + half], u);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        // silu in the activation dtype, like silu_mul_kernel: bf16(silu(g)) * u, rounded to bf16
        a[i][k] = (float)(bf16)((float)(bf16)(g[k] / (1.f + __expf(-g[k]))) * u[k]);
        amax = fmaxf(amax, fabsf(a[i][k]));
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = amax > 0.f ? amax / FP8_MAX : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) scale[row] = sc;
  uint2* qr = reinterpret_cast<uint2*>(q + row * (long)F);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nchunk) {
      uint32_t w0 = 0, w1 = 0;
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][0] * inv, a[i][1] * inv, w0, false);
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][2] * inv, a[i][3] * inv, w0, true);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][4] * inv, a[i][5] * inv, w1, false);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(a[i][6] * inv, a[i][7] * inv, w1, true);
      qr[c] = make_uint2(w0, w1);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 3/4. grouped fp8 GEMM over expert buckets
// ---------------------------------------------------------------------------------------------
#define MOE_EPI_SILU 1
#define MOE_EPI_ROUTEW 2

template <int NTF, int NW, int EPI>
__global__ void __launch_bounds__(NW * 64) moe_gemm_kernel(
    const unsigned char* __restrict__ Xq, const float* __restrict__ xs, const int* __restrict__ rows,
    const int* __restrict__ offsets, const unsigned char* __restrict__ Wt, const float* __restrict__ ws,
    const float* __restrict__ route_w, bf16* __restrict__ Y, int N, int K) {
  constexpr int NR = 16 * NTF;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [NW][NR][64]
  const int e = blockIdx.y;
  const int p0 = offsets[e], p1 = offsets[e + 1];
  if (p1 <= p0) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, col = lane & 15;
  const int n0 = blockIdx.x * NR;
  const int kper = K / NW, kb = w * kper;
  const long kpairs = K / 64;
  const unsigned char* We = Wt + (long)e * N * K;
  for (int c0 = p0; c0 < p1; c0 += 64) {  // token chunks of 64 pairs
    const int nrow = min(64, p1 - c0);
    f32x4 acc[NTF][4];
#pragma unroll
    for (int f = 0; f < NTF; ++f)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    // lane (g, col) owns physical k = 64p + 16g .. +15 of its token row: one 16-B load per row tile
    // and k-pair, matching the weight tiling (ops/moe.py tile_fp8_weight); bytes 0-7 feed the
    // first MFMA of the pair, bytes 8-15 the second
    const unsigned char* xr[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int pr = c0 + min(16 * m + col, nrow - 1);
      const int src = rows ? rows[pr] : pr;
      xr[m] = Xq + (long)src * K + kb + 16 * g;
    }
    // one k-pair of W (NTF fragments) and X (4 token tiles) in flight ahead of the MFMAs using
    // the previous one (register double buffer)
    uint4 wn[NTF], xn[4];
    auto fetch = [&](int k) {
#pragma unroll
      for (int f = 0; f < NTF; ++f)
        wn[f] = *reinterpret_cast<const uint4*>(We + (((long)(n0 / 16 + f) * kpairs + (kb + k) / 64) * 64 + lane) * 16);
#pragma unroll
      for (int m = 0; m < 4; ++m) xn[m] = *reinterpret_cast<const uint4*>(xr[m] + k);
    };
    fetch(0);
    for (int k = 0; k < kper; k += 64) {
      uint4 wv[NTF], xv[4];
#pragma unroll
      for (int f = 0; f < NTF; ++f) wv[f] = wn[f];
#pragma unroll
      for (int m = 0; m < 4; ++m) xv[m] = xn[m];
      if (k + 64 < kper) fetch(k + 64);
#pragma unroll
      // both k-halves of one accumulator back to back (a dependent MFMA pair): interleaving the
      // halves across all NTF*4 accumulators made hipcc shuffle them between AGPRs every pair
      for (int f = 0; f < NTF; ++f) {
        const long a0 = ((long)wv[f].y << 32 | wv[f].x), a1 = ((long)wv[f].w << 32 | wv[f].z);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const long b0 = ((long)xv[m].y << 32 | xv[m].x), b1 = ((long)xv[m].w << 32 | xv[m].z);
          acc[f][m] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a0, b0, acc[f][m], 0, 0, 0);
          acc[f][m] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a1, b1, acc[f][m], 0, 0, 0);
        }
      }
    }
    float* mine = red + w * NR * 64;
#pragma unroll
    for (int f = 0; f < NTF; ++f)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) mine[(16 * f + 4 * g + r) * 64 + 16 * m + col] = acc[f][m][r];
    __syncthreads();
    constexpr int OUTN = (EPI == MOE_EPI_SILU) ? NR / 2 : NR;
    const int ldy = (EPI == MOE_EPI_SILU) ? N / 2 : N;
    for (int idx = threadIdx.x; idx < 64 * (OUTN / 8); idx += NW * 64) {
      const int m = idx / (OUTN / 8), c8 = (idx % (OUTN / 8)) * 8;
      if (m >= nrow) continue;
      const int pr = c0 + m;
      const float sx = xs[rows ? rows[pr] : pr];
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (EPI == MOE_EPI_SILU) {
          const int c = c8 + j, pair = c >> 4, jj = c & 15;
          const int rg = 32 * pair + jj, ru = rg + 16;
          float gs = 0.f, us = 0.f;
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) {
            gs += red[(ww * NR + rg) * 64 + m];
            us += red[(ww * NR + ru) * 64 + m];
          }
          const float gv = (float)(bf16)(gs * sx * ws[(long)e * N + n0 + rg]);
          const float uv = (float)(bf16)(us * sx * ws[(long)e * N + n0 + ru]);
          o[j] = (float)(bf16)(gv / (1.f + __expf(-gv))) * uv;
        } else {
          float s = 0.f;
#pragma unroll
          for (int ww = 0; ww < NW; ++ww) s += red[(ww * NR + c8 + j) * 64 + m];
          o[j] = s * sx * ws[(long)e * N + n0 + c8 + j] * route_w[pr];
        }
      }
      const int ncol = (EPI == MOE_EPI_SILU) ? (n0 / 2 + c8) : (n0 + c8);
      *reinterpret_cast<uint4*>(Y + (long)pr * ldy + ncol) = pack8(o);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// 5. combine the K expert outputs of each token
// ---------------------------------------------------------------------------------------------
// W (optional, prefill path): routing weight of each sorted pair, applied here in f32 (the decode
// path already scaled its rows inside the W2 GEMM epilogue)
__global__ void moe_combine_kernel(const bf16* __restrict__ Y2, const int* __restrict__ inv,
                                   const float* __restrict__ W, int K, int H, bf16* __restrict__ out) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < K; ++j) {
      const int pos = inv[t * K + j];
      const float wj = W ? W[pos] : 1.f;
      float f[8];
      unpack8(reinterpret_cast<const uint4*>(Y2 + (long)pos * H)[c], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wj * f[i];
    }
    reinterpret_cast<uint4*>(out + (long)t * H)[c] = pack8(acc);
  }
}

PENNY_API int penny_moe_route(const void* logits, int T, int E, int K, int* sorted_tok, float* sorted_w, int* offsets,
                              int* inv, hipStream_t stream) {
  if (T <= 0) return 0;
  if (E > 64 || K > 8 || K > E || T * K > MOE_ROUTE_CAP) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(1024), 0, stream, (const bf16*)logits, T, E, K, sorted_tok,
                     sorted_w, offsets, inv);
  PENNY_RETURN_LAUNCH();
}

// prefill routing + quantisation: x [T, H] (row stride ldx) bf16, logits [T, E] bf16 ->
// xq [T, H] e4m3, xs [T]; pair expert / weight scratch pe, pw [T*K]; buckets sorted_tok /
// sorted_w [T*K], offsets [E+1], inverse map inv [T*K] (pair t*K+j -> sorted position)
PENNY_API int penny_moe_route_quant(const void* x, int ldx, const void* logits, int T, int H, int E, int K, void* xq,
                                    float* xs, int* pe, float* pw, int* sorted_tok, float* sorted_w, int* offsets,
                                    int* inv, hipStream_t stream) {
  if (T <= 0) return 0;
  if (E > 64 || K < 1 || K > 8 || K > E || H % 8 || ldx % 8) return (int)hipErrorInvalidValue;
  const int cpt = (H / 8 + 255) / 256;
#define RQ_CASE(C)                                                                                        \
  if (cpt <= C) {                                                                                         \
    hipLaunchKernelGGL(moe_route_quant_kernel<C>, dim3(T), dim3(256), 0, stream, (const bf16*)x, ldx, H, \
                       (const bf16*)logits, E, K, (unsigned char*)xq, xs, pe, pw);                       \
  } else
  RQ_CASE(1) RQ_CASE(2) RQ_CASE(4) RQ_CASE(8) return (int)hipErrorInvalidValue;
#undef RQ_CASE
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return (int)err;
  hipLaunchKernelGGL(moe_bucket_kernel, dim3(1), dim3(1024), 0, stream, pe, pw, T * K, E, K, sorted_tok, sorted_w,
                     offsets, inv);
  PENNY_RETURN_LAUNCH();
}

// gu [rows, 2F] bf16 (16-column-interleaved gate|up) -> q [rows, F] e4m3, scale [rows] f32
PENNY_API int penny_silu_quant_rows_fp8(const void* gu, int rows, int F, void* q, float* scale, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (F % 16) return (int)hipErrorInvalidValue;
  const int cpt = (F / 8 + 255) / 256;
#define SQ_CASE(C)                                                                                        \
  if (cpt <= C) {                                                                                         \
    hipLaunchKernelGGL(silu_quant_rows_kernel<C>, dim3(rows), dim3(256), 0, stream, (const bf16*)gu, F,   \
                       (unsigned char*)q, scale);                                                         \
    PENNY_RETURN_LAUNCH();                                                                                \
  }
  SQ_CASE(1) SQ_CASE(2) SQ_CASE(4) SQ_CASE(8) SQ_CASE(16)
#undef SQ_CASE
  return (int)hipErrorInvalidValue;
}

PENNY_API int penny_quant_rows_fp8(const void* x, int ld, int rows, int n, void* q, float* scale, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(quant_rows_kernel, dim3(rows), dim3(256), 0, stream, (const bf16*)x, ld, n, (unsigned char*)q,
                     scale);
  PENNY_RETURN_LAUNCH();
}

template <int NTF>
static int moe_gemm_launch(const void* Xq, const float* xs, const int* rows, const int* offsets, const void* Wt,
                           const float* ws, const float* route_w, void* Y, int E, int N, int K, int epi,
                           hipStream_t stream) {
  dim3 grid(N / (16 * NTF), E);
  // waves split K: as many as divide it into whole 64-wide k-pairs (4 for every real model)
#define MOE_LAUNCH(NW_)                                                                                          \
  {                                                                                                              \
    const size_t lds = (size_t)NW_ * 16 * NTF * 64 * sizeof(float);                                             \
    if (epi == MOE_EPI_SILU)                                                                                     \
      hipLaunchKernelGGL((moe_gemm_kernel<NTF, NW_, MOE_EPI_SILU>), grid, dim3(NW_ * 64), lds, stream,          \
                         (const unsigned char*)Xq, xs, rows, offsets, (const unsigned char*)Wt, ws, route_w,     \
                         (bf16*)Y, N, K);                                                                        \
    else                                                                                                         \
      hipLaunchKernelGGL((moe_gemm_kernel<NTF, NW_, MOE_EPI_ROUTEW>), grid, dim3(NW_ * 64), lds, stream,        \
                         (const unsigned char*)Xq, xs, rows, offsets, (const unsigned char*)Wt, ws, route_w,     \
                         (bf16*)Y, N, K);                                                                        \
  }
  if (K % 256 == 0) MOE_LAUNCH(4)
  else if (K % 128 == 0) MOE_LAUNCH(2)
  else MOE_LAUNCH(1)
#undef MOE_LAUNCH
  PENNY_RETURN_LAUNCH();
}

// epi 1: SiLU-gated (W13 interleaved, Y [P, N/2]); epi 2: scale by routing weight (Y [P, N]).
// ntf: 16-row weight groups per workgroup (2 or 4).
PENNY_API int penny_moe_gemm_fp8(const void* Xq, const float* xs, const int* rows, const int* offsets, const void* Wt,
                                 const float* ws, const float* route_w, void* Y, int E, int N, int K, int epi,
                                 int ntf, hipStream_t stream) {
  if ((ntf != 2 && ntf != 4) || N % (16 * ntf) || K % 64) return (int)hipErrorInvalidValue;
  if (ntf == 4) return moe_gemm_launch<4>(Xq, xs, rows, offsets, Wt, ws, route_w, Y, E, N, K, epi, stream);
  return moe_gemm_launch<2>(Xq, xs, rows, offsets, Wt, ws, route_w, Y, E, N, K, epi, stream);
}

PENNY_API int penny_moe_combine(const void* Y2, const int* inv, int T, int K, int H, void* out, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, stream, (const bf16*)Y2, inv, (const float*)nullptr,
                     K, H, (bf16*)out);
  PENNY_RETURN_LAUNCH();
}

// out[t] = sum_j W[inv[t*K+j]] * Y2[inv[t*K+j]]  (f32 accumulate; prefill combine, no atomics)
PENNY_API int penny_moe_combine_weighted(const void* Y2, const int* inv, const float* W, int T, int K, int H,
                                         void* out, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, stream, (const bf16*)Y2, inv, W, K, H, (bf16*)out);
  PENNY_RETURN_LAUNCH();
}
