// K12: fused temperature + Gumbel-max sampler / greedy argmax over the full vocabulary.
//
// argmax_i(logit_i / T + Gumbel_i) is an exact sample from softmax(logit / T), so one read of
// the logits row replaces softmax + cumsum + search.  Noise is counter-based (splitmix64 of
// (per-row seed, token index)): a request's sample depends only on its own seed and the step,
// never on batch composition or launch order.  T <= 0 selects greedy argmax.  Ties resolve to
// the smallest index.  One 1024-thread workgroup per row; the vocab (128256 for Llama-3) is
// read 16 B per lane.
//
// top-k / top-p (nucleus) without a sort: a per-row radix select finds a logit THRESHOLD and the
// sampler treats every logit below it as -inf.  top-k: 4 passes of an 8-bit-digit histogram over
// order-preserving uint32 keys find the k-th largest logit exactly.  top-p (over the
// temperature-scaled distribution renormalised to the top-k survivors, as vLLM/HF apply them):
// the same 4 passes histogram probability MASS instead of counts and descend to the smallest
// logit whose cumulative mass from the top reaches p.  Everything stays on the device (no host
// sync, no sort buffers), so the filter is captured in the decode hipGraphs; rows with k <= 0 and
// p >= 1 leave after reading their two parameters.
#include "common.h"

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f);
template <>
__device__ __forceinline__ void load8<bf16>(const bf16* p, float* f) {
  unpack8(*reinterpret_cast<const uint4*>(p), f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float keyf(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename T>
__device__ __forceinline__ float ld1(const T* p) { return (float)*p; }

// 256 bins (bins[0..255], ascending digit) -> the digit whose bin holds the `target`-th unit of
// weight counting from the TOP, and the weight above it.  One wave: lane l owns bins 4l..4l+3.
__device__ __forceinline__ void find_from_top(const float* bins, float target, int& digit, float& above) {
  const int lane = threadIdx.x & 63;
  const float b0 = bins[4 * lane], b1 = bins[4 * lane + 1], b2 = bins[4 * lane + 2], b3 = bins[4 * lane + 3];
  const float seg = b0 + b1 + b2 + b3;
  float suf = seg;                                   // inclusive suffix sum over lanes >= l
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float v = __shfl_down(suf, o, 64);
    if (lane + o < 64) suf += v;
  }
  const float total = __shfl(suf, 0, 64);
  target = fminf(fmaxf(target, 0.f), total);         // rounding guard (mass sums)
  const float abv = suf - seg;
  // crossing lane: abv < target <= abv + seg (the highest such lane when target <= 0)
  const bool hit = seg > 0.f && abv < target && target <= suf;
  unsigned long long m = __ballot(hit);
  if (m == 0) m = __ballot(seg > 0.f);               // target == 0 or rounding: highest nonzero
  const int src = m ? 63 - __clzll(m) : 0;
  float a = __shfl(abv, src, 64);
  const float c3 = __shfl(b3, src, 64), c2 = __shfl(b2, src, 64), c1 = __shfl(b1, src, 64);
  int d = 4 * src;
  if (a + c3 >= target && c3 > 0.f) d += 3;
  else if ((a += c3, a + c2 >= target) && c2 > 0.f) d += 2;
  else if ((a += c2, a + c1 >= target) && c1 > 0.f) d += 1;
  else a += c1;
  digit = d;
  above = a;
}

// One 1024-thread workgroup per row -> thresh[row] (a logit; -inf = keep everything).
template <typename T>
__global__ void __launch_bounds__(1024) topk_topp_threshold_kernel(const T* __restrict__ logits, long row_stride,
                                                                   const float* __restrict__ temps,
                                                                   const int* __restrict__ topk,
                                                                   const float* __restrict__ topp,
                                                                   float* __restrict__ thresh, int V) {
  // per-wave digit histograms in INTEGERS: counts for top-k, probability mass in 2^-44 fixed point
  // for top-p -- integer adds commute, so the threshold is bitwise independent of the order in
  // which waves and lanes reach the atomics (float atomics made the nucleus edge run-dependent)
  __shared__ unsigned long long hist[16][256];
  __shared__ float red[16];
  __shared__ float bins[256];
  __shared__ uint32_t s_prefix;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int k = topk[row];
  const float p = topp[row], temp = temps[row];
  const bool do_k = k > 0 && k < V, do_p = p < 1.f;
  if (!(temp > 0.f) || (!do_k && !do_p)) {
    if (tid == 0) thresh[row] = -INFINITY;
    return;
  }
  const T* lr = logits + row * row_stride;
  const float inv_t = 1.f / temp;
  uint32_t prefix = 0, pmask = 0;      // selected high digits so far (keys matching are candidates)
  // ---- top-k: radix select of the k-th largest key ---------------------------------------------
  if (do_k) {
    float want = (float)k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 16 * 256; i += 1024) (&hist[0][0])[i] = 0ull;
      __syncthreads();
      for (int i = tid; i < V; i += 1024) {
        const uint32_t key = fkey(ld1(lr + i));
        if ((key & pmask) == prefix) atomicAdd(&hist[wid][(key >> shift) & 255], 1ull);
      }
      __syncthreads();
      if (tid < 256) {
        unsigned long long t = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) t += hist[w][tid];
        bins[tid] = (float)t;
      }
      __syncthreads();
      if (wid == 0) {
        int d;
        float above;
        find_from_top(bins, want, d, above);
        if (lane == 0) {
          s_prefix = prefix | ((uint32_t)d << shift);
          red[0] = want - above;
        }
      }
      __syncthreads();
      prefix = s_prefix;
      want = red[0];
      pmask |= 255u << shift;
      __syncthreads();
    }
  }
  const uint32_t kfloor = do_k ? prefix : 0u;        // keys >= kfloor survive top-k
  if (!do_p) {
    if (tid == 0) thresh[row] = keyf(kfloor);
    return;
  }
  // ---- top-p over the renormalised top-k survivors --------------------------------------------
  float mx = -INFINITY;
  for (int i = tid; i < V; i += 1024) mx = fmaxf(mx, ld1(lr + i));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int w = 1; w < 16; ++w) mx = fmaxf(mx, red[w]);
  __syncthreads();
  prefix = 0;
  pmask = 0;
  float want = -1.f;                                  // set from the first pass's total
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 16 * 256; i += 1024) (&hist[0][0])[i] = 0ull;
    __syncthreads();
    for (int i = tid; i < V; i += 1024) {
      const float l = ld1(lr + i);
      const uint32_t key = fkey(l);
      // exp <= 1 (l <= mx): x 2^44 fits 45 bits, a 128k-entry vocabulary sums below 2^62
      if (key >= kfloor && (key & pmask) == prefix)
        atomicAdd(&hist[wid][(key >> shift) & 255],
                  (unsigned long long)(__expf((l - mx) * inv_t) * 17592186044416.f));
    }
    __syncthreads();
    if (tid < 256) {
      unsigned long long t = 0;
#pragma unroll
      for (int w = 0; w < 16; ++w) t += hist[w][tid];
      bins[tid] = (float)t * 5.684341886080802e-14f;   // 2^-44
    }
    __syncthreads();
    if (wid == 0) {
      if (want < 0.f) {                                // first pass: total mass of the survivors
        float z = bins[4 * lane] + bins[4 * lane + 1] + bins[4 * lane + 2] + bins[4 * lane + 3];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
        want = p * z;
      }
      int d;
      float above;
      find_from_top(bins, want, d, above);
      if (lane == 0) {
        s_prefix = prefix | ((uint32_t)d << shift);
        red[0] = want - above;
      }
    }
    __syncthreads();
    prefix = s_prefix;
    want = red[0];
    pmask |= 255u << shift;
    __syncthreads();
  }
  if (tid == 0) thresh[row] = keyf(max(prefix, kfloor));
}

// Pass 1: grid (B, SPLITS); each 256-thread workgroup scans one vocab slice of one row and writes
// its (best value, index).  Pass 2: one wave per row merges the SPLITS candidates.  Splitting the
// row keeps the whole chip busy at decode batch sizes (B = 64 rows alone would occupy 64 CUs,
// and the per-element noise generation makes this pass VALU-, not bandwidth-, bound).
#define SAMPLE_SPLITS 16

template <typename T>
__global__ void __launch_bounds__(256) sample_partial_kernel(const T* __restrict__ logits, long row_stride,
                                                             const float* __restrict__ temps,
                                                             const unsigned long long* __restrict__ seeds,
                                                             const float* __restrict__ thresh,
                                                             float* __restrict__ pv, int* __restrict__ pi, int V,
                                                             int voff) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x, split = blockIdx.y;
  const T* lr = logits + row * row_stride;
  const float temp = temps[row];
  const bool greedy = !(temp > 0.f);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const unsigned long long seed = seeds[row];
  const float floor_l = (thresh != nullptr && !greedy) ? thresh[row] : -INFINITY;   // top-k/top-p cut
  const int nch = V >> 3;
  const int per = (nch + SAMPLE_SPLITS - 1) / SAMPLE_SPLITS;
  const int c0 = split * per, c1 = min(nch, c0 + per);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    float f[8];
    load8<T>(lr + c * 8, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = voff + c * 8 + k;     // global token id (vocab shard offset)
      float v = f[k];
      if (v < floor_l) continue;
      if (!greedy) {
        v = v * inv_t + gumbel_noise(seed, idx);
      }
      better(bv, bi, v, idx);
    }
  }
  if (split == SAMPLE_SPLITS - 1) {  // tail (V not a multiple of 8)
    for (int loc = (V & ~7) + threadIdx.x; loc < V; loc += blockDim.x) {
      const int idx = voff + loc;
      float v = (float)lr[loc];
      if (v < floor_l) continue;
      if (!greedy) {
        v = v * inv_t + gumbel_noise(seed, idx);
      }
      better(bv, bi, v, idx);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wid] = bv;
    si[wid] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) better(bv, bi, sv[w], si[w]);
    pv[row * SAMPLE_SPLITS + split] = bv;
    pi[row * SAMPLE_SPLITS + split] = bi;
  }
}

__global__ void sample_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi, int* __restrict__ out,
                                    int* __restrict__ pairs) {
  const int row = blockIdx.x, lane = threadIdx.x;
  float bv = lane < SAMPLE_SPLITS ? pv[row * SAMPLE_SPLITS + lane] : -INFINITY;
  int bi = lane < SAMPLE_SPLITS ? pi[row * SAMPLE_SPLITS + lane] : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  if (lane == 0) {
    if (out) out[row] = bi;
    if (pairs) {
      pairs[2 * row] = __float_as_int(bv);
      pairs[2 * row + 1] = bi;
    }
  }
}

// workspace: B * SAMPLE_SPLITS floats + B * SAMPLE_SPLITS ints + B floats (thresholds)
// top_k / top_p: per-row filters (nullptr: none in this launch)
PENNY_API int penny_sample(const void* logits, int is_fp32, long row_stride, const float* temps,
                           const unsigned long long* seeds, const int* top_k, const float* top_p, int* out,
                           void* workspace, int B, int V, hipStream_t stream) {
  if (B <= 0) return 0;
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + (long)B * SAMPLE_SPLITS);
  float* th = nullptr;
  if (top_k != nullptr && top_p != nullptr) {
    th = (float*)(pi + (long)B * SAMPLE_SPLITS);
    if (is_fp32) {
      hipLaunchKernelGGL(topk_topp_threshold_kernel<float>, dim3(B), dim3(1024), 0, stream, (const float*)logits,
                         row_stride, temps, top_k, top_p, th, V);
    } else {
      hipLaunchKernelGGL(topk_topp_threshold_kernel<bf16>, dim3(B), dim3(1024), 0, stream, (const bf16*)logits,
                         row_stride, temps, top_k, top_p, th, V);
    }
  }
  dim3 grid(B, SAMPLE_SPLITS);
  if (is_fp32) {
    hipLaunchKernelGGL(sample_partial_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, row_stride,
                       temps, seeds, th, pv, pi, V, 0);
  } else {
    hipLaunchKernelGGL(sample_partial_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)logits, row_stride,
                       temps, seeds, th, pv, pi, V, 0);
  }
  hipLaunchKernelGGL(sample_final_kernel, dim3(B), dim3(64), 0, stream, pv, pi, out, (int*)nullptr);
  PENNY_RETURN_LAUNCH();
}

// Vocabulary-parallel sampling of one TP rank's logit shard [B, V] (global ids voff .. voff+V-1):
// pairs [B, 2] int32 = each row's best (score bits, global token id); the ranks' pairs are then
// all-gathered and the best taken (ops.sampling.pick_pairs) -- [B, 2] on the wire instead of the
// [B, V*tp] logits.  No top-k / top-p (they need the whole distribution).
// workspace: B * SAMPLE_SPLITS floats + as many ints.
PENNY_API int penny_sample_shard(const void* logits, int is_fp32, long row_stride, const float* temps,
                                 const unsigned long long* seeds, int* pairs, void* workspace, int B, int V, int voff,
                                 hipStream_t stream) {
  if (B <= 0) return 0;
  if (!pairs || !workspace || V <= 0 || voff < 0) return (int)hipErrorInvalidValue;
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + (long)B * SAMPLE_SPLITS);
  dim3 grid(B, SAMPLE_SPLITS);
  if (is_fp32) {
    hipLaunchKernelGGL(sample_partial_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, row_stride,
                       temps, seeds, (const float*)nullptr, pv, pi, V, voff);
  } else {
    hipLaunchKernelGGL(sample_partial_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)logits, row_stride,
                       temps, seeds, (const float*)nullptr, pv, pi, V, voff);
  }
  hipLaunchKernelGGL(sample_final_kernel, dim3(B), dim3(64), 0, stream, pv, pi, (int*)nullptr, pairs);
  PENNY_RETURN_LAUNCH();
}

// Threshold only (tests / diagnostics): thresh[B] logits.
PENNY_API int penny_topk_topp_threshold(const void* logits, int is_fp32, long row_stride, const float* temps,
                                        const int* top_k, const float* top_p, float* thresh, int B, int V,
                                        hipStream_t stream) {
  if (B <= 0) return 0;
  if (is_fp32) {
    hipLaunchKernelGGL(topk_topp_threshold_kernel<float>, dim3(B), dim3(1024), 0, stream, (const float*)logits,
                       row_stride, temps, top_k, top_p, thresh, V);
  } else {
    hipLaunchKernelGGL(topk_topp_threshold_kernel<bf16>, dim3(B), dim3(1024), 0, stream, (const bf16*)logits,
                       row_stride, temps, top_k, top_p, thresh, V);
  }
  PENNY_RETURN_LAUNCH();
}
