// K12: fused temperature + Gumbel-max sampler / greedy argmax over the full vocabulary.
//
// argmax_i(logit_i / T + Gumbel_i) is an exact sample from softmax(logit / T), so one read of
// the logits row replaces softmax + cumsum + search.  Noise is counter-based (splitmix64 of
// (per-row seed, token index)): a request's sample depends only on its own seed and the step,
// never on batch composition or launch order.  T <= 0 selects greedy argmax.  Ties resolve to
// the smallest index.  One 1024-thread workgroup per row; the vocab (128256 for Llama-3) is
// read 16 B per lane.
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

__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
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
                                                             float* __restrict__ pv, int* __restrict__ pi, int V) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x, split = blockIdx.y;
  const T* lr = logits + row * row_stride;
  const float temp = temps[row];
  const bool greedy = !(temp > 0.f);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const unsigned long long seed = seeds[row];
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
      const int idx = c * 8 + k;
      float v = f[k];
      if (!greedy) {
        const uint64_t r = mix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(idx + 1)));
        v = v * inv_t - __logf(-__logf(u01_from_bits((uint32_t)r)));
      }
      better(bv, bi, v, idx);
    }
  }
  if (split == SAMPLE_SPLITS - 1) {  // tail (V not a multiple of 8)
    for (int idx = (V & ~7) + threadIdx.x; idx < V; idx += blockDim.x) {
      float v = (float)lr[idx];
      if (!greedy) {
        const uint64_t r = mix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(idx + 1)));
        v = v * inv_t - __logf(-__logf(u01_from_bits((uint32_t)r)));
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

__global__ void sample_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi, int* __restrict__ out) {
  const int row = blockIdx.x, lane = threadIdx.x;
  float bv = lane < SAMPLE_SPLITS ? pv[row * SAMPLE_SPLITS + lane] : -INFINITY;
  int bi = lane < SAMPLE_SPLITS ? pi[row * SAMPLE_SPLITS + lane] : 0x7fffffff;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  if (lane == 0) out[row] = bi;
}

// workspace: B * SAMPLE_SPLITS floats + B * SAMPLE_SPLITS ints
PENNY_API int penny_sample(const void* logits, int is_fp32, long row_stride, const float* temps,
                           const unsigned long long* seeds, int* out, void* workspace, int B, int V,
                           hipStream_t stream) {
  if (B <= 0) return 0;
  float* pv = (float*)workspace;
  int* pi = (int*)(pv + (long)B * SAMPLE_SPLITS);
  dim3 grid(B, SAMPLE_SPLITS);
  if (is_fp32) {
    hipLaunchKernelGGL(sample_partial_kernel<float>, grid, dim3(256), 0, stream, (const float*)logits, row_stride,
                       temps, seeds, pv, pi, V);
  } else {
    hipLaunchKernelGGL(sample_partial_kernel<bf16>, grid, dim3(256), 0, stream, (const bf16*)logits, row_stride,
                       temps, seeds, pv, pi, V);
  }
  hipLaunchKernelGGL(sample_final_kernel, dim3(B), dim3(64), 0, stream, pv, pi, out);
  PENNY_RETURN_LAUNCH();
}
