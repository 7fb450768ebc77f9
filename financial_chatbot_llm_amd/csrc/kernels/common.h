// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; block sizes are multiples of 64.
//  * bf16 tensors are moved 16 B (8 elements) per lane per instruction (uint4), math in f32.
//  * every launcher is `extern "C"`, takes raw device pointers + a hipStream_t, never
//    allocates or synchronises (so it can be captured into a hipGraph), and returns the
//    hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PENNY_API extern "C" __attribute__((visibility("default")))

// Device-side bounds checks, compiled only into the debug library (PENNY_KERNEL_DEBUG=1 python -m
// financial_chatbot_llm_amd._build --debug -> _lib/libpenny_kernels_debug.so, loaded when
// PENNY_KERNEL_DEBUG=1): print the failing condition and trap at the first bad index, instead of
// an out-of-bounds access that faults somewhere later.  The production library has none of them.
#ifdef PENNY_KERNEL_DEBUG
#include <stdio.h>
#define PENNY_DASSERT(cond)                                                                         \
  do {                                                                                              \
    if (!(cond)) {                                                                                  \
      printf("[penny] device assert failed: %s (%s:%d, block %d thread %d)\n", #cond, __FILE__,     \
             __LINE__, (int)blockIdx.x, (int)threadIdx.x);                                          \
      __builtin_trap();                                                                             \
    }                                                                                               \
  } while (0)
#else
#define PENNY_DASSERT(cond) ((void)0)
#endif

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// 8 x bf16 <-> uint4 (16 B) helpers
union Pack8 {
  uint4 u;
  bf16x8 v;
  bf16 e[8];
};

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  Pack8 p;
  p.u = u;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)p.e[i];
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  Pack8 p;
#pragma unroll
  for (int i = 0; i < 8; ++i) p.e[i] = (bf16)f[i];
  return p.u;
}

// 8 consecutive outputs of a split-K GEMM (gemm_splitk.hip): the sum of its S f32 slabs (slab
// stride `ss` floats), rounded to bf16 exactly where the unsplit GEMM would round its output.
__device__ __forceinline__ void load8_slabs(const float* __restrict__ p, int S, long ss, float* o) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll 4
  for (int s = 1; s < S; ++s) {
    a += *reinterpret_cast<const f32x4*>(p + s * ss);
    b += *reinterpret_cast<const f32x4*>(p + s * ss + 4);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (float)(bf16)a[j];
    o[4 + j] = (float)(bf16)b[j];
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// splitmix64 -> two uniforms in (0, 1); counter-based so results are launch-order independent.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float u01_from_bits(uint32_t b) {
  // 24 random mantissa bits, strictly inside (0, 1)
  return ((float)(b >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Gumbel noise of vocabulary entry idx for a row seeded `seed` (K12 and the fused LM-head sampler
// draw the SAME noise, so a row samples the same token on either path for equal logits)
__device__ __forceinline__ float gumbel_noise(unsigned long long seed, int idx) {
  const uint64_t r = mix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(idx + 1)));
  return -__logf(-__logf(u01_from_bits((uint32_t)r)));
}

// running (max value, smallest index on ties) of a Gumbel-max / argmax reduction
__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

#define PENNY_RETURN_LAUNCH() return (int)hipGetLastError()
