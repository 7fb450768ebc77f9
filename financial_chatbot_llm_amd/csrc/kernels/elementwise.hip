// K9 epilogue (SiLU-gated MLP), K14 GELU, K1 token-embedding gather (vocab-parallel aware).
//
// All bandwidth-bound: 16 B per lane per access, grid-stride loops capped near
// 256 CUs x 8 workgroups (cdna_hip_programming.md Guideline 11).
#include "common.h"

// out[t, f] = silu(gate[t, f]) * up[t, f] from the fused gate|up GEMM output.  Column layout of gu:
// interleave16 = 0: [gate 0..F-1 | up 0..F-1];  interleave16 = 1: 16-column groups alternate
// gate/up (gate 16i..16i+15, up 16i..16i+15), the layout the decode skinny GEMM's fused SiLU
// epilogue needs, so one weight tensor serves both paths.
// grid (chunks/256, rows): no 64-bit index division on the hot path (it dominated at decode sizes)
__global__ void silu_mul_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out, int T, int F, int il16) {
  const int cpr = F >> 3;  // 16-byte chunks per output row
  const long t = blockIdx.y;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < cpr; c += gridDim.x * blockDim.x) {
    const uint4* row = reinterpret_cast<const uint4*>(gu + t * 2L * F);
    float g[8], u[8], o[8];
    if (il16) {  // chunk c covers output cols 8c..8c+7 = pair (8c)/16, half (c & 1)
      const int pair = c >> 1, half = c & 1;
      unpack8(row[pair * 4 + half], g);
      unpack8(row[pair * 4 + 2 + half], u);
    } else {
      unpack8(row[c], g);
      unpack8(row[cpr + c], u);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // HF SiLU is computed in the activation dtype: silu(bf16) -> bf16, then * up in bf16
      const float s = (float)(bf16)(g[k] / (1.f + __expf(-g[k])));
      o[k] = s * u[k];
    }
    reinterpret_cast<uint4*>(out + t * (long)F)[c] = pack8(o);
  }
}

// exact (erf) GELU in place, as BERT's "gelu" activation
__global__ void gelu_kernel(bf16* __restrict__ x, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    uint4* p = reinterpret_cast<uint4*>(x) + i;
    float v[8];
    unpack8(*p, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.5f * v[k] * (1.f + erff(v[k] * 0.70710678118654752f));
    *p = pack8(v);
  }
}

// out[t] = table[ids[t] - vocab_start] if the id is in this rank's shard, else 0 (the
// vocab-parallel partial is completed by an all-reduce over the TP group, C2).
__global__ void embedding_kernel(const int* __restrict__ ids, const bf16* __restrict__ table, bf16* __restrict__ out,
                                 int H, int vocab_start, int vocab_end) {
  const int t = blockIdx.x;
  const int id = ids[t];
  PENNY_DASSERT(id >= 0);
  const bool mine = id >= vocab_start && id < vocab_end;
  const uint4* src = reinterpret_cast<const uint4*>(table + (long)(mine ? id - vocab_start : 0) * H);
  uint4* dst = reinterpret_cast<uint4*>(out + (long)t * H);
  for (int c = threadIdx.x; c < (H >> 3); c += blockDim.x) dst[c] = mine ? src[c] : make_uint4(0, 0, 0, 0);
}

static inline int grid_for(long work, int threads) {
  long g = (work + threads - 1) / threads;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

PENNY_API int penny_silu_mul(const void* gu, void* out, int T, int F, int interleave16, hipStream_t stream) {
  if (T <= 0) return 0;
  if (F % (interleave16 ? 16 : 8)) return (int)hipErrorInvalidValue;
  if (T > 65535) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(silu_mul_kernel, dim3((F / 8 + 255) / 256, T), dim3(256), 0, stream, (const bf16*)gu,
                     (bf16*)out, T, F, interleave16);
  PENNY_RETURN_LAUNCH();
}

PENNY_API int penny_gelu(void* x, long n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(n / 8, 256)), dim3(256), 0, stream, (bf16*)x, n / 8);
  PENNY_RETURN_LAUNCH();
}

PENNY_API int penny_embedding(const int* ids, const void* table, void* out, int T, int H, int vocab_start,
                              int vocab_end, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embedding_kernel, dim3(T), dim3(256), 0, stream, ids, (const bf16*)table, (bf16*)out, H,
                     vocab_start, vocab_end);
  PENNY_RETURN_LAUNCH();
}
