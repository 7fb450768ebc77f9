// K3 epilogue + K4 + K5: rotary embedding of q/k taken straight from the fused QKV GEMM output,
// and the paged KV-cache write, in ONE pass over the QKV activations.
//
// qkv      [T, (Hq + 2*Hkv) * D] bf16  (q heads, then k heads, then v heads)
// q_out    [T, Hq, D] bf16              (rotated q, consumed by the attention kernels)
// k_cache  [num_blocks][Hkv][64*D]       bf16, MFMA-fragment-native tiles (kv_layout.h k_index)
// v_cache  [num_blocks][Hkv][64*D]       bf16, MFMA-fragment-native tiles (kv_layout.h v_index)
//                                        -- a K row's 8 consecutive dims are one 16-B store; V is
//                                        scattered element-wise (transposed on write, so that every
//                                        attention-side read is a contiguous fragment).
// cos_sin  [max_pos, D] f32: cos(pos * inv_freq[i]) for i < D/2, then sin(...)  (host-precomputed,
//          so the kernel stays bandwidth-bound: no on-device trig, Appendix B 'Element-wise')
// Rotation is the HF/"neox" rotate-half form used by Llama-3 checkpoints.
#include "common.h"
#include "kv_layout.h"

// SLAB: the QKV activation arrives as the S f32 split-K slabs [S, T, width] of the QKV GEMM
// (gemm_splitk.hip) and is reduced here, in the same pass that rotates and scatters it.
// QK: no paged cache -- rotated q AND k heads go to q_out [T, Hq + Hkv, D] (k heads after the q
// heads), v is left in qkv: the context-parallel prefill, whose K/V travel the ring as tensors.
template <int D, bool SLAB, bool QK = false>
__global__ void rope_kv_kernel(const bf16* __restrict__ qkv, const int* __restrict__ positions,
                               const float* __restrict__ cos_sin, const int* __restrict__ slots,
                               bf16* __restrict__ q_out, bf16* __restrict__ k_cache, bf16* __restrict__ v_cache,
                               int Hq, int Hkv, int apply_rope, const float* __restrict__ P, int S, int T) {
  constexpr int HALF = D / 2;
  constexpr int RU = HALF / 8;  // rotary units per head (8 pairs each)
  constexpr int VU = D / 8;     // copy units per v head
  const int t = blockIdx.x;
  const int pos = positions[t];
  const int slot = QK ? -1 : slots[t];
  PENNY_DASSERT(pos >= 0 && slot >= -1);
  const int width = (Hq + 2 * Hkv) * D;
  const bf16* row = qkv + (long)t * width;
  const float* prow = SLAB ? P + (long)t * width : nullptr;
  auto load8 = [&](int c0, float* o) {  // 8 activations starting at column c0 of this token's row
    if constexpr (SLAB) load8_slabs(prow + c0, S, (long)T * width, o);
    else unpack8(*reinterpret_cast<const uint4*>(row + c0), o);
  };
  const float* cs = cos_sin + (long)pos * D;
  const int n_rot = (Hq + Hkv) * RU;
  const int total = n_rot + Hkv * VU;
  const long blk = slot >= 0 ? slot / KV_BS : 0;
  const int off = slot >= 0 ? slot % KV_BS : 0;
  // gridDim.y workgroups share a token's units (decode-size T: T workgroups alone would leave
  // half the CUs idle while the split-K slabs are read)
  for (int u = threadIdx.x + blockIdx.y * blockDim.x; u < total; u += blockDim.x * gridDim.y) {
    if (u < n_rot) {
      const int h = u / RU, c = u % RU;
      float x1[8], x2[8];
      load8(h * D + c * 8, x1);
      load8(h * D + HALF + c * 8, x2);
      if (apply_rope) {
        float co[8], si[8];   // 4 x 16-B loads instead of 16 scalar loads
        *reinterpret_cast<float4*>(co) = *reinterpret_cast<const float4*>(cs + c * 8);
        *reinterpret_cast<float4*>(co + 4) = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
        *reinterpret_cast<float4*>(si) = *reinterpret_cast<const float4*>(cs + HALF + c * 8);
        *reinterpret_cast<float4*>(si + 4) = *reinterpret_cast<const float4*>(cs + HALF + c * 8 + 4);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float a = x1[i], b = x2[i];
          x1[i] = a * co[i] - b * si[i];
          x2[i] = b * co[i] + a * si[i];
        }
      }
      const uint4 p1 = pack8(x1), p2 = pack8(x2);
      if (QK) {
        bf16* dst = q_out + ((long)t * (Hq + Hkv) + h) * D;
        *reinterpret_cast<uint4*>(dst + c * 8) = p1;
        *reinterpret_cast<uint4*>(dst + HALF + c * 8) = p2;
      } else if (h < Hq) {
        bf16* dst = q_out + ((long)t * Hq + h) * D;
        *reinterpret_cast<uint4*>(dst + c * 8) = p1;
        *reinterpret_cast<uint4*>(dst + HALF + c * 8) = p2;
      } else if (slot >= 0) {
        const int kh = h - Hq;
        bf16* dst = k_cache + (blk * Hkv + kh) * (long)(KV_BS * D);
        *reinterpret_cast<uint4*>(dst + k_index(off, c * 8, D)) = p1;
        *reinterpret_cast<uint4*>(dst + k_index(off, HALF + c * 8, D)) = p2;
      }
    } else if (!QK && slot >= 0) {
      const int v = u - n_rot;
      const int h = v / VU, c = v % VU;
      float x[8];
      load8((Hq + Hkv + h) * D + c * 8, x);
      bf16* base = v_cache + (blk * Hkv + h) * (long)(KV_BS * D);
#pragma unroll
      for (int i = 0; i < 8; ++i) base[v_index(off, c * 8 + i, D)] = (bf16)x[i];
    }
  }
}

template <bool SLAB>
static int launch_rope_kv(const void* qkv, const float* P, int S, const int* positions, const float* cos_sin,
                          const int* slots, void* q_out, void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D,
                          int apply_rope, hipStream_t stream) {
  if (T <= 0) return 0;
  const int threads = 256;
  const dim3 grid(T, T <= 512 ? 2 : 1);
  if (D == 128) {
    hipLaunchKernelGGL((rope_kv_kernel<128, SLAB>), grid, dim3(threads), 0, stream, (const bf16*)qkv, positions,
                       cos_sin, slots, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, Hq, Hkv, apply_rope, P, S, T);
  } else if (D == 64) {
    hipLaunchKernelGGL((rope_kv_kernel<64, SLAB>), grid, dim3(threads), 0, stream, (const bf16*)qkv, positions,
                       cos_sin, slots, (bf16*)q_out, (bf16*)k_cache, (bf16*)v_cache, Hq, Hkv, apply_rope, P, S, T);
  } else {
    return (int)hipErrorInvalidValue;
  }
  PENNY_RETURN_LAUNCH();
}

PENNY_API int penny_rope_kv_write(const void* qkv, const int* positions, const float* cos_sin, const int* slots,
                                  void* q_out, void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D,
                                  int apply_rope, hipStream_t stream) {
  return launch_rope_kv<false>(qkv, nullptr, 0, positions, cos_sin, slots, q_out, k_cache, v_cache, T, Hq, Hkv, D,
                               apply_rope, stream);
}

// qkv given as the S split-K slabs P [S, T, (Hq + 2*Hkv) * D] f32 of the QKV GEMM
PENNY_API int penny_rope_kv_write_slabs(const void* P, int S, const int* positions, const float* cos_sin,
                                        const int* slots, void* q_out, void* k_cache, void* v_cache, int T, int Hq,
                                        int Hkv, int D, int apply_rope, hipStream_t stream) {
  if (S < 1) return (int)hipErrorInvalidValue;
  return launch_rope_kv<true>(nullptr, (const float*)P, S, positions, cos_sin, slots, q_out, k_cache, v_cache, T, Hq,
                              Hkv, D, apply_rope, stream);
}

// Context-parallel form: rotated q and k heads of qkv [T, (Hq + 2*Hkv) * D] -> qk [T, Hq + Hkv, D]
// (no KV-cache write; v stays in qkv).  positions [T] are the zig-zag shard's global positions.
PENNY_API int penny_rope_qk(const void* qkv, const int* positions, const float* cos_sin, void* qk, int T, int Hq,
                            int Hkv, int D, hipStream_t stream) {
  if (T <= 0) return 0;
  const dim3 grid(T, T <= 512 ? 2 : 1);
  if (D == 128) {
    hipLaunchKernelGGL((rope_kv_kernel<128, false, true>), grid, dim3(256), 0, stream, (const bf16*)qkv, positions,
                       cos_sin, (const int*)nullptr, (bf16*)qk, (bf16*)nullptr, (bf16*)nullptr, Hq, Hkv, 1,
                       (const float*)nullptr, 0, T);
  } else if (D == 64) {
    hipLaunchKernelGGL((rope_kv_kernel<64, false, true>), grid, dim3(256), 0, stream, (const bf16*)qkv, positions,
                       cos_sin, (const int*)nullptr, (bf16*)qk, (bf16*)nullptr, (bf16*)nullptr, Hq, Hkv, 1,
                       (const float*)nullptr, 0, T);
  } else {
    return (int)hipErrorInvalidValue;
  }
  PENNY_RETURN_LAUNCH();
}
