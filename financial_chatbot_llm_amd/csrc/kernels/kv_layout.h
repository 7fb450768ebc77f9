// Paged KV-cache layout shared by the KV writer (rope_kv.hip) and the attention kernels.
//
// A block holds KV_BS = 64 tokens of one kv head = exactly one 64-key attention tile, and is
// stored in **MFMA-fragment-native order**: the 16-byte operand fragment that lane l of a wave
// feeds to v_mfma_f32_16x16x32_bf16 for fragment f lives at byte 16*(64*f + l).  Hence
//   * decode streams a block with perfectly coalesced 1-KiB wave-instructions straight into
//     VGPRs (no LDS hop, no over-fetch), and
//   * prefill stages a block into LDS with lane-linear global_load_lds (no swizzle needed) and
//     reads fragments back with conflict-free consecutive ds_read_b128.
//
// K (A operand of S^T = K.Q^T): fragment f = t*(D/32) + c for key tile t (16 keys) and k-chunk c
//   (32 dims); lane = 16*g + r holds key 16t+r, dims 32c + 8g + 0..7.
// V (A operand of O^T = V^T.P^T): fragment f = 2*dt + s for dim tile dt (16 dims) and key step s
//   (32 keys); lane = 16*g + row holds dim 16dt+row and the 8 keys whose scores lane group g
//   already holds in registers after the S^T MFMA: 32s + 4g + 0..3 and 32s + 16 + 4g + 0..3.
#pragma once

#define KV_BS 64

// element index inside one (block, kv head) tile of K
__host__ __device__ __forceinline__ int k_index(int key, int d, int D) {
  const int t = key >> 4, r = key & 15, c = d >> 5, g = (d >> 3) & 3, j = d & 7;
  return (((t * (D >> 5) + c) * 64 + g * 16 + r) << 3) + j;
}

// element index inside one (block, kv head) tile of V
__host__ __device__ __forceinline__ int v_index(int key, int d, int D) {
  const int dt = d >> 4, row = d & 15, s = key >> 5, k = key & 31;
  const int g = (k & 15) >> 2, j = ((k >> 4) << 2) + (k & 3);
  return (((dt * 2 + s) * 64 + g * 16 + row) << 3) + j;
}
