// Paged KV-cache layout shared by the KV writer (rope_kv.hip) and the attention kernels.
//
// A block holds KV_BS = 64 tokens = exactly one 64-key attention tile.
//   K: [block][kv_head][64 keys][D]      key-major
//   V: [block][kv_head][D][64 keys]      dim-major, keys permuted inside each 32-key group
//
// Why the permutation: S^T = K.Q^T on v_mfma_f32_16x16x32_bf16 leaves lane l holding, for query
// column l&15, the scores of keys 16t + 4g + r (g = l>>4, r = 0..3) of each 16-key tile t.  The
// P.V product O^T = V^T.P^T consumes P straight from those registers if, for k-step s, lane
// group g's 8 K-elements are keys {32s+4g+0..3} (tile 2s) and {32s+16+4g+0..3} (tile 2s+1).
// Storing key k of a 32-key group at  8*((k&15)>>2) + 4*(k>>4) + (k&3)  makes those 8 keys
// physically contiguous, so each V^T A-fragment is a single 16-byte load.
#pragma once

#define KV_BS 64

__host__ __device__ __forceinline__ int kv_perm(int key) {
  const int grp = key >> 5, k = key & 31;
  return grp * 32 + 8 * ((k & 15) >> 2) + 4 * (k >> 4) + (k & 3);
}
