// K15: filtered exact top-k similarity search over an HBM-resident corpus (replaces Qdrant's
// filtered HNSW query, tools/qdrant_tool.py:98-153).
//
// Filters are the reference's: user_id == u (always) AND date >= t (optional).  Such filters are
// very selective (one user's rows out of ~1M), so the search is organised around the filter, not
// the vectors:
//   1. filter_compact: one pass over the int32 user codes + int64 dates (12 B/row, ~12 MB for
//      1M rows) evaluates every query's filter and appends matching row ids to a per-query
//      candidate list (wave-aggregated atomics).  Vectors of non-matching rows are never read.
//   2. score: one wave per candidate row computes <corpus_row, query> (768-d bf16, 16 B/lane).
//   3. select: one workgroup per query bitonic-sorts up to SORT_CAP (score, row) pairs in LDS,
//      descending by score, ties by row id, and writes the first k.
// Queries with more candidates than SORT_CAP are finished by the caller (torch.topk on the
// device-side score list), which the host detects from the returned counts.
#include "common.h"

#define SORT_CAP 8192

__global__ void filter_compact_kernel(const int* __restrict__ user_codes, const long long* __restrict__ dates, long N,
                                      const int* __restrict__ q_user, const long long* __restrict__ q_floor, int nq,
                                      int* __restrict__ counts, int* __restrict__ cand, int cap) {
  __shared__ int su[64];
  __shared__ long long sf[64];
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    su[i] = q_user[i];
    sf[i] = q_floor[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (long base = (long)blockIdx.x * blockDim.x; base < N; base += (long)gridDim.x * blockDim.x) {
    const long n = base + threadIdx.x;
    const bool in = n < N;
    const int code = in ? user_codes[n] : -2;
    const long long d = in ? dates[n] : 0;
    for (int qi = 0; qi < nq; ++qi) {
      const bool hit = in && code == su[qi] && d >= sf[qi];
      const unsigned long long mask = __ballot(hit);
      if (mask == 0ull) continue;
      int start = 0;
      if (lane == __ffsll((long long)mask) - 1) start = atomicAdd(&counts[qi], __popcll(mask));
      start = __shfl(start, __ffsll((long long)mask) - 1, 64);
      if (hit) {
        const int pos = start + __popcll(mask & ((1ull << lane) - 1ull));
        if (pos < cap) cand[(long)qi * cap + pos] = (int)n;
      }
    }
  }
}

// one wave per (query, candidate); D multiple of 8, D <= 1024
__global__ void score_kernel(const bf16* __restrict__ corpus, int D, const bf16* __restrict__ queries,
                             const int* __restrict__ counts, const int* __restrict__ cand, int cap,
                             float* __restrict__ scores) {
  const int qi = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int waves = (gridDim.x * blockDim.x) >> 6;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int cnt = min(counts[qi], cap);
  const int nch = D >> 3;
  float qv[2][8];
  for (int r = 0; r < 2; ++r) {
    const int c = lane + 64 * r;
    if (c < nch) unpack8(reinterpret_cast<const uint4*>(queries + (long)qi * D)[c], qv[r]);
  }
  for (int i = wid; i < cnt; i += waves) {
    const int row = cand[(long)qi * cap + i];
    const uint4* cr = reinterpret_cast<const uint4*>(corpus + (long)row * D);
    float acc = 0.f;
    for (int r = 0; r < 2; ++r) {
      const int c = lane + 64 * r;
      if (c < nch) {
        float f[8];
        unpack8(cr[c], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += f[k] * qv[r][k];
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) scores[(long)qi * cap + i] = acc;
  }
}

__device__ __forceinline__ bool before(float sa, int ia, float sb, int ib) {  // a ranks before b
  return sa > sb || (sa == sb && ia < ib);
}

__global__ void __launch_bounds__(1024) select_kernel(const int* __restrict__ counts, const int* __restrict__ cand,
                                                      const float* __restrict__ scores, int cap,
                                                      const int* __restrict__ ks, int kmax, int* __restrict__ out_ids,
                                                      float* __restrict__ out_scores, int* __restrict__ out_count) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  float* ss = reinterpret_cast<float*>(dyn);
  int* si = reinterpret_cast<int*>(dyn + SORT_CAP * sizeof(float));
  const int qi = blockIdx.x;
  const int total = counts[qi];
  const int cnt = min(total, cap);
  const int k = min(ks[qi], min(cnt, kmax));
  if (total > SORT_CAP) {  // host finishes this query
    if (threadIdx.x == 0) out_count[qi] = -total;
    return;
  }
  int n = 1;
  while (n < cnt) n <<= 1;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const bool v = i < cnt;
    ss[i] = v ? scores[(long)qi * cap + i] : -INFINITY;
    si[i] = v ? cand[(long)qi * cap + i] : 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;  // this run sorted "best first"
          const bool swap = desc ? before(ss[j], si[j], ss[i], si[i]) : before(ss[i], si[i], ss[j], si[j]);
          if (swap) {
            const float t = ss[i]; ss[i] = ss[j]; ss[j] = t;
            const int u = si[i]; si[i] = si[j]; si[j] = u;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    out_ids[(long)qi * kmax + i] = si[i];
    out_scores[(long)qi * kmax + i] = ss[i];
  }
  if (threadIdx.x == 0) out_count[qi] = k;
}

PENNY_API int penny_filtered_topk(const void* corpus, const int* user_codes, const long long* dates, long N, int D,
                                  const void* queries, const int* q_user, const long long* q_floor, const int* ks,
                                  int nq, int kmax, int* counts, int* cand, float* scores, int cap, int* out_ids,
                                  float* out_scores, int* out_count, hipStream_t stream) {
  if (nq <= 0) return 0;
  if (nq > 64 || D % 8 || D > 1024) return (int)hipErrorInvalidValue;
  hipMemsetAsync(counts, 0, sizeof(int) * nq, stream);
  long g = (N + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(filter_compact_kernel, dim3((int)g), dim3(256), 0, stream, user_codes, dates, N, q_user, q_floor,
                     nq, counts, cand, cap);
  hipLaunchKernelGGL(score_kernel, dim3(64, nq), dim3(256), 0, stream, (const bf16*)corpus, D, (const bf16*)queries,
                     counts, cand, cap, scores);
  const size_t lds = SORT_CAP * (sizeof(float) + sizeof(int));
  hipLaunchKernelGGL(select_kernel, dim3(nq), dim3(1024), lds, stream, counts, cand, scores, cap, ks, kmax, out_ids,
                     out_scores, out_count);
  PENNY_RETURN_LAUNCH();
}
