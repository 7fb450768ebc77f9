// C1 (custom path): one-shot / two-shot all-reduce over xGMI peer-to-peer for decode-size TP messages.
//
// RCCL's ring all-reduce moves a message through n-1 sequential hops, each bound by ONE xGMI link
// (~153 GB/s) and each paying a hop latency; a decode step's all-reduce is only a few hundred KB,
// so it is latency-bound.  One-shot instead: every rank copies its input into its own registered
// (IPC-shared) buffer, raises a flag in every peer's signal area, waits for all peers' flags, then
// reads the n buffers CONCURRENTLY over its n-1 direct links and sums them locally.  One
// publish/wait round trip, all 7 links busy at once.
//
// Protocol per launch ("round" r = *counter + 1, bumped by ar_bump_kernel after the launch, so a
// hipGraph replay advances it on the device without host involvement):
//   * data buffers are double-buffered by round parity: round r+1 writes the other half, and a
//     rank can only reach round r+2 (same half again) after every peer has signalled r+1, i.e.
//     after every peer finished READING round r;
//   * flags are monotone round numbers (no reset), one slot per (source rank, block), so each
//     block synchronises only its own chunk;
//   * writer: all threads drain their stores with a system-scope fence, barrier, then one lane
//     per peer stores the flag with system-scope release; reader: one lane per peer polls with
//     system-scope acquire, barrier, system-scope acquire fence, then reads;
//   * buffers are allocated uncached (hipDeviceMallocUncached): remote reads never hit a stale
//     L2 line of an earlier round;
//   * every wait is bounded (wall clock, 5 s).  A rank whose wait expires FAILS the collective
//     instead of summing whatever the peer buffers hold: it sets *err, POISONS its flag slots in
//     every peer's signal area (a negative value, which every later poll of that slot sees at no
//     extra cost: the poll already loads it), and writes NaN into its output.  A rank that polls a
//     poisoned slot fails the same way, and a rank whose *err is set fails at its next launch
//     without publishing -- so one stalled peer turns every rank's collectives into NaN + err
//     within one round, the host sees err with the step's sampled ids (model_runner.PendingStep)
//     and the TP group falls back to RCCL together (parallel/comm.py).  A dead rank can never
//     wedge the GPU and never yields a silently wrong sum.
#include <string.h>

#include "common.h"

#define AR_MAX_RANKS 8
#define AR_MAX_BLOCKS 64
#define AR_TIMEOUT_TICKS (5ull * 100000000ull)  // wall_clock64() runs at 100 MHz
#define AR_POISON (-1)

struct ArPeers {
  bf16* data[AR_MAX_RANKS];  // each rank's registered data buffer (2 halves of half_elems)
  int* sig[AR_MAX_RANKS];    // each rank's signal area: [2 region][AR_MAX_RANKS source][AR_MAX_BLOCKS]
};

// publish `round` for (region, this rank, this block) in every peer's signal area, after every
// thread's stores are complete at system scope
__device__ __forceinline__ void ar_publish(const ArPeers& peers, int region, int rank, int nranks, int round) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < nranks)
    __hip_atomic_store(peers.sig[threadIdx.x] + (region * AR_MAX_RANKS + rank) * AR_MAX_BLOCKS + blockIdx.x, round,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// this rank failed: every slot it publishes into, in every peer, reads AR_POISON from now on
__device__ __forceinline__ void ar_poison(const ArPeers& peers, int rank, int nranks) {
  for (int i = threadIdx.x; i < nranks * 2 * AR_MAX_BLOCKS; i += blockDim.x) {
    const int q = i / (2 * AR_MAX_BLOCKS), region = (i / AR_MAX_BLOCKS) & 1, b = i % AR_MAX_BLOCKS;
    if (q != rank)
      __hip_atomic_store(peers.sig[q] + (region * AR_MAX_RANKS + rank) * AR_MAX_BLOCKS + b, AR_POISON,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
}

// wait (bounded) until every peer published `round` for (region, this block), then acquire.
// Returns false (block-uniform) when a peer is late past the bound or has poisoned its slot; the
// caller then fails the collective (ar_fail) instead of reading the peer buffers.
__device__ __forceinline__ bool ar_wait(const ArPeers& peers, int region, int rank, int nranks, int round,
                                        int* err, int* s_fail) {
  if (threadIdx.x == 0) *s_fail = 0;
  __syncthreads();
  if (threadIdx.x < nranks) {
    const int* slot = peers.sig[rank] + (region * AR_MAX_RANKS + threadIdx.x) * AR_MAX_BLOCKS + blockIdx.x;
    const unsigned long long t0 = wall_clock64();
    while (true) {
      const int v = __hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v < 0 || wall_clock64() - t0 > AR_TIMEOUT_TICKS) {
        *s_fail = 1;
        break;
      }
      if (v >= round) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (*s_fail) {
    if (threadIdx.x == 0) atomicExch(err, 1);
    ar_poison(peers, rank, nranks);
    return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
  return true;
}

// NaN over out[base + q * stride + [lo, hi)) for q < reps: a failed collective's output
__device__ __forceinline__ void ar_fill_nan(bf16* out, long base, long stride, int reps, long lo, long hi) {
  const uint4 nan8 = make_uint4(0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u);
  for (int q = 0; q < reps; ++q)
    for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
      *reinterpret_cast<uint4*>(out + base + q * stride + i) = nan8;
}

// out[i..i+7] (or any bf16 destination) <- sum over ranks q = 0..n-1 of peers.data[q][src + i], f32,
// in fixed rank order on every rank -> bit-identical results across the group and across the
// one-shot / two-shot forms
__device__ __forceinline__ uint4 ar_sum8(const ArPeers& peers, int nranks, long src) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int q = 0; q < nranks; ++q) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(peers.data[q] + src), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  return pack8(acc);
}

__global__ void __launch_bounds__(256) ar_oneshot_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                         long n, ArPeers peers, const int* __restrict__ counter,
                                                         int* __restrict__ err, int rank, int nranks,
                                                         long half_elems) {
  __shared__ int s_fail;
  const int round = *counter + 1;
  const int dead = *err;                         // loaded beside the counter: no extra latency
  const long off = (round & 1) * half_elems;
  const long per = ((n + gridDim.x - 1) / gridDim.x + 7) / 8 * 8;
  const long lo = blockIdx.x * per, hi = min(n, lo + per);
  if (dead) {                                    // failed earlier: never publish again
    ar_fill_nan(out, 0, 0, 1, lo, hi);
    return;
  }
  bf16* mine = peers.data[rank] + off;
  for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
    *reinterpret_cast<uint4*>(mine + i) = *reinterpret_cast<const uint4*>(in + i);
  ar_publish(peers, 0, rank, nranks, round);
  if (!ar_wait(peers, 0, rank, nranks, round, err, &s_fail)) {
    ar_fill_nan(out, 0, 0, 1, lo, hi);
    return;
  }
  for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
    *reinterpret_cast<uint4*>(out + i) = ar_sum8(peers, nranks, off + i);
}

// Two-shot (reduce-scatter, then all-gather) for mid-size messages on > 2 ranks.  One-shot has
// every rank read the WHOLE message from every peer ((n-1) x bytes over its links); here rank r
// reduces only chunk r (1/n of the message from each peer), publishes the reduced chunk in its
// own buffer, and then every rank gathers the n reduced chunks: 2(n-1)/n x bytes per rank, for
// one more flag round trip.  Block b owns sub-slice b of every chunk in all three phases, so its
// flags cover exactly the bytes it reads.  Chunk r of rank r's buffer is read and rewritten only
// by rank r in the reduce phase, so the reduced chunk can overwrite its input in place.
__global__ void __launch_bounds__(256) ar_twoshot_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                         long n, ArPeers peers, const int* __restrict__ counter,
                                                         int* __restrict__ err, int rank, int nranks,
                                                         long half_elems) {
  __shared__ int s_fail;
  const int round = *counter + 1;
  const int dead = *err;
  const long off = (round & 1) * half_elems;
  const long chunk = n / nranks;
  const long per = ((chunk + gridDim.x - 1) / gridDim.x + 7) / 8 * 8;
  const long lo = blockIdx.x * per, hi = min(chunk, lo + per);
  if (dead) {
    ar_fill_nan(out, 0, chunk, nranks, lo, hi);
    return;
  }
  bf16* mine = peers.data[rank] + off;
  for (int q = 0; q < nranks; ++q)
    for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
      *reinterpret_cast<uint4*>(mine + q * chunk + i) = *reinterpret_cast<const uint4*>(in + q * chunk + i);
  ar_publish(peers, 0, rank, nranks, round);
  if (!ar_wait(peers, 0, rank, nranks, round, err, &s_fail)) {
    ar_fill_nan(out, 0, chunk, nranks, lo, hi);
    return;
  }
  const long base = (long)rank * chunk;
  for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
    *reinterpret_cast<uint4*>(mine + base + i) = ar_sum8(peers, nranks, off + base + i);
  ar_publish(peers, 1, rank, nranks, round);
  if (!ar_wait(peers, 1, rank, nranks, round, err, &s_fail)) {
    ar_fill_nan(out, 0, chunk, nranks, lo, hi);
    return;
  }
  for (int q = 0; q < nranks; ++q)
    for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
      *reinterpret_cast<uint4*>(out + q * chunk + i) =
          *reinterpret_cast<const uint4*>(peers.data[q] + off + q * chunk + i);
}

// All-gather (C2: vocab-parallel LM-head logits) on the same buffers, flags and round counter:
// copy-in, publish, wait, then read every peer's n elements over the direct links into
// out[q * n ...] (rank-major; the caller permutes to [B, V]).  One flag round trip.
__global__ void __launch_bounds__(256) ag_kernel(const bf16* __restrict__ in, bf16* __restrict__ out, long n,
                                                 ArPeers peers, const int* __restrict__ counter,
                                                 int* __restrict__ err, int rank, int nranks, long half_elems) {
  __shared__ int s_fail;
  const int round = *counter + 1;
  const int dead = *err;
  const long off = (round & 1) * half_elems;
  const long per = ((n + gridDim.x - 1) / gridDim.x + 7) / 8 * 8;
  const long lo = blockIdx.x * per, hi = min(n, lo + per);
  if (dead) {
    ar_fill_nan(out, 0, n, nranks, lo, hi);
    return;
  }
  bf16* mine = peers.data[rank] + off;
  for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
    *reinterpret_cast<uint4*>(mine + i) = *reinterpret_cast<const uint4*>(in + i);
  ar_publish(peers, 0, rank, nranks, round);
  if (!ar_wait(peers, 0, rank, nranks, round, err, &s_fail)) {
    ar_fill_nan(out, 0, n, nranks, lo, hi);
    return;
  }
  for (int q = 0; q < nranks; ++q)
    for (long i = lo + threadIdx.x * 8; i < hi; i += 256 * 8)
      *reinterpret_cast<uint4*>(out + q * n + i) = *reinterpret_cast<const uint4*>(peers.data[q] + off + i);
}

__global__ void ar_bump_kernel(int* counter) { *counter += 1; }

PENNY_API int penny_ar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Uncached device allocation + its IPC handle (written to `handle`, penny_ar_handle_size() bytes).
PENNY_API int penny_ar_alloc(size_t bytes, void** out_ptr, void* handle) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, bytes);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  memcpy(handle, &h, sizeof(h));
  *out_ptr = p;
  return 0;
}

PENNY_API int penny_ar_open(const void* handle, void** out_ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out_ptr, h, hipIpcMemLazyEnablePeerAccess);
}

PENNY_API int penny_ar_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

PENNY_API int penny_ar_free(void* p) { return (int)hipFree(p); }

static int ar_launch(bool twoshot, const void* in, void* out, long n, void* const* data_ptrs, void* const* sig_ptrs,
                     int* counter, int* err, int rank, int nranks, long half_elems, int nblocks, hipStream_t stream) {
  if (n <= 0) return 0;
  if (nranks < 1 || nranks > AR_MAX_RANKS || rank < 0 || rank >= nranks || n % 8 || n > half_elems ||
      nblocks < 1 || nblocks > AR_MAX_BLOCKS || (twoshot && n % (8L * nranks)))
    return (int)hipErrorInvalidValue;
  ArPeers peers;
  for (int q = 0; q < AR_MAX_RANKS; ++q) {
    peers.data[q] = q < nranks ? (bf16*)data_ptrs[q] : nullptr;
    peers.sig[q] = q < nranks ? (int*)sig_ptrs[q] : nullptr;
  }
  if (twoshot)
    hipLaunchKernelGGL(ar_twoshot_kernel, dim3(nblocks), dim3(256), 0, stream, (const bf16*)in, (bf16*)out, n, peers,
                       (const int*)counter, err, rank, nranks, half_elems);
  else
    hipLaunchKernelGGL(ar_oneshot_kernel, dim3(nblocks), dim3(256), 0, stream, (const bf16*)in, (bf16*)out, n, peers,
                       (const int*)counter, err, rank, nranks, half_elems);
  hipLaunchKernelGGL(ar_bump_kernel, dim3(1), dim3(1), 0, stream, counter);
  PENNY_RETURN_LAUNCH();
}

// out: [nranks * n] rank-major; n % 8 == 0, n <= half_elems
PENNY_API int penny_allgather(const void* in, void* out, long n, void* const* data_ptrs, void* const* sig_ptrs,
                              int* counter, int* err, int rank, int nranks, long half_elems, int nblocks,
                              hipStream_t stream) {
  if (n <= 0) return 0;
  if (nranks < 1 || nranks > AR_MAX_RANKS || rank < 0 || rank >= nranks || n % 8 || n > half_elems ||
      nblocks < 1 || nblocks > AR_MAX_BLOCKS)
    return (int)hipErrorInvalidValue;
  ArPeers peers;
  for (int q = 0; q < AR_MAX_RANKS; ++q) {
    peers.data[q] = q < nranks ? (bf16*)data_ptrs[q] : nullptr;
    peers.sig[q] = q < nranks ? (int*)sig_ptrs[q] : nullptr;
  }
  hipLaunchKernelGGL(ag_kernel, dim3(nblocks), dim3(256), 0, stream, (const bf16*)in, (bf16*)out, n, peers,
                     (const int*)counter, err, rank, nranks, half_elems);
  hipLaunchKernelGGL(ar_bump_kernel, dim3(1), dim3(1), 0, stream, counter);
  PENNY_RETURN_LAUNCH();
}

// data_ptrs / sig_ptrs: host arrays of nranks device pointers (own buffers + opened peer buffers).
// The signal area of each rank is [2 regions][AR_MAX_RANKS source][AR_MAX_BLOCKS] ints.
PENNY_API int penny_allreduce_oneshot(const void* in, void* out, long n, void* const* data_ptrs,
                                      void* const* sig_ptrs, int* counter, int* err, int rank, int nranks,
                                      long half_elems, int nblocks, hipStream_t stream) {
  return ar_launch(false, in, out, n, data_ptrs, sig_ptrs, counter, err, rank, nranks, half_elems, nblocks, stream);
}

// n % (8 * nranks) == 0; nblocks splits each rank's chunk
PENNY_API int penny_allreduce_twoshot(const void* in, void* out, long n, void* const* data_ptrs,
                                      void* const* sig_ptrs, int* counter, int* err, int rank, int nranks,
                                      long half_elems, int nblocks, hipStream_t stream) {
  return ar_launch(true, in, out, n, data_ptrs, sig_ptrs, counter, err, rank, nranks, half_elems, nblocks, stream);
}
