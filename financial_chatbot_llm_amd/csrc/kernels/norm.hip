// K2 / K14: fused residual-add + RMSNorm (Llama) and residual-add + LayerNorm (BERT).
//
// One workgroup per token row; each lane owns CPT 16-byte chunks (8 bf16) of the row, kept
// in registers between the statistics pass and the normalise pass, so a row is read once and
// written once (HBM-bound op: 2-3 row passes total vs 5+ for an unfused torch sequence).
//
//   rms:      y = bf16(x * rsqrt(mean(x^2) + eps) * w)
//   add_rms:  r = bf16(x + res); res <- r; y = rms(r)          (in-place residual update)
//   ln:       y = bf16((x - mu) * rsqrt(var + eps) * g + b)
//   add_ln:   r = x + res (f32); y = ln(r)                     (BERT post-LN: LN(x + sublayer(x)))
#include "common.h"

// SLAB: x is not a bf16 tensor but the S f32 split-K slabs [S, T, H] of the producing GEMM
// (gemm_splitk.hip); summing them here IS that GEMM's reduction, fused into the norm's row pass
// (one workgroup per row keeps >= T workgroups in flight for the extra slab reads).
template <int CPT, bool ADD_RES, bool SLAB>
__global__ void __launch_bounds__(1024) rmsnorm_kernel(const bf16* __restrict__ x, bf16* __restrict__ res,
                                                       const bf16* __restrict__ w, bf16* __restrict__ y,
                                                       int H, float eps, const float* __restrict__ P, int S,
                                                       int T) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  uint4* rr = reinterpret_cast<uint4*>(res + (size_t)row * H);
  float v[CPT][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = threadIdx.x + c * blockDim.x;
    if (idx < nchunk) {
      if (SLAB) load8_slabs(P + (size_t)row * H + 8 * idx, S, (long)T * H, v[c]);
      else unpack8(xr[idx], v[c]);
      if (ADD_RES) {
        float r[8];
        unpack8(rr[idx], r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = (float)(bf16)(v[c][i] + r[i]);  // residual kept in bf16
        rr[idx] = pack8(v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  const float inv = rsqrtf(block_sum(ss, scratch) / (float)H + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * H);
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = threadIdx.x + c * blockDim.x;
    if (idx < nchunk) {
      float g[8], o[8];
      unpack8(wr[idx], g);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)(v[c][i] * inv) * g[i];
      yr[idx] = pack8(o);
    }
  }
}


// One wave64 per row (rows of H = 512*CPW elements): every lane holds CPW 16-byte chunks, the
// weight is fetched together with x/residual (one memory round trip instead of three), and the
// sum of squares is a pure register/DPP reduction -- no LDS, no barrier.  Decode-size batches
// (T = 1..256 rows) are latency-bound, so this is what keeps a B=128 norm at a few us.
template <int CPW, bool ADD_RES>
__global__ void __launch_bounds__(256) rmsnorm_wave_kernel(const bf16* __restrict__ x, bf16* __restrict__ res,
                                                           const bf16* __restrict__ w, bf16* __restrict__ y,
                                                           int T, int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  uint4* rr = reinterpret_cast<uint4*>(res + (size_t)row * H);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  uint4 xv[CPW], rv[CPW], wv[CPW];
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    xv[c] = xr[lane + 64 * c];
    if (ADD_RES) rv[c] = rr[lane + 64 * c];
    wv[c] = wr[lane + 64 * c];
  }
  float v[CPW][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    unpack8(xv[c], v[c]);
    if (ADD_RES) {
      float r[8];
      unpack8(rv[c], r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = (float)(bf16)(v[c][i] + r[i]);  // residual kept in bf16
      rr[lane + 64 * c] = pack8(v[c]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
  }
  const float inv = rsqrtf(wave_sum(ss) / (float)H + eps);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * H);
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    float g[8], o[8];
    unpack8(wv[c], g);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)(bf16)(v[c][i] * inv) * g[i];
    yr[lane + 64 * c] = pack8(o);
  }
}

template <int CPT, bool ADD_RES>
__global__ void __launch_bounds__(1024) layernorm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                         const bf16* __restrict__ g, const bf16* __restrict__ b,
                                                         bf16* __restrict__ y, int H, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * H);
  const uint4* rr = reinterpret_cast<const uint4*>(res + (size_t)row * H);
  float v[CPT][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = threadIdx.x + c * blockDim.x;
    if (idx < nchunk) {
      unpack8(xr[idx], v[c]);
      if (ADD_RES) {
        float r[8];
        unpack8(rr[idx], r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] += r[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  const float mu = block_sum(s, scratch) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = threadIdx.x + c * blockDim.x;
    if (idx < nchunk) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        sq += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum(sq, scratch) / (float)H + eps);
  const uint4* gr = reinterpret_cast<const uint4*>(g);
  const uint4* br = reinterpret_cast<const uint4*>(b);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * H);
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int idx = threadIdx.x + c * blockDim.x;
    if (idx < nchunk) {
      float gg[8], bb[8], o[8];
      unpack8(gr[idx], gg);
      unpack8(br[idx], bb);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * inv * gg[i] + bb[i];
      yr[idx] = pack8(o);
    }
  }
}

// One WAVE per row for the encoder's H = 768 (bge-base) and other H % 256 == 0 up to 4096: each
// lane holds H/64 values as C4 8-byte chunks (4 bf16, at chunk lane + 64c), two wave reductions
// (mean, variance) and no LDS or block barrier.  The block-per-row kernel above spends most of
// a 128-thread block on two __syncthreads reductions at this width.
template <int C4, bool ADD_RES>
__global__ void __launch_bounds__(256) layernorm_wave_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                             const bf16* __restrict__ g, const bf16* __restrict__ b,
                                                             bf16* __restrict__ y, int T, int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const bf16x4* xr = reinterpret_cast<const bf16x4*>(x + (size_t)row * H);
  const bf16x4* rr = reinterpret_cast<const bf16x4*>(res + (size_t)row * H);
  bf16x4 xv[C4], rv[C4];
#pragma unroll
  for (int c = 0; c < C4; ++c) {
    xv[c] = xr[lane + 64 * c];
    if (ADD_RES) rv[c] = rr[lane + 64 * c];
  }
  float v[C4][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[c][i] = (float)xv[c][i] + (ADD_RES ? (float)rv[c][i] : 0.f);
      s += v[c][i];
    }
  const float mu = wave_sum(s) / (float)H;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < C4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = v[c][i] - mu;
      sq += d * d;
    }
  const float inv = rsqrtf(wave_sum(sq) / (float)H + eps);
  const bf16x4* gr = reinterpret_cast<const bf16x4*>(g);
  const bf16x4* br = reinterpret_cast<const bf16x4*>(b);
  bf16x4* yr = reinterpret_cast<bf16x4*>(y + (size_t)row * H);
#pragma unroll
  for (int c = 0; c < C4; ++c) {
    const bf16x4 gg = gr[lane + 64 * c], bb = br[lane + 64 * c];
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (bf16)((v[c][i] - mu) * inv * (float)gg[i] + (float)bb[i]);
    yr[lane + 64 * c] = o;
  }
}

static inline void pick_geometry(int H, int* threads, int* cpt) {
  const int nchunk = H / 8;
  int t = nchunk >= 256 ? 256 : ((nchunk + 63) / 64) * 64;
  int c = (nchunk + t - 1) / t;
  while (c > 8) {
    t *= 2;
    c = (nchunk + t - 1) / t;
  }
  int p = 1;
  while (p < c) p <<= 1;
  *threads = t;
  *cpt = p;
}

#define DISPATCH_CPT(CPT_VAL, ...)             \
  switch (CPT_VAL) {                           \
    case 1: { constexpr int CPT = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int CPT = 2; __VA_ARGS__; break; } \
    case 4: { constexpr int CPT = 4; __VA_ARGS__; break; } \
    default: { constexpr int CPT = 8; __VA_ARGS__; break; } \
  }

PENNY_API int penny_rmsnorm(const void* x, void* res, const void* w, void* y, int T, int H, float eps,
                            int add_residual, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  if (H % 512 == 0 && H <= 4096 && T <= 4096) {   // wave-per-row path (decode + short prefill)
    const int cpw = H / 512;
    dim3 grid((T + 3) / 4);
#define WAVE_NORM(CPW_)                                                                                        \
  if (cpw == CPW_) {                                                                                           \
    if (add_residual)                                                                                          \
      hipLaunchKernelGGL((rmsnorm_wave_kernel<CPW_, true>), grid, dim3(256), 0, stream, (const bf16*)x,        \
                         (bf16*)res, (const bf16*)w, (bf16*)y, T, H, eps);                                     \
    else                                                                                                       \
      hipLaunchKernelGGL((rmsnorm_wave_kernel<CPW_, false>), grid, dim3(256), 0, stream, (const bf16*)x,       \
                         (bf16*)res, (const bf16*)w, (bf16*)y, T, H, eps);                                     \
    PENNY_RETURN_LAUNCH();                                                                                     \
  }
    WAVE_NORM(1) WAVE_NORM(2) WAVE_NORM(4) WAVE_NORM(8)
#undef WAVE_NORM
  }
  int threads, cpt;
  pick_geometry(H, &threads, &cpt);
  if (add_residual) {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((rmsnorm_kernel<CPT, true, false>), dim3(T), dim3(threads), 0, stream,
                                         (const bf16*)x, (bf16*)res, (const bf16*)w, (bf16*)y, H, eps, nullptr, 0, T));
  } else {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((rmsnorm_kernel<CPT, false, false>), dim3(T), dim3(threads), 0, stream,
                                         (const bf16*)x, (bf16*)res, (const bf16*)w, (bf16*)y, H, eps, nullptr, 0, T));
  }
  PENNY_RETURN_LAUNCH();
}

// x given as the S split-K slabs P [S, T, H] f32 of the producing GEMM (see rmsnorm_kernel SLAB)
PENNY_API int penny_rmsnorm_slabs(const void* P, int S, void* res, const void* w, void* y, int T, int H, float eps,
                                  int add_residual, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8 || S < 1) return (int)hipErrorInvalidValue;
  int threads, cpt;
  pick_geometry(H, &threads, &cpt);
  if (T <= 512 && H / 8 <= 1024 && (H / 8) % 64 == 0) {
    // decode-size T: one 16-B chunk (x S slabs) per thread -- twice the waves per row, so the
    // S-deep slab reads of a T-row batch (T workgroups) have more latency hiding
    threads = H / 8;
    cpt = 1;
  }
  if (add_residual) {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((rmsnorm_kernel<CPT, true, true>), dim3(T), dim3(threads), 0, stream,
                                         nullptr, (bf16*)res, (const bf16*)w, (bf16*)y, H, eps, (const float*)P, S, T));
  } else {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((rmsnorm_kernel<CPT, false, true>), dim3(T), dim3(threads), 0, stream,
                                         nullptr, (bf16*)res, (const bf16*)w, (bf16*)y, H, eps, (const float*)P, S, T));
  }
  PENNY_RETURN_LAUNCH();
}

PENNY_API int penny_layernorm(const void* x, const void* res, const void* g, const void* b, void* y, int T, int H,
                              float eps, int add_residual, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  if (H % 256 == 0 && H <= 4096) {
    const dim3 grid((T + 3) / 4);
#define WAVE_LN(C4_)                                                                                           \
  if (H == 256 * C4_) {                                                                                        \
    if (add_residual)                                                                                          \
      hipLaunchKernelGGL((layernorm_wave_kernel<C4_, true>), grid, dim3(256), 0, stream, (const bf16*)x,       \
                         (const bf16*)res, (const bf16*)g, (const bf16*)b, (bf16*)y, T, H, eps);               \
    else                                                                                                       \
      hipLaunchKernelGGL((layernorm_wave_kernel<C4_, false>), grid, dim3(256), 0, stream, (const bf16*)x,      \
                         (const bf16*)res, (const bf16*)g, (const bf16*)b, (bf16*)y, T, H, eps);               \
    PENNY_RETURN_LAUNCH();                                                                                     \
  }
    WAVE_LN(1) WAVE_LN(2) WAVE_LN(3) WAVE_LN(4) WAVE_LN(8) WAVE_LN(16)
#undef WAVE_LN
  }
  int threads, cpt;
  pick_geometry(H, &threads, &cpt);
  if (add_residual) {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((layernorm_kernel<CPT, true>), dim3(T), dim3(threads), 0, stream,
                                         (const bf16*)x, (const bf16*)res, (const bf16*)g, (const bf16*)b,
                                         (bf16*)y, H, eps));
  } else {
    DISPATCH_CPT(cpt, hipLaunchKernelGGL((layernorm_kernel<CPT, false>), dim3(T), dim3(threads), 0, stream,
                                         (const bf16*)x, (const bf16*)res, (const bf16*)g, (const bf16*)b,
                                         (bf16*)y, H, eps));
  }
  PENNY_RETURN_LAUNCH();
}
