// Single-channel "valid" conv1d (cross-correlation) for gfx950 - the Module-2 kernel.
//
//   y[b, i] = sum_{k<K} x[b, i + k] * w[k],   x:[B, L], w:[K], y:[B, L-K+1]
//
// Same math and C ABI shape as the reference CPU kernel conv1d_batch_omp_simd
// (Module_2/conv1d_openmp_simd.c:21-61, OpenMP over batch + AVX2 over taps).  MI355X design:
// one 256-thread workgroup per window; the window (+ tail) is staged into LDS with 16-byte global
// loads, the K taps live in registers (compile-time K for the benchmarked 3/5/7 and a runtime
// loop otherwise), and output positions are spread over lanes so every LDS read and global store is
// unit-stride across the wave (conflict-free, fully coalesced).  The op is latency/launch bound
// (B=512, L=500 is 1 MB in / 1 MB out), so the design goal is a single short launch with no
// workspace, no solver lookup and no host sync - what beats MIOpen's general convolution path here.
#include "../include/ecg_common.h"

namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return (float)(*p); }

template <int KC, typename TX, typename TY>
__global__ __launch_bounds__(kThreads) void conv1d_valid_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                                 TY* __restrict__ y, int L, int K, int outL,
                                                                 int rows_per_block, int B) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xs = reinterpret_cast<float*>(smem);
  const int Kr = KC > 0 ? KC : K;
  float wr[KC > 0 ? KC : 1];
  if constexpr (KC > 0) {
#pragma unroll
    for (int k = 0; k < KC; ++k) wr[k] = w[k];
  }
  const int Lpad = (L + 3) & ~3;
  for (int rr = 0; rr < rows_per_block; ++rr) {
    const int b = blockIdx.x * rows_per_block + rr;
    if (b >= B) break;
    const TX* xrow = x + (long)b * L;
    // stage x row into LDS (vectorised when the row is 16-B aligned)
    if constexpr (sizeof(TX) == 4) {
      if ((((uintptr_t)xrow) & 15) == 0) {
        const int n4 = L >> 2;
        for (int i = threadIdx.x; i < n4; i += kThreads)
          reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(xrow)[i];
        for (int i = (n4 << 2) + threadIdx.x; i < L; i += kThreads) xs[i] = xrow[i];
      } else {
        for (int i = threadIdx.x; i < L; i += kThreads) xs[i] = xrow[i];
      }
    } else {
      for (int i = threadIdx.x; i < L; i += kThreads) xs[i] = ld(xrow + i);
    }
    for (int i = L + threadIdx.x; i < Lpad + 64; i += kThreads) xs[i] = 0.f;
    __syncthreads();
    TY* yrow = y + (long)b * outL;
    for (int i = threadIdx.x; i < outL; i += kThreads) {
      float acc = 0.f;
      if constexpr (KC > 0) {
#pragma unroll
        for (int k = 0; k < KC; ++k) acc = fmaf(xs[i + k], wr[k], acc);
      } else {
        for (int k = 0; k < Kr; ++k) acc = fmaf(xs[i + k], w[k], acc);
      }
      yrow[i] = (TY)acc;
    }
    __syncthreads();
  }
}

template <typename TX, typename TY>
int launch(const TX* x, const float* w, TY* y, int B, int L, int K, hipStream_t stream) {
  if (B <= 0 || L <= 0 || K <= 0 || K > L) return ecg::kBadArg;
  const int outL = L - K + 1;
  const size_t smem = (size_t)(((L + 3) & ~3) + 64) * sizeof(float);
  if (smem > 160 * 1024) return ecg::kTooLarge;
  // one window per block; big batches pack two rows per block to halve the block count
  const int rpb = B >= 2048 ? 2 : 1;
  dim3 grid((B + rpb - 1) / rpb), block(kThreads);
  switch (K) {
#define ECG_CASE(KK)                                                                                           \
  case KK:                                                                                                     \
    if (smem > 64 * 1024)                                                                                      \
      ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_valid_kernel<KK, TX, TY>,                         \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));               \
    hipLaunchKernelGGL((conv1d_valid_kernel<KK, TX, TY>), grid, block, smem, stream, x, w, y, L, K, outL, rpb, B); \
    break;
    ECG_CASE(3)
    ECG_CASE(5)
    ECG_CASE(7)
    ECG_CASE(9)
    ECG_CASE(11)
    ECG_CASE(15)
    ECG_CASE(32)
#undef ECG_CASE
    default:
      if (smem > 64 * 1024)
        ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_valid_kernel<0, TX, TY>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
      hipLaunchKernelGGL((conv1d_valid_kernel<0, TX, TY>), grid, block, smem, stream, x, w, y, L, K, outL, rpb, B);
  }
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

}  // namespace

// C-ABI twin of the reference's conv1d_batch_omp_simd(x, w, y, batch, L, K, nthreads):
// the thread count is replaced by the HIP stream the kernel is enqueued on (async, no sync).
ECG_API int conv1d_batch_hip(const float* x, const float* w, float* y, int batch, int L, int K, hipStream_t stream) {
  return launch<float, float>(x, w, y, batch, L, K, stream);
}

// bf16 activations in/out, fp32 taps and accumulation.
ECG_API int conv1d_batch_hip_bf16(const __bf16* x, const float* w, __bf16* y, int batch, int L, int K,
                                  hipStream_t stream) {
  return launch<__bf16, __bf16>(x, w, y, batch, L, K, stream);
}
