// Common device helpers for the CrossScale-ECG gfx950 (MI355X / CDNA4) kernels.
// Written for wave64 + MFMA; no CUDA or multi-platform paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ECG_API extern "C" __attribute__((visibility("default")))

// The inter-workgroup hand-offs of these kernels (bn_tail.h tickets, the split-K / slab last-arriver reducers,
// the conv1d flag call) rely on gfx950 code generation: relaxed agent-scope atomic stores/loads lower to
// global_* ... sc1 (write-through / L1-bypassing), which is row 1 of the MI355X guide's sc1 hand-off table and
// needs no release/acquire fence.  Another target may lower them differently, so refuse to build for it.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "CrossScale-ECG kernels are written for gfx950 (MI355X) only: the sc1 hand-offs are not valid elsewhere"
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace ecg {

constexpr int kWave = 64;

// Status codes returned by every C-ABI launcher (0 == success).
enum Status : int {
  kOk = 0,
  kBadArg = 1,
  kTooLarge = 2,
  kHipError = 3,
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Round-to-nearest-even fp32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ __bf16 to_bf16(float x) { return (__bf16)x; }
__device__ __forceinline__ float from_bf16(__bf16 x) { return (float)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sum across the 4 lane-quarters that share (lane & 15): lanes l, l^16, l^32, l^48.
__device__ __forceinline__ float quarter_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

template <typename T>
__host__ __device__ __forceinline__ T ceil_div(T a, T b) { return (a + b - 1) / b; }

}  // namespace ecg

#define ECG_HIP_CHECK(expr)                          \
  do {                                               \
    hipError_t _e = (expr);                          \
    if (_e != hipSuccess) return ecg::kHipError;     \
  } while (0)
