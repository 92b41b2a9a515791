// Batch gather + optional per-window z-score for gfx950.
//
// Reference: the per-step device gather ``x_gpu[perm[start:start+B]]`` of
// Module_3/shard_dataset.py:133-136 (index kernel + unsqueeze) and the LABL prefetcher's per-window
// normalisation ``(x - mean) / (std + 1e-8)`` computed in float64 on the CPU
// (Module_1/labl_loader(EXPERIMENTAL).py:65-69).  Here one wave handles one window: 16-byte loads,
// mean/variance by wave reductions in fp32 (two-pass, numerically matched to the float64 reference
// within fp32 rounding), written into a preallocated (graph-capturable) batch buffer in fp32 or bf16.
#include "../include/ecg_common.h"

namespace {

constexpr int kWavesPerBlock = 4;

template <typename TO>
__global__ __launch_bounds__(kWavesPerBlock * 64) void gather_rows_kernel(const float* __restrict__ X, long ldx, int L,
                                                                          const int* __restrict__ idx, int B,
                                                                          TO* __restrict__ out, long ldo, int normalize,
                                                                          float eps) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (b >= B) return;
  const long r = idx ? (long)idx[b] : (long)b;
  const float* src = X + r * ldx;
  TO* dst = out + (long)b * ldo;
  float mean = 0.f, inv = 1.f;
  if (normalize) {
    float s = 0.f;
    for (int i = lane; i < L; i += 64) s += src[i];
    mean = ecg::wave_sum(s) / (float)L;
    float v = 0.f;
    for (int i = lane; i < L; i += 64) {
      float d = src[i] - mean;
      v = fmaf(d, d, v);
    }
    float var = ecg::wave_sum(v) / (float)L;  // population std, as numpy .std()
    inv = 1.f / (sqrtf(var) + eps);
  }
  const bool vec = ((((uintptr_t)src) & 15) == 0) && (L % 4 == 0) && sizeof(TO) == 4 &&
                   ((((uintptr_t)dst) & 15) == 0);
  if (vec) {
    for (int i = lane; i < (L >> 2); i += 64) {
      float4 v = reinterpret_cast<const float4*>(src)[i];
      v.x = (v.x - mean) * inv; v.y = (v.y - mean) * inv; v.z = (v.z - mean) * inv; v.w = (v.w - mean) * inv;
      reinterpret_cast<float4*>(dst)[i] = v;
    }
  } else {
    for (int i = lane; i < L; i += 64) dst[i] = (TO)((src[i] - mean) * inv);
  }
}

template <typename TO>
int launch(const float* X, long ldx, int L, const int* idx, int B, TO* out, long ldo, int normalize, float eps,
           hipStream_t stream) {
  if (!X || !out || L <= 0 || B <= 0 || ldx < L || ldo < L) return ecg::kBadArg;
  dim3 grid(ecg::ceil_div(B, kWavesPerBlock)), block(kWavesPerBlock * 64);
  hipLaunchKernelGGL(gather_rows_kernel<TO>, grid, block, 0, stream, X, ldx, L, idx, B, out, ldo, normalize, eps);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

}  // namespace

ECG_API int ecg_gather_rows_f32(const float* X, long ldx, int L, const int* idx, int B, float* out, long ldo,
                                int normalize, float eps, hipStream_t stream) {
  return launch<float>(X, ldx, L, idx, B, out, ldo, normalize, eps, stream);
}

ECG_API int ecg_gather_rows_bf16(const float* X, long ldx, int L, const int* idx, int B, __bf16* out, long ldo,
                                 int normalize, float eps, hipStream_t stream) {
  return launch<__bf16>(X, ldx, L, idx, B, out, ldo, normalize, eps, stream);
}
