// Flat-buffer SGD (+momentum / dampening / weight decay / nesterov) in ONE launch for gfx950.
//
// Reference: torch.optim.SGD(lr=1e-2, momentum=0.9) stepped per tensor
// (Module_3/TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:181, Module_3/part3_mpi_gpu_train.py:106), which
// dispatches several elementwise kernels per parameter.  Here all parameters live in one contiguous fp32
// buffer (models flatten their parameters), so the whole update is one vectorised streaming kernel.
// Optional fp16-AMP support (the reference's GradScaler path, part3_mpi_gpu_train.py:317,371-376):
// grads are multiplied by ``inv_scale`` and a non-finite grad sets ``*found_inf`` and skips the update.
// Semantics match torch.optim.SGD exactly, including the first-step ``buf = grad`` rule (``first`` != 0).
#include "../include/ecg_common.h"

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void check_finite_kernel(const float* __restrict__ g, long n, float inv_scale,
                                                                 int* __restrict__ found_inf) {
  long i = (long)blockIdx.x * kThreads + threadIdx.x;
  bool bad = false;
  for (; i < n; i += (long)gridDim.x * kThreads) bad |= !isfinite(g[i] * inv_scale);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(found_inf, 1);
}

__device__ __forceinline__ float sgd_one(float p, float g, float& buf, float lr, float momentum, float dampening,
                                         float wd, int nesterov, int first) {
  float d = g + wd * p;
  if (momentum != 0.f) {
    buf = first ? d : momentum * buf + (1.f - dampening) * d;
    d = nesterov ? d + momentum * buf : buf;
  }
  return p - lr * d;
}

__global__ __launch_bounds__(kThreads) void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                             float* __restrict__ mom, long n, float lr, float momentum,
                                                             float dampening, float wd, int nesterov, int first,
                                                             float inv_scale, const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;  // AMP overflow: skip the step (GradScaler semantics)
  const long n4 = n >> 2;
  long i = (long)blockIdx.x * kThreads + threadIdx.x;
  const long stride = (long)gridDim.x * kThreads;
  for (long v = i; v < n4; v += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[v];
    float4 gv = reinterpret_cast<const float4*>(g)[v];
    float4 bv = momentum != 0.f ? reinterpret_cast<float4*>(mom)[v] : make_float4(0.f, 0.f, 0.f, 0.f);
    pv.x = sgd_one(pv.x, gv.x * inv_scale, bv.x, lr, momentum, dampening, wd, nesterov, first);
    pv.y = sgd_one(pv.y, gv.y * inv_scale, bv.y, lr, momentum, dampening, wd, nesterov, first);
    pv.z = sgd_one(pv.z, gv.z * inv_scale, bv.z, lr, momentum, dampening, wd, nesterov, first);
    pv.w = sgd_one(pv.w, gv.w * inv_scale, bv.w, lr, momentum, dampening, wd, nesterov, first);
    reinterpret_cast<float4*>(p)[v] = pv;
    if (momentum != 0.f) reinterpret_cast<float4*>(mom)[v] = bv;
  }
  for (long e = (n4 << 2) + i; e < n; e += stride) {
    float b = momentum != 0.f ? mom[e] : 0.f;
    p[e] = sgd_one(p[e], g[e] * inv_scale, b, lr, momentum, dampening, wd, nesterov, first);
    if (momentum != 0.f) mom[e] = b;
  }
}

}  // namespace

ECG_API int ecg_sgd_flat(float* params, const float* grads, float* mom, long n, float lr, float momentum,
                         float dampening, float wd, int nesterov, int first, float inv_scale, int* found_inf,
                         hipStream_t stream) {
  if (!params || !grads || n <= 0) return ecg::kBadArg;
  if (momentum != 0.f && !mom) return ecg::kBadArg;
  if ((((uintptr_t)params) | ((uintptr_t)grads) | ((uintptr_t)mom)) & 15) return ecg::kBadArg;
  long blocks = ecg::ceil_div<long>(ecg::ceil_div<long>(n, 4), kThreads);
  if (blocks > 2048) blocks = 2048;
  if (found_inf) {
    hipLaunchKernelGGL(check_finite_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, stream, grads, n, inv_scale,
                       found_inf);
    ECG_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(sgd_flat_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, stream, params, grads, mom, n, lr,
                     momentum, dampening, wd, nesterov, first, inv_scale, found_inf);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}
