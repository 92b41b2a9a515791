// Single-channel "valid" conv1d (cross-correlation) for gfx950 - the Module-2 kernel, forward and backward.
//
//   forward  y[b, i]  = sum_{k<K} x[b, i + k] * w[k]                 x:[B, L], w:[K], y:[B, outL], outL = L-K+1
//   dgrad    dx[b, j] = sum_{k<K} dy[b, j - k] * w[k]   (0 <= j-k < outL)
//   wgrad    dw[k]    = sum_{b, i} x[b, i + k] * dy[b, i]
//
// Same math and C ABI shape as the reference CPU kernel conv1d_batch_omp_simd
// (Module_2/conv1d_openmp_simd.c:21-61: OpenMP over the batch, AVX2 over taps).  The op moves ~2 KB per window
// and is launch/latency bound (B=512, L=500 is 1 MB in, 1 MB out), so the MI355X design minimises the dependent
// chain of a launch rather than arithmetic:
//   * one thread per QUAD of outputs (4 consecutive positions of one window), flat grid over (window, quad):
//     B=256, L=500 is 124 quads x 256 windows = 124 workgroups of 256 threads, well under one wave per SIMD;
//   * the quad's input span x[4q .. 4q+3+K-1] comes straight from global memory into registers as 16-byte
//     vectors (ceil((K+3)/4) loads, all issued before the first FMA; neighbouring lanes share cache lines, so
//     the halo costs L1/L2 hits, not HBM bytes) - no LDS staging, no barrier, one memory round trip;
//   * the K taps are scalar loads kept in SGPRs (compile-time K for 3/5/7/9/11/15/32, a runtime loop
//     otherwise); 4K FMAs per thread; 16-byte stores when the output rows are 16-byte aligned.
//   * wgrad: per-workgroup partial sums [G][K] (fixed order) + a one-workgroup second pass - deterministic.
#include "../include/ecg_common.h"

#include <chrono>
#include <cstring>
#include <mutex>

namespace {

constexpr int kThreads = 256;

template <typename T>
struct Vec4;
template <>
struct Vec4<float> {
  typedef float4 type;
  __device__ static inline void unpack(const float4& v, float* o) {
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
};
template <>
struct Vec4<__bf16> {
  typedef bf16x4 type;
  __device__ static inline void unpack(const bf16x4& v, float* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (float)v[j];
  }
};

__device__ __forceinline__ void store1(float* p, float v) { *p = v; }
__device__ __forceinline__ void store1(__bf16* p, float v) { *p = (__bf16)v; }

// Loads 4 * NV consecutive elements of a row starting at ``pos`` (zero at and beyond ``len``) into ``o``.
// ``vec``: the row base is 16-byte (fp32) / 8-byte (bf16) aligned and len % 4 == 0, so a 4-vector is either
// entirely inside the row or entirely past its end.
template <int NV, typename T>
__device__ __forceinline__ void load_span(const T* __restrict__ row, int pos, int len, bool vec, float* o) {
  if (vec) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (pos + 4 * v < len) {
        const typename Vec4<T>::type q = reinterpret_cast<const typename Vec4<T>::type*>(row + pos)[v];
        Vec4<T>::unpack(q, o + 4 * v);
      } else {
        o[4 * v] = o[4 * v + 1] = o[4 * v + 2] = o[4 * v + 3] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4 * NV; ++e) o[e] = (pos + e < len) ? (float)row[pos + e] : 0.f;
  }
}

template <typename TY>
__device__ __forceinline__ void store_quad(TY* __restrict__ yrow, int pos, int len, bool vec, const float* acc) {
  if (vec && pos + 3 < len) {
    if constexpr (sizeof(TY) == 4) {
      *reinterpret_cast<float4*>(yrow + pos) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (__bf16)acc[j];
      *reinterpret_cast<bf16x4*>(yrow + pos) = o;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (pos + j < len) store1(yrow + pos + j, acc[j]);
  }
}

// ------------------------------------------------------------------------------- forward, completion flag
// The blocking single call (Module-2's "one call returns a complete output", Module_2/benchmark_part_2.py:61-67):
// the same per-quad math with kFlagQPT quads per thread (all loads first), then a completion hand-off the host
// can see without the runtime's kernel-completion path: every wave drains its stores (vmcnt(0)), one lane per
// workgroup takes an agent-scope ticket, and the last workgroup resets the ticket counter and stores ``epoch``
// to ONE host-mapped word (system scope) that the calling thread polls.  (Measured: one word per workgroup, all
// polled by the host, instead of the ticket - 13.4 vs 11.3 us per call at B=256: 31 fabric writes into the
// polled lines cost more than the ~12 ns-per-arrival ticket.)  Later device work is stream-ordered behind the
// kernel as usual; the host only stops waiting for the runtime's end-of-kernel signal.
template <int KC, int kFlagQPT, int kFlagThreads>
__global__ __launch_bounds__(kFlagThreads) void conv1d_valid_fwd_flag_kernel(
    const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int B, int L, int K, int outL,
    int nquads, int xvec, int yvec, unsigned* __restrict__ counter, unsigned* __restrict__ host_flag,
    unsigned epoch) {
  constexpr int NV = (KC + 3 + 3) / 4;
  const long total = (long)B * nquads;
  const long base = (long)blockIdx.x * kFlagThreads * kFlagQPT + threadIdx.x;  // quad u: base + u * threads
  float xv[kFlagQPT][4 * NV];
  float wr[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) wr[k] = w[k];
#pragma unroll
  for (int u = 0; u < kFlagQPT; ++u) {
    const long gq = base + (long)u * kFlagThreads;
    if (gq < total) {
      const int b = (int)(gq / nquads), q = (int)(gq - (long)b * nquads);
      load_span<NV>(x + (long)b * L, 4 * q, L, xvec != 0, xv[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < kFlagQPT; ++u) {
    const long gq = base + (long)u * kFlagThreads;
    if (gq < total) {
      const int b = (int)(gq / nquads), q = (int)(gq - (long)b * nquads);
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(xv[u][j + k], wr[k], acc[j]);
      store_quad(y + (long)b * outL, 4 * q, outL, yvec != 0, acc);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's output stores have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // relaxed: the host learns "done" from this word and never reads y through it (later device work is
      // stream-ordered behind the kernel), so no L2 write-back (buffer_wbl2) is needed in front of it
      __hip_atomic_store(host_flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ------------------------------------------------------------------------------------------------- forward
template <int KC, typename TX, typename TY>
__global__ __launch_bounds__(kThreads) void conv1d_valid_fwd_kernel(const TX* __restrict__ x,
                                                                     const float* __restrict__ w,
                                                                     TY* __restrict__ y, int B, int L, int K,
                                                                     int outL, int nquads, int xvec, int yvec) {
  const long gq = (long)blockIdx.x * kThreads + threadIdx.x;
  if (gq >= (long)B * nquads) return;
  const int b = (int)(gq / nquads), q = (int)(gq - (long)b * nquads);
  const int i0 = 4 * q;
  const TX* xrow = x + (long)b * L;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (KC > 0) {
    constexpr int NV = (KC + 3 + 3) / 4;
    float xv[4 * NV];
    load_span<NV>(xrow, i0, L, xvec != 0, xv);
    float wr[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) wr[k] = w[k];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(xv[j + k], wr[k], acc[j]);
  } else {
    for (int k = 0; k < K; ++k) {
      const float wk = w[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = i0 + j + k;
        acc[j] = fmaf(e < L ? (float)xrow[e] : 0.f, wk, acc[j]);
      }
    }
  }
  store_quad(y + (long)b * outL, i0, outL, yvec != 0, acc);
}

// --------------------------------------------------------------------------------------------- data grad
// dx[j] for j in [4q, 4q+4): needs dy[j-K+1 .. j] -> the span dy[4q-K+1 .. 4q+3] (zero outside [0, outL)).
template <int KC, typename T>
__global__ __launch_bounds__(kThreads) void conv1d_valid_dgrad_kernel(const T* __restrict__ dy,
                                                                       const float* __restrict__ w,
                                                                       T* __restrict__ dx, int B, int L, int K,
                                                                       int outL, int nquads, int xvec) {
  const long gq = (long)blockIdx.x * kThreads + threadIdx.x;
  if (gq >= (long)B * nquads) return;
  const int b = (int)(gq / nquads), q = (int)(gq - (long)b * nquads);
  const int j0 = 4 * q;
  const T* dyrow = dy + (long)b * outL;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (KC > 0) {
    // span element s <-> dy index j0 - KC + 1 + s, s in [0, KC + 3)
    const int base = j0 - KC + 1;
    float dv[KC + 3];
#pragma unroll
    for (int s = 0; s < KC + 3; ++s) {
      const int e = base + s;
      dv[s] = (e >= 0 && e < outL) ? (float)dyrow[e] : 0.f;
    }
    float wr[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) wr[k] = w[k];
    // dx[j0 + jj] = sum_k dy[j0 + jj - k] w[k] = sum_k dv[jj - k + KC - 1] w[k]
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[jj] = fmaf(dv[jj - k + KC - 1], wr[k], acc[jj]);
  } else {
    for (int k = 0; k < K; ++k) {
      const float wk = w[k];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int e = j0 + jj - k;
        acc[jj] = fmaf((e >= 0 && e < outL) ? (float)dyrow[e] : 0.f, wk, acc[jj]);
      }
    }
  }
  store_quad(dx + (long)b * L, j0, L, xvec != 0, acc);
}

// ------------------------------------------------------------------------------------------- weight grad
// Pass 1: workgroup g sums x[b, i+k] * dy[b, i] over its (window, quad) range for every tap k < K (K <= 64),
// reducing lanes -> waves -> workgroup in a fixed order; partial[g][k].  Pass 2: one workgroup sums the G rows.
constexpr int kMaxWgradK = 64;

template <typename T>
__global__ __launch_bounds__(kThreads) void conv1d_valid_wgrad_partial_kernel(const T* __restrict__ x,
                                                                               const T* __restrict__ dy,
                                                                               float* __restrict__ partial, int B,
                                                                               int L, int K, int outL, int nquads) {
  __shared__ float red[kThreads / 64][kMaxWgradK];
  const long gq = (long)blockIdx.x * kThreads + threadIdx.x;
  const bool live = gq < (long)B * nquads;
  const int b = live ? (int)(gq / nquads) : 0, q = live ? (int)(gq - (long)b * nquads) : 0;
  const int i0 = 4 * q;
  const T* xrow = x + (long)b * L;
  const T* dyrow = dy + (long)b * outL;
  float d[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) d[j] = (live && i0 + j < outL) ? (float)dyrow[i0 + j] : 0.f;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = i0 + j + k;
      s = fmaf((live && e < L) ? (float)xrow[e] : 0.f, d[j], s);
    }
    s = ecg::wave_sum(s);
    if (lane == 0) red[wv][k] = s;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += kThreads) {
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < kThreads / 64; ++v) s += red[v][k];
    partial[(long)blockIdx.x * K + k] = s;
  }
}

__global__ __launch_bounds__(kThreads) void conv1d_valid_wgrad_final_kernel(const float* __restrict__ partial,
                                                                             float* __restrict__ dw, int G, int K) {
  __shared__ float red[kThreads / 64];
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
    for (int g = threadIdx.x; g < G; g += kThreads) s += partial[(long)g * K + k];
    s = ecg::wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
#pragma unroll
      for (int v = 0; v < kThreads / 64; ++v) t += red[v];
      dw[k] = t;
    }
    __syncthreads();
  }
}

template <typename T>
inline bool vec_ok(const T* p, int len) {
  return (((uintptr_t)p) % (4 * sizeof(T))) == 0 && (len % 4) == 0;
}

#define ECG_K_SWITCH(K, LAUNCH) \
  switch (K) {                  \
    case 3: LAUNCH(3); break;   \
    case 5: LAUNCH(5); break;   \
    case 7: LAUNCH(7); break;   \
    case 9: LAUNCH(9); break;   \
    case 11: LAUNCH(11); break; \
    case 15: LAUNCH(15); break; \
    case 32: LAUNCH(32); break; \
    default: LAUNCH(0);         \
  }

template <typename TX, typename TY>
int launch_fwd(const TX* x, const float* w, TY* y, int B, int L, int K, hipStream_t stream) {
  if (B <= 0 || L <= 0 || K <= 0 || K > L) return ecg::kBadArg;
  const int outL = L - K + 1;
  const int nquads = (outL + 3) / 4;
  const long threads = (long)B * nquads;
  const dim3 grid((unsigned)((threads + kThreads - 1) / kThreads)), block(kThreads);
  const int xv = vec_ok(x, L), yv = vec_ok(y, outL);
#define ECG_FWD(KK)                                                                                          \
  hipLaunchKernelGGL((conv1d_valid_fwd_kernel<KK, TX, TY>), grid, block, 0, stream, x, w, y, B, L, K, outL, \
                     nquads, xv, yv)
  ECG_K_SWITCH(K, ECG_FWD)
#undef ECG_FWD
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

template <typename T>
int launch_dgrad(const T* dy, const float* w, T* dx, int B, int L, int K, hipStream_t stream) {
  if (B <= 0 || L <= 0 || K <= 0 || K > L) return ecg::kBadArg;
  const int outL = L - K + 1;
  const int nquads = (L + 3) / 4;
  const long threads = (long)B * nquads;
  const dim3 grid((unsigned)((threads + kThreads - 1) / kThreads)), block(kThreads);
  const int xv = vec_ok(dx, L);
#define ECG_DG(KK)                                                                                              \
  hipLaunchKernelGGL((conv1d_valid_dgrad_kernel<KK, T>), grid, block, 0, stream, dy, w, dx, B, L, K, outL, nquads, \
                     xv)
  ECG_K_SWITCH(K, ECG_DG)
#undef ECG_DG
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

template <typename T>
int launch_wgrad(const T* x, const T* dy, float* dw, float* ws, long ws_floats, int B, int L, int K,
                 hipStream_t stream) {
  if (B <= 0 || L <= 0 || K <= 0 || K > L || K > kMaxWgradK) return ecg::kBadArg;
  const int outL = L - K + 1;
  const int nquads = (outL + 3) / 4;
  const long threads = (long)B * nquads;
  const int G = (int)((threads + kThreads - 1) / kThreads);
  if ((long)G * K > ws_floats) return ecg::kBadArg;
  hipLaunchKernelGGL((conv1d_valid_wgrad_partial_kernel<T>), dim3(G), dim3(kThreads), 0, stream, x, dy, ws, B, L, K,
                     outL, nquads);
  hipLaunchKernelGGL(conv1d_valid_wgrad_final_kernel, dim3(1), dim3(kThreads), 0, stream, ws, dw, G, K);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

}  // namespace

// C-ABI twin of the reference's conv1d_batch_omp_simd(x, w, y, batch, L, K, nthreads):
// the thread count is replaced by the HIP stream the kernel is enqueued on (async, no sync).
ECG_API int conv1d_batch_hip(const float* x, const float* w, float* y, int batch, int L, int K, hipStream_t stream) {
  return launch_fwd<float, float>(x, w, y, batch, L, K, stream);
}

// Blocking twin (the reference's CPU kernel returns when its output is complete): launch, then wait for the
// stream.  One native call covers the whole "result ready" path the Module-2 single-call metric times.
ECG_API int conv1d_batch_hip_sync(const float* x, const float* w, float* y, int batch, int L, int K,
                                  hipStream_t stream) {
  const int st = launch_fwd<float, float>(x, w, y, batch, L, K, stream);
  if (st) return st;
  ECG_HIP_CHECK(hipStreamSynchronize(stream));
  return ecg::kOk;
}

// Same, but the host polls the stream instead of sleeping in hipStreamSynchronize (no wake-up latency; the
// calling thread spins for the few microseconds the kernel runs).
ECG_API int conv1d_batch_hip_spin(const float* x, const float* w, float* y, int batch, int L, int K,
                                  hipStream_t stream) {
  const int st = launch_fwd<float, float>(x, w, y, batch, L, K, stream);
  if (st) return st;
  hipError_t e;
  while ((e = hipStreamQuery(stream)) == hipErrorNotReady) {
  }
  return e == hipSuccess ? ecg::kOk : ecg::kHipError;
}

// Per-device completion state of the flag call: a zeroed ticket counter (device) and a host-mapped flag word.
namespace {
struct FlagState {
  unsigned* counter = nullptr;
  unsigned* flag_host = nullptr;
  unsigned* flag_dev = nullptr;
  unsigned epoch = 0;
};
std::mutex g_flag_mu;
FlagState g_flag[64];
}  // namespace

// Blocking forward that returns as soon as the kernel's last workgroup has published completion (see
// conv1d_valid_fwd_flag_kernel): launch, then poll a host-mapped word.  K must be one of the compile-time tap
// counts (3, 5, 7, 9, 11, 15, 32) - else the plain launch + hipStreamSynchronize runs.  A poll that outlives
// ``timeout`` falls back to hipStreamSynchronize (so a fault is reported by the runtime, never hidden).
ECG_API int conv1d_batch_hip_flag(const float* x, const float* w, float* y, int batch, int L, int K,
                                  hipStream_t stream) {
  if (batch <= 0 || L <= 0 || K <= 0 || K > L) return ecg::kBadArg;
  const bool kc = K == 3 || K == 5 || K == 7 || K == 9 || K == 11 || K == 15 || K == 32;
  if (!kc) return conv1d_batch_hip_sync(x, w, y, batch, L, K, stream);
  int dev = 0;
  ECG_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return ecg::kBadArg;
  std::lock_guard<std::mutex> lk(g_flag_mu);
  FlagState& f = g_flag[dev];
  const int outL = L - K + 1, nquads = (outL + 3) / 4;
  const long total = (long)batch * nquads;
  // ECG_CONV1D_FLAG_CFG (A/B, read once): threads x quads per thread = 0: 512x2, 1: 512x4, 2: 1024x2, 3: 256x1
  // (default), 4: 128x1, 5: 64x1.  B=256, L=500, K=7 single call (profiles/r2/conv1d_flag_call_ab.txt): 10.6,
  // 12.4, 12.4, 9.4-9.6, 10.5, 13.4 us - the 124 workgroups of one quad per thread beat fatter threads (less
  // ticket fan-in) and thinner workgroups (more of it).
  // 6: 256x2.  Default (unset): 256x1 up to 160 workgroups, else 256x2 (the ticket fan-in grows with the
  // workgroup count: B=512 at 256x1 is 248 tickets).
  static const int cfg = [] {
    const char* e = getenv("ECG_CONV1D_FLAG_CFG");
    return e ? atoi(e) : -1;
  }();
  static const int kNT[7] = {512, 512, 1024, 256, 128, 64, 256}, kQ[7] = {2, 4, 2, 1, 1, 1, 2};
  const int ci = cfg < 0 ? ((total + 255) / 256 <= 160 ? 3 : 6) : (cfg > 6 ? 0 : cfg);
  const int nt = kNT[ci], qpt = kQ[ci];
  const long G = (total + (long)nt * qpt - 1) / ((long)nt * qpt);
  if (G > 0x7fffffffL) return ecg::kBadArg;
  if (!f.counter) {
    ECG_HIP_CHECK(hipMalloc(&f.counter, 64));
    ECG_HIP_CHECK(hipMemset(f.counter, 0, 64));
    ECG_HIP_CHECK(hipHostMalloc(&f.flag_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
    ECG_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&f.flag_dev), f.flag_host, 0));
    __atomic_store_n(f.flag_host, 0u, __ATOMIC_RELEASE);
    ECG_HIP_CHECK(hipDeviceSynchronize());  // the counter's memset has landed before the first ticket
  }
  const unsigned epoch = ++f.epoch == 0 ? ++f.epoch : f.epoch;  // never 0 (the flag's initial value)
  const dim3 grid((unsigned)G);
  const int xv = vec_ok(x, L), yv = vec_ok(y, outL);
#define ECG_FLAG_CFG(KK, Q, T)                                                                                    \
  hipLaunchKernelGGL((conv1d_valid_fwd_flag_kernel<KK, Q, T>), grid, dim3(T), 0, stream, x, w, y, batch, L, K, outL, \
                     nquads, xv, yv, f.counter, f.flag_dev, epoch)
#define ECG_FLAG(KK)                                              \
  do {                                                            \
    if (ci == 1) ECG_FLAG_CFG(KK, 4, 512);                        \
    else if (ci == 2) ECG_FLAG_CFG(KK, 2, 1024);                  \
    else if (ci == 3) ECG_FLAG_CFG(KK, 1, 256);                   \
    else if (ci == 4) ECG_FLAG_CFG(KK, 1, 128);                   \
    else if (ci == 5) ECG_FLAG_CFG(KK, 1, 64);                    \
    else if (ci == 6) ECG_FLAG_CFG(KK, 2, 256);                   \
    else ECG_FLAG_CFG(KK, 2, 512);                                \
  } while (0)
  switch (K) {
    case 3: ECG_FLAG(3); break;
    case 5: ECG_FLAG(5); break;
    case 7: ECG_FLAG(7); break;
    case 9: ECG_FLAG(9); break;
    case 11: ECG_FLAG(11); break;
    case 15: ECG_FLAG(15); break;
    default: ECG_FLAG(32); break;
  }
#undef ECG_FLAG_CFG
#undef ECG_FLAG
  ECG_HIP_CHECK(hipGetLastError());
  // Poll the word; from 8 us on (a typical call is done by ~9.5 us) also ask the runtime every 3 us
  // (hipStreamQuery costs ~1 us of host time per call), so a call whose completion word is slow to reach host
  // memory (seen in some Module-2 grid cells: 28 us against 9-11 typical) returns no later than the runtime's
  // own completion signal would let it.
  const auto t0 = std::chrono::steady_clock::now();
  auto next_q = t0 + std::chrono::microseconds(8);
  for (long it = 0; __atomic_load_n(f.flag_host, __ATOMIC_ACQUIRE) != epoch; ++it) {
    __builtin_ia32_pause();
    if ((it & 31) == 31) {
      const auto now = std::chrono::steady_clock::now();
      if (now >= next_q) {
        const hipError_t q = hipStreamQuery(stream);
        if (q == hipSuccess) return ecg::kOk;  // the kernel (and everything before it) completed
        if (q != hipErrorNotReady) return ecg::kHipError;
        next_q = now + std::chrono::microseconds(3);
      }
      if (now - t0 > std::chrono::milliseconds(2000)) {  // a fault or a stuck queue
        ECG_HIP_CHECK(hipStreamSynchronize(stream));
        return __atomic_load_n(f.flag_host, __ATOMIC_ACQUIRE) == epoch ? ecg::kOk : ecg::kHipError;
      }
    }
  }
  return ecg::kOk;
}

// bf16 activations in/out, fp32 taps and accumulation.
ECG_API int conv1d_batch_hip_bf16(const __bf16* x, const float* w, __bf16* y, int batch, int L, int K,
                                  hipStream_t stream) {
  return launch_fwd<__bf16, __bf16>(x, w, y, batch, L, K, stream);
}

// Backward: dx [B, L] from dy [B, L-K+1] (fp32 or bf16 with fp32 accumulation).
ECG_API int conv1d_valid_dgrad_hip(const float* dy, const float* w, float* dx, int batch, int L, int K,
                                   hipStream_t stream) {
  return launch_dgrad<float>(dy, w, dx, batch, L, K, stream);
}
ECG_API int conv1d_valid_dgrad_hip_bf16(const __bf16* dy, const float* w, __bf16* dx, int batch, int L, int K,
                                        hipStream_t stream) {
  return launch_dgrad<__bf16>(dy, w, dx, batch, L, K, stream);
}

// Floats of workspace the weight gradient needs (one partial row of K per workgroup).
ECG_API long conv1d_valid_wgrad_ws_floats(int batch, int L, int K) {
  const long nquads = (L - K + 1 + 3) / 4;
  return ((long)batch * nquads + kThreads - 1) / kThreads * (long)K;
}

// dw [K] (fp32) from x [B, L] and dy [B, L-K+1]; deterministic two-pass reduction through ``ws``.
ECG_API int conv1d_valid_wgrad_hip(const float* x, const float* dy, float* dw, float* ws, long ws_floats, int batch,
                                   int L, int K, hipStream_t stream) {
  return launch_wgrad<float>(x, dy, dw, ws, ws_floats, batch, L, K, stream);
}
ECG_API int conv1d_valid_wgrad_hip_bf16(const __bf16* x, const __bf16* dy, float* dw, float* ws, long ws_floats,
                                        int batch, int L, int K, hipStream_t stream) {
  return launch_wgrad<__bf16>(x, dy, dw, ws, ws_floats, batch, L, K, stream);
}
