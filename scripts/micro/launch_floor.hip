// Dispatch floor of a grid shaped like the fused TinyECG step (B workgroups x T threads, S bytes of dynamic LDS):
// N back-to-back launches of a kernel that touches its LDS once and exits, captured in one hipGraph; prints
// microseconds per launch for each shape.  Also the same with a dependent second kernel of 46 x 512 threads (the
// slab reduce's shape) in between.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void touch(float* out) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = lds[1];
}

__global__ void small(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = 1.f;
}

static int run(int B, int T, int S, bool pair, float* out, hipStream_t st) {
  const int N = 200;
  if (S > 64 * 1024) CK(hipFuncSetAttribute((const void*)touch, hipFuncAttributeMaxDynamicSharedMemorySize, S));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < N; ++i) {
    hipLaunchKernelGGL(touch, dim3(B), dim3(T), S, st, out);
    if (pair) hipLaunchKernelGGL(small, dim3(46), dim3(512), 0, st, out);
  }
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("B=%4d T=%4d LDS=%6d %s: %.3f us per %s\n", B, T, S, pair ? "+reduce-shape" : "alone        ",
         ms * 1e3f / (5 * N), pair ? "pair" : "launch");
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  float* out;
  hipStream_t st;
  CK(hipMalloc(&out, 64));
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int shapes[][3] = {{256, 64, 0}, {256, 256, 0}, {256, 1024, 0}, {256, 1024, 40 * 1024}, {256, 1024, 80 * 1024}, {256, 1024, 83472},
                           {256, 512, 40 * 1024}, {128, 1024, 40 * 1024}, {512, 512, 40 * 1024}};
  for (auto& s : shapes)
    for (int pair = 0; pair < 2; ++pair)
      if (run(s[0], s[1], s[2], pair, out, st)) return 1;
  return 0;
}
