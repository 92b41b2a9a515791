// Feasibility probe for the ResNet step's two lanes as LINEAR graphs (one per lane) joined by external event
// nodes, against the eager two-stream enqueue the plan runner uses (csrc/kernels/resnet_nlc.hip ecg_plan_run_ex):
//   main lane: NM kernels, an external event record after every FK-th (the fork points)
//   side lane: NF kernels, kernel k behind an external wait on fork k; an external record of ``join`` at its end
//   join:      a last main-lane kernel behind an external wait on ``join`` (the optimizer)
// Modes: 0 eager (events without the system fence, as the plan runner), 1 three linear graphs (A = main lane,
// S = side lane, B = join + last kernel), launched A, S, B.  Every kernel records s_memrealtime at its start (first
// workgroup) and end (last workgroup to finish, via an atomic ticket), so the run checks the ordering it needs
// (side k starts after main kernel FK*k+FK-1 ended; the last kernel starts after every side kernel ended) and reports
// the main lane's idle time between kernels and the wall time per iteration.
//   hipcc -O3 --offload-arch=gfx950 lane_graphs.hip -o lane_graphs && ./lane_graphs
// Result (round 6, profiles/r6/lane_graphs.txt): the lane graphs order correctly but do not shorten the main lane's
// boundaries - and neither does a linear graph of the main lane alone against the same kernels launched eagerly
// (~1.0 us per boundary either way on ROCm 7): the two-lane plan stays eager.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                             \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

constexpr int NM = 40, FK = 4, NF = NM / FK, NSLOT = NM + NF + 1;

// stamps[slot][0] = start (first block), [1] = end (last block); tick[slot] = finished blocks
__global__ void work(unsigned long long* stamps, unsigned* tick, int slot, long cycles) {
  __shared__ float lds[8192];  // 32 KB: two of these fit next to each other on a CU
  if (threadIdx.x == 0) {
    unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0) stamps[slot * 2] = t;
  }
  const long t0 = __builtin_amdgcn_s_memtime();
  float acc = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memtime() - t0 < cycles) acc = acc * 1.0001f + 1.f;
  lds[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (lds[1] == -1.f) stamps[slot * 2] = 0;  // keep the loop alive
    __threadfence();
    const unsigned n = atomicAdd(&tick[slot], 1u);
    if (n == gridDim.x - 1) {
      stamps[slot * 2 + 1] = __builtin_amdgcn_s_memrealtime();
      tick[slot] = 0;
    }
  }
}

// An event record / wait node appended to a stream's ongoing capture by hand (the capture-time External flags
// crashed the ROCm 7.0 runtime: hipStreamWaitEvent(..., hipEventWaitExternal) on an event recorded in an earlier
// capture): the node depends on the capture's current tail, then becomes the new tail.
static void add_node(hipStream_t s, hipEvent_t e, bool record) {
  hipStreamCaptureStatus cs;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  CK(hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &n));
  hipGraphNode_t node;
  if (record)
    CK(hipGraphAddEventRecordNode(&node, g, deps, n, e));
  else
    CK(hipGraphAddEventWaitNode(&node, g, deps, n, e));
  CK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
}

static void enqueue(hipStream_t m, hipStream_t s, std::vector<hipEvent_t>& fork, hipEvent_t join,
                    unsigned long long* st, unsigned* tk, bool capture_lanes, hipGraph_t* gA, hipGraph_t* gS,
                    hipGraph_t* gB) {
  const long MC = 20000, SC = 60000, LC = 20000;  // ~10 / 30 / 10 us at ~2 GHz
  if (capture_lanes) CK(hipStreamBeginCapture(m, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < NM; ++i) {
    hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, m, st, tk, i, MC);
    if (i % FK == FK - 1) {
      if (capture_lanes) add_node(m, fork[i / FK], true);
      else CK(hipEventRecord(fork[i / FK], m));
    }
  }
  if (capture_lanes) {
    CK(hipStreamEndCapture(m, gA));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  }
  for (int k = 0; k < NF; ++k) {
    if (capture_lanes) add_node(s, fork[k], false);
    else CK(hipStreamWaitEvent(s, fork[k], 0));
    hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, s, st, tk, NM + k, SC);
  }
  if (capture_lanes) add_node(s, join, true);
  else CK(hipEventRecord(join, s));
  if (capture_lanes) {
    CK(hipStreamEndCapture(s, gS));
    CK(hipStreamBeginCapture(m, hipStreamCaptureModeThreadLocal));
  }
  if (capture_lanes) add_node(m, join, false);
  else CK(hipStreamWaitEvent(m, join, 0));
  hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, m, st, tk, NM + NF, LC);
  if (capture_lanes) CK(hipStreamEndCapture(m, gB));
}

int main() {
  hipStream_t m, s;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipEvent_t> fork(NF);
  for (auto& e : fork) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  hipEvent_t join;
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming | hipEventDisableSystemFence));
  unsigned long long* st;
  unsigned* tk;
  CK(hipMalloc(&st, NSLOT * 2 * sizeof(unsigned long long)));
  CK(hipMalloc(&tk, NSLOT * sizeof(unsigned)));
  CK(hipMemset(tk, 0, NSLOT * sizeof(unsigned)));
  hipGraph_t gA, gS, gB;
  hipGraphExec_t eA, eS, eB;
  enqueue(m, s, fork, join, st, tk, true, &gA, &gS, &gB);
  CK(hipGraphInstantiate(&eA, gA, nullptr, nullptr, 0));
  CK(hipGraphInstantiate(&eS, gS, nullptr, nullptr, 0));
  CK(hipGraphInstantiate(&eB, gB, nullptr, nullptr, 0));
  std::vector<unsigned long long> h(NSLOT * 2);
  for (int mode = 0; mode < 2; ++mode) {
    double wall_sum = 0, idle_sum = 0;
    int bad = 0, n = 0;
    for (int it = 0; it < 12; ++it) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(st, 0, NSLOT * 2 * sizeof(unsigned long long)));
      CK(hipDeviceSynchronize());
      if (mode == 0) {
        enqueue(m, s, fork, join, st, tk, false, nullptr, nullptr, nullptr);
      } else {
        CK(hipGraphLaunch(eA, m));
        CK(hipGraphLaunch(eS, s));
        CK(hipGraphLaunch(eB, m));
      }
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      if (it < 2) continue;  // warm-up
      // ordering the lanes need
      for (int k = 0; k < NF; ++k)
        if (h[(NM + k) * 2] < h[(FK * k + FK - 1) * 2 + 1]) ++bad;
      for (int k = 0; k < NF; ++k)
        if (h[(NM + NF) * 2] < h[(NM + k) * 2 + 1]) ++bad;
      for (int i = 0; i + 1 < NM; ++i)
        if (h[(i + 1) * 2] < h[i * 2 + 1]) ++bad;
      double idle = 0;
      for (int i = 0; i + 1 < NM; ++i) idle += (double)(h[(i + 1) * 2] - h[i * 2 + 1]) * 10.0 / 1000.0;  // 100 MHz
      idle_sum += idle;
      wall_sum += (double)(h[(NM + NF) * 2 + 1] - h[0]) * 10.0 / 1000.0;
      ++n;
    }
    printf("%s: %.1f us per iteration (first start -> last end), main-lane idle %.1f us over %d boundaries, "
           "ordering violations %d\n", mode == 0 ? "eager two-stream" : "lane graphs A/S/B", wall_sum / n, idle_sum / n,
           NM - 1, bad);
  }
  // calibration: the main lane alone (no side kernels), eager vs one linear graph
  hipGraph_t gM;
  hipGraphExec_t eM;
  CK(hipStreamBeginCapture(m, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < NM; ++i) hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, m, st, tk, i, 20000L);
  CK(hipStreamEndCapture(m, &gM));
  CK(hipGraphInstantiate(&eM, gM, nullptr, nullptr, 0));
  for (int mode = 0; mode < 2; ++mode) {
    double idle_sum = 0;
    int n = 0;
    for (int it = 0; it < 12; ++it) {
      CK(hipDeviceSynchronize());
      if (mode == 0)
        for (int i = 0; i < NM; ++i) hipLaunchKernelGGL(work, dim3(256), dim3(256), 0, m, st, tk, i, 20000L);
      else
        CK(hipGraphLaunch(eM, m));
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      if (it < 2) continue;
      double idle = 0;
      for (int i = 0; i + 1 < NM; ++i) idle += (double)(h[(i + 1) * 2] - h[i * 2 + 1]) * 10.0 / 1000.0;
      idle_sum += idle;
      ++n;
    }
    printf("main lane alone, %s: idle %.1f us over %d boundaries\n", mode == 0 ? "eager" : "one graph", idle_sum / n,
           NM - 1);
  }
  return 0;
}
