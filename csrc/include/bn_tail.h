// BatchNorm finalize fused into the tail of the kernel that produces the statistics (ResNet step engine).
//
// A statistics-producing kernel (conv forward: sum z, sum z^2; data-grad conv: sum dz, sum dz*xhat [, sum
// dz*xhat_d]) writes one partial row per M tile: stats[st][mt][Cout], columns [n0, n0 + BN) per workgroup.
// With a BnTail the same launch finishes the BatchNorm: a deterministic two-level last-arriver reduction over
// the M tiles of each column block, then the per-channel finalize (mean / rstd / scale / shift + running
// statistics, or the backward coefficients c1 / c2 and dgamma / dbeta) - replacing the two extra launches
// (partial + final reduce) and their two kernel boundaries that each BatchNorm cost per direction.
//
// Hand-off (MI355X guide, inter-workgroup visibility, row 1 of the sc1 hand-off table): partials are stored
// write-through (agent-scope relaxed atomic stores = global_store ... sc1) by every wave, drained with
// s_waitcnt vmcnt(0) before a workgroup barrier, then ONE lane takes an agent-scope ticket; the workgroup whose
// ticket is last reads the partials only with sc1 loads after its ticket returned (the other waves after a
// barrier).  No fences: valid for gfx950's sc1 lowering of relaxed agent-scope atomics (ecg_common.h refuses
// any other device target), measured as the guide's hand-off row 1 under load.  Level 1: the last arriver of each group of ``gs`` M tiles sums the group's rows (fp64)
// into ``gpart``; level 2: the last group reducer of the column block sums the group rows in group order and
// finalizes.  The summation order never depends on arrival order: bitwise reproducible.  The final reducer
// zeroes the block's counters for the next launch.
#pragma once

#include <stdint.h>

namespace ecg {

// One BatchNorm's finalize.  Every field is 8 bytes (packed by ops/resnet_engine.py).
struct BnFin {
  int64_t mode;   // 0: forward statistics -> mean/rstd/scale/shift (+running); 1: backward -> dgamma/dbeta/c1/c2
  int64_t statB;  // stat row of the second moment: fwd 1 (sum z^2); bwd 1 (sum dz*xhat) or 2 (sum dz*xhat_d)
  double n, eps, momentum;
  const float* gamma;
  const float* beta;
  float* mean;
  float* rstd;
  float* scale;  // gamma * rstd
  float* shift;  // beta - mean * scale
  float* run_mean;
  float* run_var;
  float* dgamma;
  float* dbeta;
  float* c1;  // sum dz / n
  float* c2;  // sum dz*xhat / n
};

struct BnTail {
  unsigned* counters;  // [Cout/64][NG + 1] (column block nt uses row nt), zero between launches
  double* gpart;       // [Cout/64][NG][3][64] level-1 group partials (row stride in doubles: NG * 3 * 64)
  int64_t gs;          // M tiles per level-1 group
  int64_t nfin;        // 1 or 2 BatchNorms finalized from the same statistics (data-grad conv + downsample); bits
                       // 8+: diagnostic early exit (scripts/conv_cold_probe.py): 1 after the level-1 ticket, 2 after
                       // the level-2 ticket (counters reset, nothing finalized), 3 after the level-2 loads - never
                       // set by the engine
  BnFin fin[2];
};

__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int c, double v1, double v2) {
  const double n = f.n;
  if (f.mode == 0) {
    const double mu = v1 / n;
    const double var = fmax(v2 / n - mu * mu, 0.0);
    const float rs = (float)(1.0 / sqrt(var + f.eps));
    const float sc = f.gamma[c] * rs;
    f.mean[c] = (float)mu;
    f.rstd[c] = rs;
    f.scale[c] = sc;
    f.shift[c] = f.beta[c] - (float)mu * sc;
    if (f.run_mean) {
      const float m = (float)f.momentum;
      f.run_mean[c] = (1.f - m) * f.run_mean[c] + m * (float)mu;
      f.run_var[c] = (1.f - m) * f.run_var[c] + m * (float)(var * n / fmax(n - 1.0, 1.0));
    }
  } else {
    if (f.dbeta) f.dbeta[c] = (float)v1;
    if (f.dgamma) f.dgamma[c] = (float)v2;
    f.c1[c] = (float)(v1 / n);
    f.c2[c] = (float)(v2 / n);
  }
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by EVERY thread of a statistics-producing workgroup after it stored its partial row (sc1) for M tile
// ``mt`` of column block ``nt`` (columns n0 .. n0 + BN, BN <= 256 and a multiple of 64).  ``lds``: >= 3 * 256
// doubles + 16 bytes of dead LDS.
template <int NTHR>
__device__ __forceinline__ void bn_tail(const BnTail* __restrict__ tp, const float* __restrict__ stats, int NS,
                                        int MT, int Cout, int mt, int n0, int BN, unsigned char* lds) {
  const int tid = threadIdx.x;
  int* flag = reinterpret_cast<int*>(lds);
  double* sums = reinterpret_cast<double*>(lds + 16);
  const int gs = (int)tp->gs;
  const int stop = (int)(tp->nfin >> 8);
  const int NG = (MT + gs - 1) / gs;
  const int g = mt / gs, members = min(gs, MT - g * gs);
  const int nb0 = n0 / 64, nblk = BN / 64;  // 64-column blocks of this workgroup
  // counters / group partials are kept per 64-column block so the host need not know the tile width: the
  // workgroup's blocks arrive together (one ticket on the first block's counter stands for all of them).
  unsigned* cnt = tp->counters + (long)nb0 * (NG + 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores have completed
  __syncthreads();
  if (tid == 0)
    flag[0] = __hip_atomic_fetch_add(&cnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(members - 1);
  __syncthreads();
  if (!flag[0]) return;
  if (stop == 1) {
    if (tid == 0) __hip_atomic_store(&cnt[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // ---- level 1: the group's rows, in row order, per (stat, column).  Every load of a batch (up to 32 rows) is
  // issued before the first add: one round trip per batch, not one per row.
  const long gstride = (long)NG * 3 * 64;  // doubles per 64-column block
  for (int p = tid; p < NS * BN; p += NTHR) {
    const int st = p / BN, c = p - st * BN;
    const float* src = stats + ((long)st * MT + g * gs) * Cout + n0 + c;
    double s = 0.0;
    for (int r0 = 0; r0 < members; r0 += 32) {
      float v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = ld_sc1(src + (long)min(r0 + u, members - 1) * Cout);  // clamped: no branch
#pragma unroll
      for (int u = 0; u < 32; ++u) s += r0 + u < members ? (double)v[u] : 0.0;
    }
    st_sc1(tp->gpart + (long)(nb0 + c / 64) * gstride + ((long)g * 3 + st) * 64 + (c & 63), s);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    flag[1] = __hip_atomic_fetch_add(&cnt[NG], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(NG - 1);
  __syncthreads();
  if (!flag[1]) return;
  if (stop == 2 || stop == 3) {
    for (int i = tid; i <= NG; i += NTHR) __hip_atomic_store(&cnt[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (stop == 2) return;
  }
  // ---- level 2: the group partials in group order (batches of 32 in flight), then the per-channel finalize
  for (int p = tid; p < NS * BN; p += NTHR) {
    const int st = p / BN, c = p - st * BN;
    const double* src = tp->gpart + (long)(nb0 + c / 64) * gstride + (long)st * 64 + (c & 63);
    double s = 0.0;
    for (int g0 = 0; g0 < NG; g0 += 32) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = ld_sc1(src + (long)min(g0 + u, NG - 1) * 3 * 64);
#pragma unroll
      for (int u = 0; u < 32; ++u) s += g0 + u < NG ? v[u] : 0.0;
    }
    sums[p] = s;
  }
  __syncthreads();
  if (stop == 3) return;
  for (int c = tid; c < BN; c += NTHR) {
    for (int f = 0; f < (int)(tp->nfin & 0xff); ++f) {
      const BnFin& fin = tp->fin[f];
      bn_fin_channel(fin, n0 + c, sums[c], sums[(int)fin.statB * BN + c]);
    }
  }
  for (int i = tid; i <= NG; i += NTHR) __hip_atomic_store(&cnt[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  (void)nblk;
}

}  // namespace ecg
