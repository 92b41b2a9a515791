// ResNet1D training-step engine for gfx950: channels-last (NLC) bf16 activations, fp32 master weights in one
// flat buffer, BatchNorm in training mode, and a native "step plan" executor that replays the whole
// forward + backward + SGD step as a list of kernel launches - eagerly or as ONE hipGraph.
//
// BASELINE.json config 5 ("Deeper ResNet1D-34 ECG, large-batch bf16 ... scaling stress").
// Not in the reference (its only model is TinyECG, Module_1/bench_locality.py:8-21); the conv kernels are the
// MFMA implicit GEMMs of conv1d_mc.hip, everything around them lives here:
//
//   stem      conv(1->64, k7, s2, p3) on VALU (C_in = 1 has no GEMM shape) with fused BN statistics,
//             BN + ReLU + MaxPool(3,2,1) in one pass; backward re-derives the pool argmax (no index tensor).
//   BN        statistics come out of the producing conv's epilogue (per-64-row-tile partials), a ticketed
//             finalize kernel reduces them (fp64) and emits scale/shift + running stats in ONE launch;
//             apply kernels fuse ReLU and the residual (identity or the downsample branch's own BN).
//   BN bwd    one reduce pass (sum dz, sum dz*xhat [, sum dz*xhat_ds]) + one apply pass; the identity
//             residual gradient is folded into the data-grad conv's epilogue (add * (out > 0)).
//   head      global average pool + Linear + softmax cross-entropy + its gradient, one block per sample, and
//             a deterministic split reduction for dW / db / loss.
//   weights   one launch converts every conv weight of the flat fp32 master buffer into the bf16 forward
//             layout [Cout][K][Cin] and the flipped data-grad layout [Cin][K][Cout].
//   SGD       the flat-buffer SGD kernel (fused_sgd.hip) over all parameters at once.
//
// All reductions have a fixed order: the step is bitwise deterministic for a given batch.
#include "../include/ecg_common.h"
#include <cstdlib>

#include "../include/bn_tail.h"

#include <algorithm>
#include <type_traits>

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

extern "C" int ecg_conv1d_nlc_fwd_ex(const void* x, const void* w, const float* bias, void* y, float* stats,
                                     const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout,
                                     int Cout, int Kw, int stride, int pad, int in_dil, int relu,
                                     const void* const* bnb, const void* tail, hipStream_t stream);
extern "C" int ecg_conv1d_nlc_fwd_pa(const void* x, const void* w, const float* bias, void* y, float* stats,
                                     const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout,
                                     int Cout, int Kw, int stride, int pad, int in_dil, int relu,
                                     const void* const* bnb, const void* tail, const void* const* pa,
                                     hipStream_t stream);
extern "C" int ecg_conv1d_nlc_wgrad(const void* dy, const void* x, float* part, int splits, int B, int Lin, int Cin,
                                    int Lout, int Cout, int Kw, int stride, int pad, hipStream_t stream);
extern "C" int ecg_sgd_flat(float* params, const float* grads, float* mom, long n, float lr, float momentum,
                            float dampening, float wd, int nesterov, int first, float inv_scale, int* found_inf,
                            hipStream_t stream);

namespace {

constexpr int TPB = 256;

__device__ __forceinline__ void ld8(const __bf16* p, float* f) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ void st8(__bf16* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (__bf16)f[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}
__device__ __forceinline__ void ldf8(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// ------------------------------------------------------------------------------------------------ stem
// y[b,t,c] = sum_k w[c,k] x[b, t*s + k - p].  Block = STEM_ROWS rows; thread = 8 channels (16-B stores) of one
// row per pass (8 channel groups x 32 row lanes); BN partials per block.  The block's input taps are staged in
// LDS first (thread r loads row r's <= 8 taps, all loads in flight together), so the block pays one global round
// trip instead of one per pass.
constexpr int STEM_ROWS = 256;
__global__ __launch_bounds__(TPB) void stem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       __bf16* __restrict__ y, float* __restrict__ stats, int B,
                                                       int L, int Lo, int K, int stride, int pad,
                                                       const ecg::BnTail* __restrict__ tail) {  // fused BN finalize
  static_assert(STEM_ROWS == TPB, "one staging row per thread");
  __shared__ float red[4][2][64];
  __shared__ __attribute__((aligned(16))) float xs[STEM_ROWS][8];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cg = tid & 7, rl = tid >> 3, c0 = cg * 8;
  const long M = (long)B * Lo;
  {
    const long m = (long)blockIdx.x * STEM_ROWS + tid;
    float xv[8];
    if (m < M) {
      const int b = (int)(m / Lo), t = (int)(m % Lo);
      const float* xb = x + (long)b * L;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int u = t * stride + k - pad;
        xv[k] = (k < K && u >= 0 && u < L) ? xb[min(max(u, 0), L - 1)] : 0.f;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) xv[k] = 0.f;
    }
    *reinterpret_cast<float4*>(&xs[tid][0]) = make_float4(xv[0], xv[1], xv[2], xv[3]);
    *reinterpret_cast<float4*>(&xs[tid][4]) = make_float4(xv[4], xv[5], xv[6], xv[7]);
  }
  float wk[8][8];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) wk[e][k] = k < K ? w[(c0 + e) * K + k] : 0.f;
  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = ss[e] = 0.f;
  __syncthreads();
#pragma unroll 2
  for (int i = 0; i < STEM_ROWS / 32; ++i) {
    const int r = rl + 32 * i;
    const long m = (long)blockIdx.x * STEM_ROWS + r;
    if (m >= M) break;
    const float4 xa = *reinterpret_cast<const float4*>(&xs[r][0]), xb4 = *reinterpret_cast<const float4*>(&xs[r][4]);
    const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb4.x, xb4.y, xb4.z, xb4.w};
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += wk[e][k] * xv[k];
      v[e] = (float)(__bf16)acc;
      s[e] += v[e];
      ss[e] += v[e] * v[e];
    }
    st8(y + m * 64 + c0, v);
  }
#pragma unroll
  for (int off = 8; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s[e] += __shfl_xor(s[e], off);
      ss[e] += __shfl_xor(ss[e], off);
    }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wv][0][c0 + e] = s[e];
      red[wv][1][c0 + e] = ss[e];
    }
  }
  __syncthreads();
  if (tid < 128) {
    const int st = tid >> 6, c = tid & 63;
    const float v = red[0][st][c] + red[1][st][c] + red[2][st][c] + red[3][st][c];
    if (tail)
      ecg::st_sc1(&stats[((long)st * gridDim.x + blockIdx.x) * 64 + c], v);  // handed to the tail's last arriver
    else
      stats[((long)st * gridDim.x + blockIdx.x) * 64 + c] = v;
  }
  if (tail)  // the staging rows are dead: 8 KB of LDS for the tail's scratch
    ecg::bn_tail<TPB>(tail, stats, 2, gridDim.x, 64, blockIdx.x, 0, 64, reinterpret_cast<unsigned char*>(&xs[0][0]));
}

// out[b,o,c] = max_{j in {2o-1,2o,2o+1}} relu(z[b,j,c]*scale[c] + shift[c])   (MaxPool1d(3, 2, 1)); am[b,o,c]
// (optional) = j - (2o-1) of the first maximum, for the backward
__global__ __launch_bounds__(TPB) void stem_pool_kernel(const __bf16* __restrict__ z, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, __bf16* __restrict__ out,
                                                        uint8_t* __restrict__ am, int B, int Lz, int Lp, int C) {
  const int cg = C / 8;
  const long nv = (long)B * Lp * cg;
  for (long v = (long)blockIdx.x * TPB + threadIdx.x; v < nv; v += (long)gridDim.x * TPB) {
    const int c0 = (int)(v % cg) * 8;
    const long bo = v / cg;
    const int o = (int)(bo % Lp), b = (int)(bo / Lp);
    float sc[8], sh[8], mx[8];
    uint32_t ix[8];
    ldf8(scale + c0, sc);
    ldf8(shift + c0, sh);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mx[i] = -INFINITY;
      ix[i] = 0u;
    }
#pragma unroll
    for (int d = -1; d <= 1; ++d) {
      const int j = 2 * o + d;
      if (j < 0 || j >= Lz) continue;
      float zf[8];
      ld8(z + ((long)b * Lz + j) * C + c0, zf);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float av = fmaxf(zf[i] * sc[i] + sh[i], 0.f);
        if (av > mx[i]) {  // strict: the first maximum wins (the order the backward has always used)
          mx[i] = av;
          ix[i] = (uint32_t)(d + 1);
        }
      }
    }
    st8(out + bo * C + c0, mx);
    if (am) {
      uint2 w;
      w.x = ix[0] | ix[1] << 8 | ix[2] << 16 | ix[3] << 24;
      w.y = ix[4] | ix[5] << 8 | ix[6] << 16 | ix[7] << 24;
      *reinterpret_cast<uint2*>(am + bo * C + c0) = w;
    }
  }
}

// Backward of ReLU(BN(z)) -> MaxPool: dz[b,j,c] = (a_j > 0) * sum_{windows o whose first argmax is j} gp[b,o,c]
// (written bf16) and BN partials sum(dz), sum(dz * xhat) per block of rows.  The argmax comes from the forward
// (stem_pool_kernel's ``am``, as PyTorch's max_pool1d backward uses the forward's indices): one z row per output
// row instead of recomputing both windows from five (round 4: 3.363-3.370 vs 3.369-3.377 ms/step, r4_stemam1).
__global__ __launch_bounds__(TPB) void stem_bwd_reduce_kernel(
    const __bf16* __restrict__ gp, const __bf16* __restrict__ z, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ rstd,
    __bf16* __restrict__ dz, float* __restrict__ part, int B, int Lz, int Lp, int C, int chunk,
    const ecg::BnTail* __restrict__ tail,  // tail: the stem BatchNorm's backward finalize fused here, or null
    const uint8_t* __restrict__ am) {      // am: the forward's argmax per pooled output (stem_pool_kernel)
  __shared__ __attribute__((aligned(16))) float red[TPB * 16];
  const int cg = C / 8, tid = threadIdx.x;
  const int rpp = TPB / cg, roff = tid / cg, c0 = (tid % cg) * 8;
  const bool active = roff < rpp;  // C/8 need not divide the block: spare threads idle
  const long R = (long)B * Lz;
  float sc[8], sh[8], mu[8], rs[8], a1[8], a2[8];
  ldf8(scale + c0, sc);
  ldf8(shift + c0, sh);
  ldf8(mean + c0, mu);
  ldf8(rstd + c0, rs);
#pragma unroll
  for (int i = 0; i < 8; ++i) a1[i] = a2[i] = 0.f;
  const long r1 = active ? min(R, (long)(blockIdx.x + 1) * chunk) : 0;
  for (long r = (long)blockIdx.x * chunk + roff; r < r1; r += rpp) {
    const int b = (int)(r / Lz), j = (int)(r % Lz);
    // the windows containing j are o0 = j>>1 (rows p0 .. p0+2, p0 = 2*o0 - 1) and, for odd j, o1 = o0 + 1 (rows
    // j .. j+2): row j is window o0's first maximum when am = 1 + (j & 1), window o1's when am = 0.  All loads are
    // issued from clamped addresses, validity applied to the values.
    const int o0 = j >> 1, o1 = (j + 1) >> 1;
    const bool has1 = o1 != o0 && o1 < Lp;
    float zj[8], g0[8], g1[8];
    ld8(z + ((long)b * Lz + j) * C + c0, zj);
    ld8(gp + ((long)b * Lp + o0) * C + c0, g0);
    ld8(gp + ((long)b * Lp + min(o1, Lp - 1)) * C + c0, g1);
    const uint2 a0 = *reinterpret_cast<const uint2*>(am + ((long)b * Lp + o0) * C + c0);
    const uint2 a1w = *reinterpret_cast<const uint2*>(am + ((long)b * Lp + min(o1, Lp - 1)) * C + c0);
    const uint32_t want0 = 1u + (uint32_t)(j & 1);
    float d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t m0 = ((i < 4 ? a0.x : a0.y) >> (8 * (i & 3))) & 0xffu;
      const uint32_t m1 = ((i < 4 ? a1w.x : a1w.y) >> (8 * (i & 3))) & 0xffu;
      float gi = m0 == want0 ? g0[i] : 0.f;
      if (has1 && m1 == 0u) gi += g1[i];
      const float av = zj[i] * sc[i] + sh[i];
      d[i] = av > 0.f ? gi : 0.f;
    }
    st8(dz + r * C + c0, d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float dv = (float)(__bf16)d[i];
      a1[i] += dv;
      a2[i] += dv * (zj[i] - mu[i]) * rs[i];
    }
  }
  // reduce over the rpp row groups: red[roff][stat][c]
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(roff * 2 + 0) * C + c0 + i] = a1[i];
      red[(roff * 2 + 1) * C + c0 + i] = a2[i];
    }
  }
  __syncthreads();
  const int T = gridDim.x;
  for (int idx = tid; idx < 2 * C; idx += TPB) {
    const int st = idx / C, c = idx % C;
    float v = 0.f;
    for (int q = 0; q < rpp; ++q) v += red[(q * 2 + st) * C + c];
    if (tail)
      ecg::st_sc1(&part[((long)st * T + blockIdx.x) * C + c], v);  // handed to the tail's last arriver
    else
      part[((long)st * T + blockIdx.x) * C + c] = v;
  }
  if (tail) ecg::bn_tail<TPB>(tail, part, 2, T, C, blockIdx.x, 0, C, reinterpret_cast<unsigned char*>(red));
}

// dW[c,k] partials: sum over rows of dzz[b,j,c] * x[b, j*s + k - p], dzz = scale*(dz - c1 - xhat*c2).
// Thread = 8 channels (16-B loads) x all taps of one row per pass; 8 channel groups x 32 row lanes per block.
__global__ __launch_bounds__(TPB) void stem_wgrad_kernel(
    const __bf16* __restrict__ dz, const __bf16* __restrict__ z, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ scale, const float* __restrict__ c1,
    const float* __restrict__ c2, const float* __restrict__ x, float* __restrict__ part, int B, int L, int Lz, int K,
    int stride, int pad, int chunk) {
  __shared__ float red[4][64 * 8];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cg = tid & 7, rl = tid >> 3, c0 = cg * 8;
  float mu[8], rs[8], sc[8], k1[8], k2[8], acc[8][8];
  ldf8(mean + c0, mu);
  ldf8(rstd + c0, rs);
  ldf8(scale + c0, sc);
  ldf8(c1 + c0, k1);
  ldf8(c2 + c0, k2);
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[e][k] = 0.f;
  const long R = (long)B * Lz;
  const long r1 = min(R, (long)(blockIdx.x + 1) * chunk);
  for (long r = (long)blockIdx.x * chunk + rl; r < r1; r += 32) {
    const int b = (int)(r / Lz), j = (int)(r % Lz);
    float dv[8], zv[8], xv[8];
    ld8(dz + r * 64 + c0, dv);
    ld8(z + r * 64 + c0, zv);
    const float* xb = x + (long)b * L;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int u = j * stride + k - pad;
      xv[k] = (k < K && u >= 0 && u < L) ? xb[u] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = sc[e] * (dv[e] - k1[e] - (zv[e] - mu[e]) * rs[e] * k2[e]);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[e][k] += g * xv[k];
    }
  }
#pragma unroll
  for (int off = 8; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[e][k] += __shfl_xor(acc[e][k], off);
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[wv][(c0 + e) * 8 + k] = acc[e][k];
  }
  __syncthreads();
  for (int idx = tid; idx < 64 * K; idx += TPB) {
    const int cc = idx / K, k = idx % K;
    part[(long)blockIdx.x * 64 * K + idx] =
        red[0][cc * 8 + k] + red[1][cc * 8 + k] + red[2][cc * 8 + k] + red[3][cc * 8 + k];
  }
}

// ------------------------------------------------------------------------------------------------ BatchNorm
struct FinArgs {
  const float* sA;  // [T][C] partials of stat A (fwd: sum x; bwd: sum dz)
  const float* sB;  // [T][C] partials of stat B (fwd: sum x^2; bwd: sum dz*xhat)
  int T, C, mode;   // mode 0 = forward statistics, 1 = backward coefficients
  double* scratch;  // [gridDim.y][2][C]
  float n, eps, momentum;
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

__device__ __forceinline__ void bn_fin_outputs(const FinArgs& a, int c, double v1, double v2) {
  const double n = (double)a.n;
  if (a.mode == 0) {
    const double mu = v1 / n;
    const double var = fmax(v2 / n - mu * mu, 0.0);
    const float rs = (float)(1.0 / sqrt(var + (double)a.eps));
    const float sc = a.gamma[c] * rs;
    a.mean[c] = (float)mu;
    a.rstd[c] = rs;
    a.scale[c] = sc;
    a.shift[c] = a.beta[c] - (float)mu * sc;
    if (a.run_mean) {
      const float m = a.momentum;
      a.run_mean[c] = (1.f - m) * a.run_mean[c] + m * (float)mu;
      a.run_var[c] = (1.f - m) * a.run_var[c] + m * (float)(var * n / fmax(n - 1.0, 1.0));
    }
  } else {
    if (a.dbeta) a.dbeta[c] = (float)v1;
    if (a.dgamma) a.dgamma[c] = (float)v2;
    a.c1[c] = (float)(v1 / n);
    a.c2[c] = (float)(v2 / n);
  }
}

// One launch: a 1024-thread block per 64 channels sums the T partial rows of both statistics (16 row groups x 64
// channels; each thread's rows t = rg, rg + 16, ... issued 16 at a time, so T <= 256 is ONE memory round trip),
// combines the row groups in a fixed order (fp64, bitwise reproducible) and finalizes.  The producing conv stores
// its partial rows with plain stores; the kernel boundary makes them visible.
__global__ __launch_bounds__(1024) void bn_fin1_kernel(FinArgs a) {
  __shared__ double red[16][2][64];
  const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  for (int t0 = rg; t0 < a.T; t0 += 16 * 16) {
    float v1[16], v2[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int t = min(t0 + 16 * u, a.T - 1);  // clamped: no branch, the extra rows are not added
      v1[u] = a.sA[(long)t * a.C + c];
      v2[u] = a.sB[(long)t * a.C + c];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (t0 + 16 * u < a.T) {
        s1 += (double)v1[u];
        s2 += (double)v2[u];
      }
  }
  red[rg][0][cl] = s1;
  red[rg][1][cl] = s2;
  __syncthreads();
  if (tid < 64) {
    double v1 = 0.0, v2 = 0.0;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      v1 += red[g][0][cl];
      v2 += red[g][1][cl];
    }
    bn_fin_outputs(a, c, v1, v2);
  }
}

// MODE 0: out = relu(z*scale + shift); 1: out = relu(z*scale + shift + res); 2: + (zd*scale_d + shift_d).
// mbits (optional): the ReLU mask of out as one byte per 8-channel vector (bit e: out[e] > 0) - the backward's
// data-grad epilogue reads it instead of out (FwdArgs::smask_bits: 1/16 of the bytes).
template <int MODE>
__global__ __launch_bounds__(TPB) void bn_act_kernel(const __bf16* __restrict__ z, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, const __bf16* __restrict__ res,
                                                     const float* __restrict__ scale_d,
                                                     const float* __restrict__ shift_d, __bf16* __restrict__ out,
                                                     long R, int C, uint8_t* __restrict__ mbits) {
  const int cg = C / 8;
  const long nv = R * cg;
  int cur = -1;  // the thread's channel group, fixed under bn_pass_grid: coefficients loaded once
  float sc[8], sh[8], sd[8], hd[8];
  for (long v = (long)blockIdx.x * TPB + threadIdx.x; v < nv; v += (long)gridDim.x * TPB) {
    const int c0 = (int)(v % cg) * 8;
    const long o = v * 8;
    float zf[8], y[8], rf[8];
    ld8(z + o, zf);
    if (MODE >= 1) ld8(res + o, rf);
    if (c0 != cur) {
      cur = c0;
      ldf8(scale + c0, sc);
      ldf8(shift + c0, sh);
      if (MODE == 2) {
        ldf8(scale_d + c0, sd);
        ldf8(shift_d + c0, hd);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = fmaf(zf[i], sc[i], sh[i]);  // (the data-grad epilogue's mask re-derives it)
    if (MODE >= 1) {
      if (MODE == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) rf[i] = rf[i] * sd[i] + hd[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] += rf[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) y[i] = fmaxf(y[i], 0.f);
    st8(out + o, y);
    if (mbits) {
      unsigned mb = 0u;
#pragma unroll
      for (int i = 0; i < 8; ++i) mb |= ((float)(__bf16)y[i] > 0.f ? 1u : 0u) << i;  // the stored value's sign
      mbits[v] = (uint8_t)mb;
    }
  }
}

// dz = gy * (mask_src > 0); partial sums of dz, dz*xhat (and dz*xhat_d when NS == 3) per block of rows.
template <int NS>
__global__ __launch_bounds__(TPB) void bn_bwd_reduce_kernel(
    const __bf16* __restrict__ gy, const __bf16* __restrict__ msk, const __bf16* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ rstd, const __bf16* __restrict__ zd,
    const float* __restrict__ mean_d, const float* __restrict__ rstd_d, float* __restrict__ part, long R, int C,
    int chunk, __bf16* __restrict__ dzm, const ecg::BnTail* __restrict__ tail) {  // tail: fused finalize(s) or null
  __shared__ __attribute__((aligned(16))) float red[TPB * 8 * 3];
  const int cg = C / 8, tid = threadIdx.x;
  const int rpp = TPB / cg, roff = tid / cg, c0 = (tid % cg) * 8;
  const bool active = roff < rpp;
  float mu[8], rs[8], mud[8], rsd[8], a1[8], a2[8], a3[8];
  ldf8(mean + c0, mu);
  ldf8(rstd + c0, rs);
  if (NS == 3) {
    ldf8(mean_d + c0, mud);
    ldf8(rstd_d + c0, rsd);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) a1[i] = a2[i] = a3[i] = 0.f;
  const long r1 = active ? min(R, (long)(blockIdx.x + 1) * chunk) : 0;
  for (long r = (long)blockIdx.x * chunk + roff; r < r1; r += rpp) {
    const long o = r * C + c0;
    float g[8], m[8], zf[8];
    ld8(gy + o, g);
    ld8(msk + o, m);
    ld8(z + o, zf);
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = m[i] > 0.f ? g[i] : 0.f;
    if (dzm) {  // optional masked copy (the block's ReLU-backward output, consumed by the apply/dgrad ops)
      st8(dzm + o, g);
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (float)(__bf16)g[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = g[i];
      a1[i] += d;
      a2[i] += d * (zf[i] - mu[i]) * rs[i];
    }
    if (NS == 3) {
      float zdf[8];
      ld8(zd + o, zdf);
#pragma unroll
      for (int i = 0; i < 8; ++i) a3[i] += g[i] * (zdf[i] - mud[i]) * rsd[i];
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(roff * NS + 0) * C + c0 + i] = a1[i];
      red[(roff * NS + 1) * C + c0 + i] = a2[i];
      if (NS == 3) red[(roff * NS + 2) * C + c0 + i] = a3[i];
    }
  }
  __syncthreads();
  const int T = gridDim.x;
  for (int idx = tid; idx < NS * C; idx += TPB) {
    const int st = idx / C, c = idx % C;
    float v = 0.f;
    for (int q = 0; q < rpp; ++q) v += red[(q * NS + st) * C + c];
    if (tail)
      ecg::st_sc1(&part[((long)st * T + blockIdx.x) * C + c], v);  // handed to the tail's last arriver
    else
      part[((long)st * T + blockIdx.x) * C + c] = v;
  }
  if (tail) {  // every column block of C (64 wide) is finalized by this launch's tail
    for (int n0 = 0; n0 < C; n0 += 256) {
      const int bn = C - n0 < 256 ? C - n0 : 256;
      ecg::bn_tail<TPB>(tail, part, NS, T, C, blockIdx.x, n0, bn, reinterpret_cast<unsigned char*>(red));
    }
  }
}

// dzz = scale*(dz - c1 - xhat*c2) with dz = gy*(mask > 0); DS: also dzd = scale_d*(dz - c1 - xhat_d*c2_d).
// Grid-stride with a stride that is a multiple of C/8 (bn_pass_grid), so a thread's channel group is the same in
// every iteration: its per-channel coefficients are loaded ONCE (the one-vector-per-thread form re-read 5 coefficient
// vectors - 160 B of L1/L2 traffic - per 16-B element vector: 4.4-4.5 TB/s of tensor traffic at the B=1024 stage
// shapes against 8 TB/s for a plain copy, scripts/r4_bn_probe.py).  Same expression, bitwise the same output.
template <bool DS>
__global__ __launch_bounds__(TPB) void bn_bwd_apply_kernel(
    const __bf16* __restrict__ gy, const __bf16* __restrict__ msk, const __bf16* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ scale,
    const float* __restrict__ c1, const float* __restrict__ c2, __bf16* __restrict__ out,
    const __bf16* __restrict__ zd, const float* __restrict__ mean_d, const float* __restrict__ rstd_d,
    const float* __restrict__ scale_d, const float* __restrict__ c2_d, __bf16* __restrict__ out_d, long R, int C) {
  const int cg = C / 8;
  const long nv = R * cg;
  int cur = -1;
  float mu[8], rs[8], sc[8], k1[8], k2[8], mud[8], rsd[8], scd[8], k2d[8];
  for (long v = (long)blockIdx.x * TPB + threadIdx.x; v < nv; v += (long)gridDim.x * TPB) {
    const int c0 = (int)(v % cg) * 8;
    const long o = v * 8;
    float g[8], zf[8], y[8];
    ld8(gy + o, g);
    ld8(z + o, zf);
    if (DS) ld8(zd + o, y);  // (y holds zd until the first output is computed)
    if (c0 != cur) {  // first iteration (and any grid whose stride is not a multiple of C/8)
      cur = c0;
      ldf8(mean + c0, mu);
      ldf8(rstd + c0, rs);
      ldf8(scale + c0, sc);
      ldf8(c1 + c0, k1);
      ldf8(c2 + c0, k2);
      if (DS) {
        ldf8(mean_d + c0, mud);
        ldf8(rstd_d + c0, rsd);
        ldf8(scale_d + c0, scd);
        ldf8(c2_d + c0, k2d);
      }
    }
    if (msk) {
      float m[8];
      ld8(msk + o, m);
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = m[i] > 0.f ? g[i] : 0.f;
    }
    float zdv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      zdv[i] = y[i];
      y[i] = sc[i] * (g[i] - k1[i] - (zf[i] - mu[i]) * rs[i] * k2[i]);
    }
    st8(out + o, y);
    if (DS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = scd[i] * (g[i] - k1[i] - (zdv[i] - mud[i]) * rsd[i] * k2d[i]);
      st8(out_d + o, y);
    }
  }
}

// Grid of the per-element BatchNorm passes: enough 256-thread blocks for ~4 element vectors per thread (capped at
// 8 resident blocks per CU) and a thread count that is a multiple of C/8, so each thread keeps one channel group.
inline unsigned bn_pass_grid(long R, int C) {
  const long nv = R * (C / 8);
  long g = (nv + 4L * TPB - 1) / (4L * TPB);
  if (g < 256) g = std::min<long>(256, (nv + TPB - 1) / TPB);
  if (g > 2048) g = 2048;
  return (unsigned)std::max<long>(1, g);
}

// ------------------------------------------------------------------------------------------------ head
// One block per sample: feat = mean_t h[b,t,:]; logits = W feat + bias; CE loss; g = (softmax - onehot)/B;
// gh[b,t,c] = (W^T g)[c] / Lf.  Stores g, feat and loss/B for the split reduction.  Thread = 8 channels (16-byte
// loads / stores) x one of TPB / (C/8) row groups; the row groups' sums are combined in a fixed order (17.7 -> 13.7
// us per ResNet1D-34 B=1024 step against one channel per thread with 2-byte loads, profiles/r5/stem_head_ab.txt).
constexpr int MAXC = 16;
__global__ __launch_bounds__(TPB) void head_fwd_bwd_kernel(const __bf16* __restrict__ h, const float* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const int* __restrict__ labels, __bf16* __restrict__ gh,
                                                           float* __restrict__ gbuf, float* __restrict__ fbuf,
                                                           float* __restrict__ lbuf, int B, int Lf, int C, int ncls) {
  __shared__ __attribute__((aligned(16))) float part[TPB * 8];  // [row group][C] partial sums, then the gh row
  __shared__ float feat[1024];
  __shared__ float wred[TPB / 64][MAXC];
  __shared__ float gs[MAXC];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ncg = C / 8, nrg = TPB / ncg, cg = tid % ncg, rg = tid / ncg;
  const bool act = rg < nrg;
  const __bf16* hb = h + (long)b * Lf * C;
  const float invL = 1.f / (float)Lf;
  if (act) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t = rg; t < Lf; t += nrg) {
      float v[8];
      ld8(hb + (long)t * C + cg * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[rg * C + cg * 8 + e] = s[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += TPB) {
    float s = 0.f;
    for (int q = 0; q < nrg; ++q) s += part[q * C + c];
    s *= invL;
    feat[c] = s;
    fbuf[(long)b * C + c] = s;
  }
  __syncthreads();
  for (int j = 0; j < ncls; ++j) {
    float p = 0.f;
    for (int c = tid; c < C; c += TPB) p += W[(long)j * C + c] * feat[c];
    p = ecg::wave_sum(p);
    if (lane == 0) wred[wv][j] = p;
  }
  __syncthreads();
  if (tid == 0) {
    float lg[MAXC], mx = -INFINITY;
    for (int j = 0; j < ncls; ++j) {
      float v = bias[j];
      for (int q = 0; q < TPB / 64; ++q) v += wred[q][j];
      lg[j] = v;
      mx = fmaxf(mx, v);
    }
    float se = 0.f;
    for (int j = 0; j < ncls; ++j) se += expf(lg[j] - mx);
    const int y = labels[b];
    const float lse = mx + logf(se);
    lbuf[b] = (lse - lg[y]) / (float)B;
    for (int j = 0; j < ncls; ++j) {
      const float g = (expf(lg[j] - lse) - (j == y ? 1.f : 0.f)) / (float)B;
      gs[j] = g;
      gbuf[(long)b * ncls + j] = g;
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += TPB) {
    float d = 0.f;
    for (int j = 0; j < ncls; ++j) d += gs[j] * W[(long)j * C + c];
    part[c] = (float)(__bf16)(d * invL);
  }
  __syncthreads();
  if (act) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = part[cg * 8 + e];
    for (int t = rg; t < Lf; t += nrg) st8(gh + ((long)b * Lf + t) * C + cg * 8, v);
  }
}

// partial[gb][j*C + c] = sum_{b in slice} g[b,j] feat[b,c]; [ncls*C + j] = sum g[b,j]; [ncls*C + ncls] = sum loss
__global__ __launch_bounds__(TPB) void head_reduce_kernel(const float* __restrict__ gbuf,
                                                          const float* __restrict__ fbuf,
                                                          const float* __restrict__ lbuf, float* __restrict__ part,
                                                          int B, int C, int ncls) {
  __shared__ float red[4][64][MAXC + 1];
  const int tid = threadIdx.x, cl = tid & 63, g4 = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int Gb = gridDim.y;
  const int b0 = (int)((long)B * blockIdx.y / Gb), b1 = (int)((long)B * (blockIdx.y + 1) / Gb);
  float acc[MAXC + 1];
#pragma unroll
  for (int j = 0; j <= MAXC; ++j) acc[j] = 0.f;
  const bool extra = blockIdx.x == 0 && cl < 1;
#pragma unroll 8  // the rows' loads in flight together (15.7 -> 13.4 us, profiles/r5/stem_head_ab.txt)
  for (int b = b0 + g4; b < b1; b += 4) {
    const float f = c < C ? fbuf[(long)b * C + c] : 0.f;
#pragma unroll
    for (int j = 0; j < MAXC; ++j)
      if (j < ncls) acc[j] += gbuf[(long)b * ncls + j] * f;
    if (extra) acc[MAXC] += lbuf[b];
  }
#pragma unroll
  for (int j = 0; j <= MAXC; ++j) red[g4][cl][j] = acc[j];
  __syncthreads();
  const long N = (long)ncls * C + ncls + 1;
  float* out = part + (long)blockIdx.y * N;
  if (tid < 64 && c < C) {
    for (int j = 0; j < ncls; ++j)
      out[(long)j * C + c] = red[0][cl][j] + red[1][cl][j] + red[2][cl][j] + red[3][cl][j];
  }
  if (blockIdx.x == 0 && tid < ncls + 1) {  // db[j] = sum_b g[b,j] (own pass: tiny), loss
    float v = 0.f;
    if (tid < ncls) {
#pragma unroll 8
      for (int b = b0; b < b1; ++b) v += gbuf[(long)b * ncls + tid];
    } else {
      v = red[0][0][MAXC] + red[1][0][MAXC] + red[2][0][MAXC] + red[3][0][MAXC];
    }
    out[(long)ncls * C + tid] = v;
  }
}

// ------------------------------------------------------------------------------------------------ reductions
// out[i] = sum_s part[s*N + i] for i < split; out2[i - split] += sum for i >= split (accumulating tail).
// Block = 64 columns x 16 split groups (1024 threads), 4 loads in flight per thread, fixed-order LDS combine.
constexpr int RS_GROUPS = 16;
__global__ __launch_bounds__(64 * RS_GROUPS) void reduce_sum_kernel(const float* __restrict__ part, int S, long N,
                                                                    float* __restrict__ out, long split,
                                                                    float* __restrict__ out2) {
  __shared__ float red[RS_GROUPS][64];
  const int col = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + col;
  float v = 0.f;
  if (i < N) {
    int s = sg;
    for (; s + 3 * RS_GROUPS < S; s += 4 * RS_GROUPS) {
      float t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = part[(long)(s + u * RS_GROUPS) * N + i];
      v += (t[0] + t[1]) + (t[2] + t[3]);
    }
    for (; s < S; s += RS_GROUPS) v += part[(long)s * N + i];
  }
  red[sg][col] = v;
  __syncthreads();
  if (sg == 0 && i < N) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < RS_GROUPS; ++q) r += red[q][col];
    if (i < split) out[i] = r;
    else out2[i - split] += r;
  }
}

// grad[co][ci][k] = sum_s part[s][co][k*Cin + ci]  (nn.Conv1d weight layout).  Block = 64 float4 columns of
// the source layout x 4 split groups (coalesced 16-B loads, 4 independent chains), reduced through LDS, then
// scattered into the parameter layout.  N = Cout*K*Cin is a multiple of 4096 (C_in, C_out % 64 == 0).
__global__ __launch_bounds__(TPB) void reduce_wgrad_kernel(const float* __restrict__ part, int S, int Cout, int K,
                                                           int Cin, float* __restrict__ grad) {
  __shared__ float4 red[4][64];
  const long N = (long)Cout * K * Cin;
  const int tid = threadIdx.x, col = tid & 63, sg = tid >> 6;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const long N4 = N / 4;
  // grid-stride over 64-column groups
  for (long blk = blockIdx.x; blk * 64 < N4; blk += gridDim.x) {
  const long i4 = blk * 64 + col;  // float4 index
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < N4) {
    int s = sg;
    for (; s + 12 < S; s += 16) {
      float4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = p4[(long)(s + 4 * u) * N4 + i4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += t[u].x; acc.y += t[u].y; acc.z += t[u].z; acc.w += t[u].w;
      }
    }
    for (; s < S; s += 4) {
      const float4 t = p4[(long)s * N4 + i4];
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
  }
  red[sg][col] = acc;
  __syncthreads();
  if (sg == 0 && i4 < N4) {
    float4 v = red[0][col];
    for (int q = 1; q < 4; ++q) {
      v.x += red[q][col].x; v.y += red[q][col].y; v.z += red[q][col].z; v.w += red[q][col].w;
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long src = i4 * 4 + e;  // = co*K*Cin + k*Cin + ci
      const int ci = (int)(src % Cin);
      const long r = src / Cin;
      const int k = (int)(r % K), co = (int)(r / K);
      grad[((long)co * Cin + ci) * K + k] = vv[e];
    }
  }
  __syncthreads();  // red[] is rewritten by the next column group
  }
}

// Same sum, for the tap-shared weight gradient's many-split partials (S up to 256 x 48 KB slabs): block = 16 float4
// columns x 16 split groups, each thread's loads of a 16-split batch in flight together (one memory round trip per
// 256 splits), fixed summation order (bitwise reproducible); 16x the blocks of reduce_wgrad_kernel for a small |dW|.
__global__ __launch_bounds__(TPB) void reduce_wgrad_wide_kernel(const float* __restrict__ part, int S, int Cout, int K,
                                                                int Cin, float* __restrict__ grad) {
  __shared__ float4 red[16][17];
  const long N = (long)Cout * K * Cin, N4 = N / 4;
  const int tid = threadIdx.x, col = tid & 15, sg = tid >> 4;
  const long i4 = (long)blockIdx.x * 16 + col;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < N4) {
    int s = sg;
    for (; s + 16 * 15 < S; s += 256) {
      float4 t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = p4[(long)(s + 16 * u) * N4 + i4];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        acc.x += t[u].x; acc.y += t[u].y; acc.z += t[u].z; acc.w += t[u].w;
      }
    }
    for (; s + 16 * 3 < S; s += 64) {
      float4 t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = p4[(long)(s + 16 * u) * N4 + i4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += t[u].x; acc.y += t[u].y; acc.z += t[u].z; acc.w += t[u].w;
      }
    }
    for (; s < S; s += 16) {
      const float4 t = p4[(long)s * N4 + i4];
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
  }
  red[sg][col] = acc;
  __syncthreads();
  if (tid < 64) {  // 16 columns x 4 elements: one output element per thread
    const int c = tid >> 2, e = tid & 3;
    const long i = ((long)blockIdx.x * 16 + c) * 4 + e;  // = co*K*Cin + k*Cin + ci
    if (i < N) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float4 r = red[g][c];
        v += e == 0 ? r.x : e == 1 ? r.y : e == 2 ? r.z : r.w;
      }
      const int ci = (int)(i % Cin);
      const long rk = i / Cin;
      const int k = (int)(rk % K), co = (int)(rk / K);
      grad[((long)co * Cin + ci) * K + k] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------ data
// Batch staging inside the step graph: the step index comes from a device counter, so one captured step is
// replayed for every batch of a round; the index table [S][B] is refilled in place between rounds.
__global__ __launch_bounds__(TPB) void gather_step_kernel(const float* __restrict__ X, long ldx,
                                                          const int* __restrict__ Y, const int* __restrict__ table,
                                                          const int* __restrict__ counter, int S, int B, int L,
                                                          float* __restrict__ out_x, int* __restrict__ out_y) {
  const int b = blockIdx.x;
  const int step = *counter % S;
  const long row = table[(long)step * B + b];
  const float* src = X + row * ldx;
  float* dst = out_x + (long)b * L;
  for (int i = threadIdx.x; i < L; i += TPB) dst[i] = src[i];
  if (threadIdx.x == 0) out_y[b] = Y[row];
}

__global__ void counter_inc_kernel(int* counter) { *counter += 1; }

// ------------------------------------------------------------------------------------------------ weights
struct WEntry {
  long src;  // offset (elements) of the fp32 [Cout][Cin][K] weight in the flat buffer
  long wf;   // offset of the bf16 [Cout][K][Cin] copy
  long wb;   // offset of the bf16 [Cin][K][Cout] flipped copy (data-grad)
  int Cout, Cin, K, block0;  // block0: first 64x64 (Cout x Cin) tile of this conv in the launch
};

// Both bf16 layouts of every conv weight from the fp32 master copy, one 64 (Cout) x 64 (Cin) tile per workgroup:
// the tile's source rows (64 x Cin-slice x K floats, contiguous per output channel) are read with 16-byte loads,
// converted once into an LDS image [k][co][ci], and both destinations are written as whole 16-byte runs -
// [Cout][K][Cin] along ci and the flipped [Cin][K][Cout] along co (the transpose happens in LDS).  (Was one
// element per thread with two scattered 2-byte stores and a serial entry scan: 46 us per ResNet1D-34 step.)
constexpr int WP_LD = 64 + 8;  // bf16 per LDS row (16-byte pad: conflict-free column reads)

__global__ __launch_bounds__(TPB) void weight_prep_kernel(const WEntry* __restrict__ tab, int n,
                                                          const float* __restrict__ flat, __bf16* __restrict__ arena) {
  __shared__ int sel;
  __shared__ __attribute__((aligned(16))) __bf16 img[3 * 64 * WP_LD];  // [k][co][ci], K <= 3
  const int tid = threadIdx.x;
  if (tid < n) {  // every entry checks its own tile range (one pass, no serial scan)
    const int b0 = tab[tid].block0, b1 = tid + 1 < n ? tab[tid + 1].block0 : 0x7fffffff;
    if ((int)blockIdx.x >= b0 && (int)blockIdx.x < b1) sel = tid;
  }
  __syncthreads();
  const WEntry e = tab[sel];
  const int K = e.K, tci_n = e.Cin / 64;
  const int t = (int)blockIdx.x - e.block0;
  const int co0 = (t / tci_n) * 64, ci0 = (t % tci_n) * 64;
  // source: row co (64 of them) holds 64*K consecutive floats [ci][k] starting at ci0*K
  const int row_f = 64 * K, row_v = row_f / 4;  // floats / float4 per row (K=1: 16, K=3: 48)
  for (int v = tid; v < 64 * row_v; v += TPB) {
    const int co = v / row_v, q = v - co * row_v;
    const float4 f = *reinterpret_cast<const float4*>(flat + e.src + ((long)(co0 + co) * e.Cin + ci0) * K + 4 * q);
    const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int idx = 4 * q + j, ci = idx / K, k = idx - ci * K;
      img[(k * 64 + co) * WP_LD + ci] = (__bf16)fv[j];
    }
  }
  __syncthreads();
  // [Cout][K][Cin]: row (co, k) = 64 consecutive ci = 8 runs of 8 bf16
  for (int v = tid; v < 64 * K * 8; v += TPB) {
    const int r = v >> 3, j = v & 7, co = r / K, k = r - co * K;
    const bf16x8 val = *reinterpret_cast<const bf16x8*>(img + (k * 64 + co) * WP_LD + 8 * j);
    *reinterpret_cast<bf16x8*>(arena + e.wf + ((long)(co0 + co) * K + k) * e.Cin + ci0 + 8 * j) = val;
  }
  // [Cin][K][Cout] flipped taps: row (ci, k') = 64 consecutive co, read down an LDS column
  for (int v = tid; v < 64 * K * 8; v += TPB) {
    const int r = v >> 3, j = v & 7, ci = r / K, kp = r - ci * K, k = K - 1 - kp;
    bf16x8 val;
#pragma unroll
    for (int u = 0; u < 8; ++u) val[u] = img[(k * 64 + 8 * j + u) * WP_LD + ci];
    *reinterpret_cast<bf16x8*>(arena + e.wb + ((long)(ci0 + ci) * K + kp) * e.Cout + co0 + 8 * j) = val;
  }
}

inline unsigned grid_for(long n, long per_block = TPB, long cap = 8192) {
  long g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ------------------------------------------------------------------------------------------------ plan
enum OpKind : int {
  OP_CONV_FWD = 1,
  OP_CONV_WGRAD = 2,
  OP_REDUCE_WGRAD = 3,
  OP_BN_FIN = 4,
  OP_BN_ACT = 5,
  OP_BN_BWD_REDUCE = 6,
  OP_BN_BWD_APPLY = 7,
  OP_STEM_FWD = 8,
  OP_STEM_POOL = 9,
  OP_STEM_BWD_REDUCE = 10,
  OP_STEM_WGRAD = 11,
  OP_REDUCE_SUM = 12,
  OP_WEIGHT_PREP = 13,
  OP_HEAD = 14,
  OP_HEAD_REDUCE = 15,
  OP_SGD = 16,
  OP_GATHER = 17,
  OP_COUNTER_INC = 18,
};
constexpr int OP_WORDS = 32;

template <typename T>
inline T* P(int64_t v) { return reinterpret_cast<T*>(static_cast<intptr_t>(v)); }
inline float F(int64_t v) {
  double d;
  memcpy(&d, &v, sizeof d);
  return (float)d;
}

// The 16-split-group weight-gradient reduce for the many-split partials (S >= 128: the tap-shared 64-channel
// gradients, 256 splits of a 48 KB |dW|, whose 4-group reduce is a 16-deep dependent load chain), else the 4-group
// one: on the side lane the wide reduce's 4x blocks crowd the data-gradient chain's CUs (3.87 vs 3.75 ms/step when
// used for every conv, profiles/r3/resnet_knob_matrix.txt; -0.2 % for S >= 128 only, profiles/r3/resnet_reduce_ab.txt).
inline bool reduce_wide(int S) { return S >= 128; }

int run_op(const int64_t* o, hipStream_t st) {
  const int kind = (int)o[0];
  switch (kind) {
    case OP_CONV_FWD: {  // words 18..24: BN-backward statistics operands (stat_mode 1 when o[19] != 0);
                         // word 25: fused BatchNorm finalize (ecg::BnTail in device memory) or 0;
                         // words 26, 27: scale / shift that re-derive the ReLU mask from sz (or 0: load smask);
                         // words 28..30: input pre-activation {scale, shift, out} (ecg_conv1d_nlc_fwd_pa) or 0
      const void* bnb[9] = {P<void>(o[18]), P<void>(o[19]), P<void>(o[20]), P<void>(o[21]), P<void>(o[22]),
                            P<void>(o[23]), P<void>(o[24]), P<void>(o[26]), P<void>(o[27])};
      const void* pa[3] = {P<void>(o[28]), P<void>(o[29]), P<void>(o[30])};
      return ecg_conv1d_nlc_fwd_pa(P<void>(o[1]), P<void>(o[2]), P<float>(o[3]), P<void>(o[4]), P<float>(o[5]),
                                   P<void>(o[6]), P<void>(o[7]), (int)o[8], (int)o[9], (int)o[10], (int)o[11],
                                   (int)o[12], (int)o[13], (int)o[14], (int)o[15], (int)o[16], (int)o[17],
                                   o[19] ? bnb : nullptr, P<void>(o[25]), o[28] ? pa : nullptr, st);
    }
    case OP_CONV_WGRAD:
      return ecg_conv1d_nlc_wgrad(P<void>(o[1]), P<void>(o[2]), P<float>(o[3]), (int)o[4], (int)o[5], (int)o[6],
                                  (int)o[7], (int)o[8], (int)o[9], (int)o[10], (int)o[11], (int)o[12], st);
    case OP_REDUCE_WGRAD: {
      const long N = o[3] * o[4] * o[5];
      if (N % 256) return ecg::kBadArg;
      if (reduce_wide((int)o[2])) {
        hipLaunchKernelGGL(reduce_wgrad_wide_kernel, dim3((unsigned)(N / 64)), dim3(TPB), 0, st, P<const float>(o[1]),
                           (int)o[2], (int)o[3], (int)o[4], (int)o[5], P<float>(o[6]));
      } else {
        hipLaunchKernelGGL(reduce_wgrad_kernel, dim3((unsigned)(N / 256)), dim3(TPB), 0, st, P<const float>(o[1]),
                           (int)o[2], (int)o[3], (int)o[4], (int)o[5], P<float>(o[6]));
      }
      break;
    }
    case OP_BN_FIN: {
      FinArgs a{};
      a.sA = P<const float>(o[1]);
      a.sB = P<const float>(o[2]);
      a.T = (int)o[3];
      a.C = (int)o[4];
      a.mode = (int)o[5];
      a.scratch = P<double>(o[6]);
      a.n = F(o[8]);
      a.eps = F(o[9]);
      a.momentum = F(o[10]);
      a.gamma = P<const float>(o[11]);
      a.beta = P<const float>(o[12]);
      a.mean = P<float>(o[13]);
      a.rstd = P<float>(o[14]);
      a.scale = P<float>(o[15]);
      a.shift = P<float>(o[16]);
      a.run_mean = P<float>(o[17]);
      a.run_var = P<float>(o[18]);
      a.dgamma = P<float>(o[19]);
      a.dbeta = P<float>(o[20]);
      a.c1 = P<float>(o[21]);
      a.c2 = P<float>(o[22]);
      const int G = (int)o[23];
      if (a.C % 64 || G < 1 || G > 1024) return ecg::kBadArg;
      // one launch (ResNet1D-34 B=1024 with ECG_BN_TAIL=0: 3.48 ms/step vs 3.76 for the former two-launch
      // partial + final form; the fused tail stays the default at 3.39, profiles/r4/bn_fin_ab.txt)
      hipLaunchKernelGGL(bn_fin1_kernel, dim3(a.C / 64), dim3(1024), 0, st, a);
      (void)G;
      break;
    }
    case OP_BN_ACT: {
      const int mode = (int)o[1];
      const long R = o[9];
      const int C = (int)o[10];
      if (C % 8) return ecg::kBadArg;
      const dim3 g(bn_pass_grid(R, C));
      if (mode == 0)
        hipLaunchKernelGGL(bn_act_kernel<0>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]), P<const float>(o[3]),
                           P<const float>(o[4]), nullptr, nullptr, nullptr, P<__bf16>(o[8]), R, C, P<uint8_t>(o[11]));
      else if (mode == 1)
        hipLaunchKernelGGL(bn_act_kernel<1>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]), P<const float>(o[3]),
                           P<const float>(o[4]), P<const __bf16>(o[5]), nullptr, nullptr, P<__bf16>(o[8]), R, C,
                           P<uint8_t>(o[11]));
      else
        hipLaunchKernelGGL(bn_act_kernel<2>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]), P<const float>(o[3]),
                           P<const float>(o[4]), P<const __bf16>(o[5]), P<const float>(o[6]), P<const float>(o[7]),
                           P<__bf16>(o[8]), R, C, P<uint8_t>(o[11]));
      break;
    }
    case OP_BN_BWD_REDUCE: {
      const int ns = (int)o[1];
      const long R = o[11];
      const int C = (int)o[12], chunk = (int)o[13];
      if (C % 8 || C > 8 * TPB || chunk <= 0 || (o[15] && C % 64)) return ecg::kBadArg;
      const dim3 g((unsigned)((R + chunk - 1) / chunk));
      if (ns == 2)
        hipLaunchKernelGGL(bn_bwd_reduce_kernel<2>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]), P<const __bf16>(o[3]),
                           P<const __bf16>(o[4]), P<const float>(o[5]), P<const float>(o[6]), nullptr, nullptr,
                           nullptr, P<float>(o[10]), R, C, chunk, P<__bf16>(o[14]), P<const ecg::BnTail>(o[15]));
      else
        hipLaunchKernelGGL(bn_bwd_reduce_kernel<3>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]), P<const __bf16>(o[3]),
                           P<const __bf16>(o[4]), P<const float>(o[5]), P<const float>(o[6]), P<const __bf16>(o[7]),
                           P<const float>(o[8]), P<const float>(o[9]), P<float>(o[10]), R, C, chunk,
                           P<__bf16>(o[14]), P<const ecg::BnTail>(o[15]));
      break;
    }
    case OP_BN_BWD_APPLY: {
      const bool ds = o[1] != 0;
      const long R = o[17];
      const int C = (int)o[18];
      if (C % 8) return ecg::kBadArg;
      const dim3 g(bn_pass_grid(R, C));
      if (!ds)
        hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]),
                           P<const __bf16>(o[3]), P<const __bf16>(o[4]), P<const float>(o[5]), P<const float>(o[6]),
                           P<const float>(o[7]), P<const float>(o[8]), P<const float>(o[9]), P<__bf16>(o[10]),
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, R, C);
      else
        hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, g, dim3(TPB), 0, st, P<const __bf16>(o[2]),
                           P<const __bf16>(o[3]), P<const __bf16>(o[4]), P<const float>(o[5]), P<const float>(o[6]),
                           P<const float>(o[7]), P<const float>(o[8]), P<const float>(o[9]), P<__bf16>(o[10]),
                           P<const __bf16>(o[11]), P<const float>(o[12]), P<const float>(o[13]),
                           P<const float>(o[14]), P<const float>(o[15]), P<__bf16>(o[16]), R, C);
      break;
    }
    case OP_STEM_FWD: {
      const int B = (int)o[5], L = (int)o[6], Lo = (int)o[7], K = (int)o[8];
      if (K > 8) return ecg::kBadArg;
      const long M = (long)B * Lo;
      hipLaunchKernelGGL(stem_fwd_kernel, dim3((unsigned)((M + STEM_ROWS - 1) / STEM_ROWS)), dim3(TPB), 0, st,
                         P<const float>(o[1]),
                         P<const float>(o[2]), P<__bf16>(o[3]), P<float>(o[4]), B, L, Lo, K, (int)o[9], (int)o[10],
                         P<const ecg::BnTail>(o[11]));
      break;
    }
    case OP_STEM_POOL: {
      const int B = (int)o[5], Lz = (int)o[6], Lp = (int)o[7], C = (int)o[8];
      hipLaunchKernelGGL(stem_pool_kernel, dim3(grid_for((long)B * Lp * C / 8)), dim3(TPB), 0, st,
                         P<const __bf16>(o[1]), P<const float>(o[2]), P<const float>(o[3]), P<__bf16>(o[4]),
                         P<uint8_t>(o[9]), B, Lz, Lp, C);
      break;
    }
    case OP_STEM_BWD_REDUCE: {
      const int B = (int)o[9], Lz = (int)o[10], Lp = (int)o[11], C = (int)o[12], chunk = (int)o[13];
      if (C % 8 || 2 * C * (TPB / (C / 8)) > TPB * 16 || (o[14] && (C % 64 || C > 256)) || !o[15]) return ecg::kBadArg;
      const long R = (long)B * Lz;
      hipLaunchKernelGGL(stem_bwd_reduce_kernel, dim3((unsigned)((R + chunk - 1) / chunk)), dim3(TPB), 0, st,
                         P<const __bf16>(o[1]), P<const __bf16>(o[2]), P<const float>(o[3]), P<const float>(o[4]),
                         P<const float>(o[5]), P<const float>(o[6]), P<__bf16>(o[7]), P<float>(o[8]), B, Lz, Lp, C,
                         chunk, P<const ecg::BnTail>(o[14]), P<const uint8_t>(o[15]));
      break;
    }
    case OP_STEM_WGRAD: {
      const int B = (int)o[10], L = (int)o[11], Lz = (int)o[12], K = (int)o[13], chunk = (int)o[16];
      if (K > 8) return ecg::kBadArg;
      const long R = (long)B * Lz;
      hipLaunchKernelGGL(stem_wgrad_kernel, dim3((unsigned)((R + chunk - 1) / chunk)), dim3(TPB), 0, st,
                         P<const __bf16>(o[1]), P<const __bf16>(o[2]), P<const float>(o[3]), P<const float>(o[4]),
                         P<const float>(o[5]), P<const float>(o[6]), P<const float>(o[7]), P<const float>(o[8]),
                         P<float>(o[9]), B, L, Lz, K, (int)o[14], (int)o[15], chunk);
      break;
    }
    case OP_REDUCE_SUM: {
      const long N = o[3];
      hipLaunchKernelGGL(reduce_sum_kernel, dim3((unsigned)((N + 63) / 64)), dim3(64 * RS_GROUPS), 0, st,
                         P<const float>(o[1]), (int)o[2], N,
                         P<float>(o[4]), (long)o[5], P<float>(o[6]));
      break;
    }
    case OP_WEIGHT_PREP:
      if (o[2] < 1 || o[2] > TPB) return ecg::kBadArg;  // one thread per table entry picks the workgroup's conv
      hipLaunchKernelGGL(weight_prep_kernel, dim3((unsigned)o[3]), dim3(TPB), 0, st, P<const WEntry>(o[1]),
                         (int)o[2], P<const float>(o[4]), P<__bf16>(o[5]));
      break;
    case OP_HEAD: {
      const int B = (int)o[9], Lf = (int)o[10], C = (int)o[11], ncls = (int)o[12];
      if (C > 1024 || C % 8 || ncls > MAXC || ncls < 1) return ecg::kBadArg;
      hipLaunchKernelGGL(head_fwd_bwd_kernel, dim3(B), dim3(TPB), 0, st, P<const __bf16>(o[1]), P<const float>(o[2]),
                         P<const float>(o[3]), P<const int>(o[4]), P<__bf16>(o[5]), P<float>(o[6]), P<float>(o[7]),
                         P<float>(o[8]), B, Lf, C, ncls);
      break;
    }
    case OP_HEAD_REDUCE: {
      const int B = (int)o[5], C = (int)o[6], ncls = (int)o[7], Gb = (int)o[8];
      hipLaunchKernelGGL(head_reduce_kernel, dim3((unsigned)((C + 63) / 64), (unsigned)Gb), dim3(TPB), 0, st,
                         P<const float>(o[1]), P<const float>(o[2]), P<const float>(o[3]), P<float>(o[4]), B, C, ncls);
      break;
    }
    case OP_SGD:
      return ecg_sgd_flat(P<float>(o[1]), P<const float>(o[2]), P<float>(o[3]), (long)o[4], F(o[5]), F(o[6]), 0.f,
                          F(o[7]), (int)o[8], 0, 1.f, nullptr, st);
    case OP_GATHER: {
      const int S = (int)o[6], B = (int)o[7], L = (int)o[8];
      if (S <= 0 || B <= 0 || L <= 0) return ecg::kBadArg;
      hipLaunchKernelGGL(gather_step_kernel, dim3(B), dim3(TPB), 0, st, P<const float>(o[1]), (long)o[2],
                         P<const int>(o[3]), P<const int>(o[4]), P<const int>(o[5]), S, B, L, P<float>(o[9]),
                         P<int>(o[10]));
      break;
    }
    case OP_COUNTER_INC:
      hipLaunchKernelGGL(counter_inc_kernel, dim3(1), dim3(1), 0, st, P<int>(o[1]));
      break;
    default:
      return ecg::kBadArg;
  }
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

struct PlanGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

}  // namespace

// Size of one encoded op (int64 words).
ECG_API int ecg_plan_op_words() { return OP_WORDS; }

// Rows per block of the stem forward kernel (= rows per BN-statistics partial of the stem BN).
ECG_API int ecg_plan_stem_rows() { return STEM_ROWS; }

// Number of blocks the weight-prep op needs for a table; fills WEntry.block0 in a host-side copy.
ECG_API int ecg_plan_wentry_bytes() { return (int)sizeof(WEntry); }

namespace {
// Lanes (word OP_LANE of an op): the weight-gradient ops (CONV_WGRAD + REDUCE_WGRAD) are off the backward's
// critical path - only the optimizer reads what they write - so the plan can put them on a side stream: the
// MFMA-bound weight-gradient kernels then fill the data-gradient chain's idle time (kernel boundaries, the
// BatchNorm finalize tails, the memory-bound BN_BWD_APPLY passes).  Ordering: before a side op, the side
// stream waits for everything enqueued on the main stream so far (it reads the gradient the main chain just
// produced); LANE_JOIN ops (the optimizer) and the end of every run wait for the side stream.  Inside a
// capture the same event record / wait pairs become graph edges, so a graph is the fork-join DAG.
constexpr int OP_LANE = OP_WORDS - 1;
enum : int { LANE_MAIN = 0, LANE_SIDE = 1, LANE_JOIN = 2 };

struct SideLane {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

int side_lane(SideLane** out) {
  static SideLane lanes[64];
  int dev = 0;
  ECG_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return ecg::kBadArg;
  SideLane& l = lanes[dev];
  if (!l.side) {
    // lowest priority: the data-gradient chain is the critical path (profiles/r2/resnet_side_prio_ab.txt; a
    // CU-masked side queue, hipExtStreamCreateWithCUMask with 2/4/6 of every 8 CUs, measured 7.5-7.8 ms/step
    // against 3.93 on ResNet1D-34 B=1024)
    int lo = 0, hi = 0;
    ECG_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    ECG_HIP_CHECK(hipStreamCreateWithPriority(&l.side, hipStreamNonBlocking, lo));
    // The fork / join markers carry no system-scope fence (hipEventDisableSystemFence; ECG_SIDE_NOFENCE=0 restores
    // the default event): they only order two streams of this device, and the producing kernel's own end-of-kernel
    // release plus the consumer kernel's acquire already make the data visible device-wide; the system-scope fence
    // of a default event made each fork's marker flush caches on the main lane.  3.308-3.329 vs 3.344-3.361 ms/step
    // (ResNet1D-34 B=1024, interleaved; profiles/r6/bn_tail_xcd_ab.txt), engine GPU tests pass with it.
    const char* nf = getenv("ECG_SIDE_NOFENCE");
    const unsigned ef = hipEventDisableTiming | ((nf == nullptr || atoi(nf)) ? hipEventDisableSystemFence : 0u);
    ECG_HIP_CHECK(hipEventCreateWithFlags(&l.fork, ef));
    ECG_HIP_CHECK(hipEventCreateWithFlags(&l.join, ef));
  }
  *out = &l;
  return ecg::kOk;
}
}  // namespace

// Run ``nops`` encoded ops back to back on ``stream`` (side-lane ops on the device's side stream, joined back
// before LANE_JOIN ops and before returning).  Returns the first failing op's status (ops before it have been
// enqueued).  ``first_bad`` (optional) receives its index.
ECG_API int ecg_plan_run_ex(const int64_t* ops, int nops, int* first_bad, hipStream_t stream, int join_end,
                            hipStream_t* side_out);

ECG_API int ecg_plan_run(const int64_t* ops, int nops, int* first_bad, hipStream_t stream) {
  return ecg_plan_run_ex(ops, nops, first_bad, stream, 1, nullptr);
}

// The device's side-lane stream (created on first use): callers that run a plan range with join_end = 0 order
// their own work (a gradient bucket's all-reduce) after it instead of making the main stream wait.
ECG_API int ecg_plan_side_stream(hipStream_t* out) {
  if (!out) return ecg::kBadArg;
  SideLane* lane = nullptr;
  const int st = side_lane(&lane);
  if (st) return st;
  *out = lane->side;
  return ecg::kOk;
}

// Make ``stream`` wait for everything enqueued on the device's side lane so far.
ECG_API int ecg_plan_join(hipStream_t stream) {
  SideLane* lane = nullptr;
  const int st = side_lane(&lane);
  if (st) return st;
  ECG_HIP_CHECK(hipEventRecord(lane->join, lane->side));
  ECG_HIP_CHECK(hipStreamWaitEvent(stream, lane->join, 0));
  return ecg::kOk;
}

// ecg_plan_run with the end-of-run join optional: join_end = 0 leaves the range's side-lane work running (the
// caller joins later with ecg_plan_join, or orders a consumer after the side stream); *side_out (optional) receives
// the side stream when the range put work on it, else null.  LANE_JOIN ops still join.
ECG_API int ecg_plan_run_ex(const int64_t* ops, int nops, int* first_bad, hipStream_t stream, int join_end,
                            hipStream_t* side_out) {
  if (side_out) *side_out = nullptr;
  if (!ops || nops < 0) return ecg::kBadArg;
  SideLane* lane = nullptr;
  bool side_busy = false, main_ahead = true;  // side has unjoined work / main has work the side has not waited for
  int st = ecg::kOk;
  auto join = [&]() -> int {
    if (!side_busy) return ecg::kOk;
    ECG_HIP_CHECK(hipEventRecord(lane->join, lane->side));
    ECG_HIP_CHECK(hipStreamWaitEvent(stream, lane->join, 0));
    side_busy = false;
    return ecg::kOk;
  };
  int bad = -1;
  for (int i = 0; i < nops && bad < 0; ++i) {
    const int64_t* o = ops + (long)i * OP_WORDS;
    const int64_t ln = o[OP_LANE];
    if (ln == LANE_SIDE) {
      if (!lane) st = side_lane(&lane);
      if (st == 0 && main_ahead) {
        ECG_HIP_CHECK(hipEventRecord(lane->fork, stream));
        ECG_HIP_CHECK(hipStreamWaitEvent(lane->side, lane->fork, 0));
        main_ahead = false;
      }
      if (st == 0) {
        st = run_op(o, lane->side);
        side_busy = true;
      }
    } else {
      if (ln == LANE_JOIN) st = join();
      if (st == 0) st = run_op(o, stream);
      main_ahead = true;
    }
    if (st) bad = i;
  }
  if (st) {
    if (first_bad) *first_bad = bad;
    (void)join();  // leave no side work unjoined (a capture must end with every stream joined)
    return st;
  }
  if (!join_end) {
    if (side_out && side_busy) *side_out = lane->side;
    return ecg::kOk;
  }
  return join();
}

// Capture the plan into one hipGraph (all pointers baked in; callers keep every buffer alive).
ECG_API int ecg_plan_graph_create(void** handle, const int64_t* ops, int nops, int* first_bad) {
  if (!handle || !ops || nops <= 0) return ecg::kBadArg;
  hipStream_t cap;
  ECG_HIP_CHECK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  PlanGraph* pg = new PlanGraph();
  hipError_t e = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete pg;
    (void)hipStreamDestroy(cap);
    return ecg::kHipError;
  }
  const int st = ecg_plan_run(ops, nops, first_bad, cap);
  e = hipStreamEndCapture(cap, &pg->graph);
  (void)hipStreamDestroy(cap);
  if (st != 0 || e != hipSuccess) {
    if (pg->graph) (void)hipGraphDestroy(pg->graph);
    delete pg;
    return st ? st : ecg::kHipError;
  }
  e = hipGraphInstantiate(&pg->exec, pg->graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(pg->graph);
    delete pg;
    return ecg::kHipError;
  }
  *handle = pg;
  return ecg::kOk;
}

ECG_API int ecg_plan_graph_launch(void* handle, hipStream_t stream) {
  if (!handle) return ecg::kBadArg;
  ECG_HIP_CHECK(hipGraphLaunch(static_cast<PlanGraph*>(handle)->exec, stream));
  return ecg::kOk;
}

ECG_API int ecg_plan_graph_destroy(void* handle) {
  if (!handle) return ecg::kOk;
  PlanGraph* pg = static_cast<PlanGraph*>(handle);
  if (pg->exec) (void)hipGraphExecDestroy(pg->exec);
  if (pg->graph) (void)hipGraphDestroy(pg->graph);
  delete pg;
  return ecg::kOk;
}
