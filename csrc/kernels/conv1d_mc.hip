// Multi-channel conv1d for gfx950 on bf16 MFMA (v_mfma_f32_16x16x32_bf16), channels-last (NLC) implicit GEMM.
//
// Used by the ResNet1D stress model (BASELINE.json config 5) and any conv1d with C_in % 64 == 0 and
// C_out % 64 == 0; TinyECG's own convs run inside the fused step kernel (tiny_ecg_step.hip).
// SURVEY §2.2 "conv1d_mc_fwd / conv1d_mc_bwd": forward, data-grad and weight-grad of a padded, strided conv.
//
//   forward   y[b,t,co] = bias[co] + sum_{k,ci} x[b, t*s + k - p, ci] * w[co,k,ci]
//             GEMM M = B*L_out (rows (b,t)), N = C_out, K = Kw*C_in (kk = k*C_in + ci).  Both operands are
//             contiguous along kk (NLC activations, [C_out][Kw][C_in] weights), so tiles are staged into LDS
//             with 16-byte loads in exactly the MFMA fragment order (8 consecutive kk per lane).
//   data-grad dx = the same kernel on dy with input dilation s (zero-insertion), taps flipped, pad Kw-1-p,
//             weights re-laid out as [C_in][Kw][C_out].
//   wgrad     dw[co,k,ci] = sum_{(b,t)} dy[b,t,co] * x[b, t*s+k-p, ci]: the reduction index (b,t) is the ROW
//             of both staged tiles, so fragments come from gfx950's transposing LDS read ds_read_b64_tr_b16;
//             the (b,t) range is split over workgroups into fp32 partials (summed deterministically after).
//
// Forward block tile 64x64 / 128x64 / 128x128 (by size), BK = 64, 4 waves (2x2), double-buffered LDS with the
// next tile's global loads issued before the current tile's MFMAs (register staging).
#include "../include/ecg_common.h"

#include "../include/bn_tail.h"
#include <climits>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int BK = 64;
constexpr int THREADS = 256;
constexpr int LDS_ROW = BK + 8;  // bf16 elements per LDS row (+16 B pad: conflict-free ds_read_b128)

typedef short s16x8 __attribute__((ext_vector_type(8)));

struct FwdArgs {
  const __bf16* x;    // [B][Lin][Cin]
  const __bf16* w;    // [Cout][Kw][Cin]
  const float* bias;  // [Cout] or nullptr
  __bf16* y;          // [B][Lout][Cout]
  float* stats;       // [2][gridDim.x][Cout] per-M-tile partial sum / sum of squares of the stored outputs, or null
  const __bf16* add;  // [B*Lout][Cout] added before the store (residual-gradient path), or null
  const __bf16* add_mask;  // if non-null the added term is add * (add_mask > 0)  (ReLU backward of the residual)
  int B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil, relu;
  // BatchNorm-backward statistics mode (stat_mode == 1; data-grad convs): the stored value is masked by
  // smask > 0 (ReLU backward) and the partials are sum(v), sum(v * xhat) [, sum(v * xhat_d)] with
  // xhat = (sz - smean) * srstd (and the downsample branch's szd / smean_d / srstd_d when szd != null).
  int stat_mode;
  int Lph, tpp;  // strided data-grad (in_dil > 1): output rows per sample per phase, M tiles per phase
  const __bf16* smask;
  const __bf16* sz;
  const float* smean;
  const float* srstd;
  const __bf16* szd;
  const float* smean_d;
  const float* srstd_d;
  // Mask from sz (stat_mode 1): when non-null the ReLU mask is bf16(max(fmaf(sz, mscale, mshift), 0)) > 0 - the
  // exact values the BN_ACT pass stored as smask (conv -> BN -> ReLU), so smask need not be read
  const float* mscale;
  const float* mshift;
  // A-operand transform (register-staged forward only): when non-null the staged activation is
  // bf16(max(fmaf(x, ascale[c], ashift[c]), 0)) - a BatchNorm + ReLU folded into the consumer conv's operand load
  // (padding rows stay zero)
  const float* ascale;
  const float* ashift;
  const ecg::BnTail* tail;  // BatchNorm finalize fused into this launch's tail (bn_tail.h), or null
};

// A tile: 64 rows (b,t) x 64 kk (one tap k, channels c0..c0+63); element e (0..511) = row e>>3, 8 bf16 part e&7
__device__ __forceinline__ uint4 load_a_fwd(const FwdArgs a, int m0, int kk0, int e) {
  const int k = kk0 / a.Cin, c0 = kk0 % a.Cin;
  const int row = e >> 3, part = e & 7;
  const int m = m0 + row;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (m < a.B * a.Lout) {
    const int b = m / a.Lout, t = m % a.Lout;
    int u = t * a.stride + k - a.pad;  // position in the (dilated) input
    bool ok = u >= 0;
    if (a.in_dil > 1) {
      ok = ok && (u % a.in_dil == 0);
      u /= a.in_dil;
    }
    ok = ok && u < a.Lin;
    if (ok) v = *reinterpret_cast<const uint4*>(a.x + ((long)b * a.Lin + u) * a.Cin + c0 + part * 8);
  }
  return v;
}

__device__ __forceinline__ uint4 load_b_fwd(const FwdArgs a, int n0, int kk0, int e) {
  const int row = e >> 3, part = e & 7;
  return *reinterpret_cast<const uint4*>(a.w + (long)(n0 + row) * (a.Kw * a.Cin) + kk0 + part * 8);
}

__device__ __forceinline__ void store_one(__bf16* lds, int e, uint4 v) {
  *reinterpret_cast<uint4*>(lds + (e >> 3) * LDS_ROW + (e & 7) * 8) = v;
}

// Block tile BM x BN (64/128), 4 waves as 2x2, each wave (BM/2) x (BN/2) = FM x FN MFMA 16x16 tiles.
// Grid is 1-D over MT*NT tiles with a bijective XCD remap: consecutive tile ids (same M panel, all N tiles)
// run on one XCD, so the A panel (the activations) is read from HBM once per XCD-L2.
// Epilogue: accumulators -> LDS (fp32) -> row-major pass with 16-B loads/stores: + bias, + residual
// (optionally ReLU-masked), ReLU, bf16 round, and per-channel BN partials of the rounded values.
// NWR = waves along M (2 x NWR waves per workgroup, 64 * 2 * NWR threads); the register-staged kernel uses 2.
template <int BM, int BN, int NWR = 2>
struct FwdCfg {
  static constexpr int NW = 2 * NWR, NTHR = 64 * NW;
  static constexpr int WM = BM / NWR, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  static constexpr int NA = BM * 8 / THREADS, NB = BN * 8 / THREADS;
  static constexpr int A_EL = BM * LDS_ROW, B_EL = BN * LDS_ROW;
  static constexpr int EP_LD = WN + 4;
  static constexpr int EP_BYTES = NW * (WM / 2) * EP_LD * 4 + NWR * 3 * BN * 4;  // epilogue staged in two halves
  static constexpr int stage_bytes(int nbuf) { return nbuf * (A_EL + B_EL) * 2; }
  static constexpr int smem(int nbuf) { return stage_bytes(nbuf) > EP_BYTES ? stage_bytes(nbuf) : EP_BYTES; }
};

// Forward / data-grad epilogue shared by the main loops: accumulators -> LDS (fp32, per-wave region, two halves
// of WM/2 rows) -> row-major pass with 8 channels per lane: + bias, + residual (optionally ReLU-masked), ReLU,
// bf16 round, and the per-channel BatchNorm partials of the rounded values (stat_mode 0) or the BN-backward
// partials (stat_mode 1).  The staging buffers must be dead (all waves past the main loop's last barrier).
// Split in three so the multi-tile kernel can store several M tiles and emit ONE partial row for all of them:
// EpiConst (per-lane channel constants, fixed for a column block), fwd_epi_tile (one tile's store + the
// lane's running statistics), fwd_epi_stats (cross-lane / cross-wave reduction and the partial-row store).
template <int BN, int NWR>
struct EpiLane {
  static constexpr int WN = BN / 2, CG = WN / 8;
  __device__ static int n(int n0) { return n0 + ((threadIdx.x >> 6) & 1) * WN + ((threadIdx.x & 63) % CG) * 8; }
};

struct EpiConst {
  float bv[8], mu[8], rsd[8], mud[8], rsdd[8], msc[8], msh[8];
  float s1[8], s2[8], s3[8];
  template <bool BWD>
  __device__ __forceinline__ void load(const FwdArgs& a, int n) {
    const bool ds = BWD && a.szd != nullptr;
    const bool mz = BWD && a.mscale != nullptr;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bv[e] = a.bias ? a.bias[n + e] : 0.f;
      s1[e] = s2[e] = s3[e] = 0.f;
      mu[e] = BWD ? a.smean[n + e] : 0.f;
      rsd[e] = BWD ? a.srstd[n + e] : 0.f;
      mud[e] = ds ? a.smean_d[n + e] : 0.f;
      rsdd[e] = ds ? a.srstd_d[n + e] : 0.f;
      msc[e] = mz ? a.mscale[n + e] : 0.f;
      msh[e] = mz ? a.mshift[n + e] : 0.f;
    }
  }
};

template <int BM, int BN, int EPI, int NWR = 2>
__device__ __forceinline__ void fwd_epi_tile_rowwise(const FwdArgs& a, f32x4 (&acc)[BM / NWR / 16][BN / 32],
                                             unsigned char* smem, EpiConst& k, int m0, int n0, int Lrow, int M, int P,
                                             int ph) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1;
  constexpr int EP_LD = Cfg::EP_LD, HR = WM / 2;
  float* ep = reinterpret_cast<float*>(smem) + wv * HR * EP_LD;
  constexpr int CG = WN / 8, RSTEP = 64 / CG, ITEMS = HR / RSTEP;
  const int cg = lane % CG, rs = lane / CG;
  const int n = EpiLane<BN, NWR>::n(n0);
  constexpr bool bwd = EPI == 1;  // compile-time: the forward epilogue carries none of the backward code
  const bool ds = bwd && a.szd != nullptr;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) __syncthreads();  // previous half fully read
#pragma unroll
    for (int i = 0; i < FM / 2; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          ep[(i * 16 + 4 * (lane >> 4) + q) * EP_LD + j * 16 + (lane & 15)] = acc[h * (FM / 2) + i][j][q];
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < ITEMS; ++it) {
      const int rl = rs + it * RSTEP;
      const int r = h * HR + rl;
      const int m = m0 + wr * WM + r;
      const int bb = m / Lrow, tt = m - bb * Lrow;
      const int uu = P > 1 ? tt * P + ph : tt;
      if (m < M && uu < a.Lout) {
        const long o = ((long)bb * a.Lout + uu) * a.Cout + n;
        const float4 v0 = *reinterpret_cast<const float4*>(ep + rl * EP_LD + cg * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(ep + rl * EP_LD + cg * 8 + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += k.bv[e];
        if (a.add) {
          const bf16x8 ad = *reinterpret_cast<const bf16x8*>(a.add + o);
          if (a.add_mask) {
            const bf16x8 mk = *reinterpret_cast<const bf16x8*>(a.add_mask + o);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)mk[e] > 0.f ? (float)ad[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)ad[e];
          }
        }
        bf16x8 zz;
        if constexpr (bwd) zz = *reinterpret_cast<const bf16x8*>(a.sz + o);
        if (bwd && a.mscale != nullptr) {  // the mask the BN_ACT pass stored, recomputed from sz
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const __bf16 act = (__bf16)fmaxf(fmaf((float)zz[e], k.msc[e], k.msh[e]), 0.f);
            v[e] = (float)act > 0.f ? v[e] : 0.f;
          }
        } else if (bwd && a.smask != nullptr) {
          const bf16x8 mk = *reinterpret_cast<const bf16x8*>(a.smask + o);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (float)mk[e] > 0.f ? v[e] : 0.f;
        }
        bf16x8 outv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (a.relu) v[e] = fmaxf(v[e], 0.f);
          outv[e] = (__bf16)v[e];
          v[e] = (float)outv[e];
        }
        *reinterpret_cast<bf16x8*>(a.y + o) = outv;
        if constexpr (bwd) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            k.s1[e] += v[e];
            k.s2[e] += v[e] * ((float)zz[e] - k.mu[e]) * k.rsd[e];
          }
          if (ds) {
            const bf16x8 zd = *reinterpret_cast<const bf16x8*>(a.szd + o);
#pragma unroll
            for (int e = 0; e < 8; ++e) k.s3[e] += v[e] * ((float)zd[e] - k.mud[e]) * k.rsdd[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            k.s1[e] += v[e];
            k.s2[e] += v[e] * v[e];
          }
        }
      }
    }
  }
}

template <int BM, int BN, int EPI, int NWR = 2>
__device__ __forceinline__ void fwd_epi_tile_pref(const FwdArgs& a, f32x4 (&acc)[BM / NWR / 16][BN / 32],
                                             unsigned char* smem, EpiConst& k, int m0, int n0, int Lrow, int M, int P,
                                             int ph) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1;
  constexpr int EP_LD = Cfg::EP_LD, HR = WM / 2;
  float* ep = reinterpret_cast<float*>(smem) + wv * HR * EP_LD;
  constexpr int CG = WN / 8, RSTEP = 64 / CG, ITEMS = HR / RSTEP;
  const int cg = lane % CG, rs = lane / CG;
  const int n = EpiLane<BN, NWR>::n(n0);
  constexpr bool bwd = EPI == 1;  // compile-time: the forward epilogue carries none of the backward code
  const bool ds = bwd && a.szd != nullptr;
  const bool mk_smask = bwd && a.mscale == nullptr && a.smask != nullptr;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // The half's global operands (z, z_d, residual gradient and its mask) for all ITEMS rows are issued before the
    // accumulators are staged, so the half costs ONE load round trip instead of one per row pair.  Rows outside
    // the output read offset 0 (valid memory, value unused).
    long po[ITEMS];
    bool pv[ITEMS];
    bf16x8 pz[ITEMS], pzd[ITEMS], pad[ITEMS], pmk[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int r = h * HR + rs + it * RSTEP;
      const int m = m0 + wr * WM + r;
      const int bb = m / Lrow, tt = m - bb * Lrow;
      const int uu = P > 1 ? tt * P + ph : tt;
      pv[it] = m < M && uu < a.Lout;
      po[it] = pv[it] ? ((long)bb * a.Lout + uu) * a.Cout + n : 0;
      if constexpr (bwd) pz[it] = *reinterpret_cast<const bf16x8*>(a.sz + po[it]);
      if (ds) pzd[it] = *reinterpret_cast<const bf16x8*>(a.szd + po[it]);
      if (a.add) pad[it] = *reinterpret_cast<const bf16x8*>(a.add + po[it]);
      if (a.add && a.add_mask) pmk[it] = *reinterpret_cast<const bf16x8*>(a.add_mask + po[it]);
      else if (mk_smask) pmk[it] = *reinterpret_cast<const bf16x8*>(a.smask + po[it]);
    }
    if (h) __syncthreads();  // previous half fully read
#pragma unroll
    for (int i = 0; i < FM / 2; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          ep[(i * 16 + 4 * (lane >> 4) + q) * EP_LD + j * 16 + (lane & 15)] = acc[h * (FM / 2) + i][j][q];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int rl = rs + it * RSTEP;
      if (pv[it]) {
        const long o = po[it];
        const float4 v0 = *reinterpret_cast<const float4*>(ep + rl * EP_LD + cg * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(ep + rl * EP_LD + cg * 8 + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += k.bv[e];
        if (a.add) {
          const bf16x8 ad = pad[it];
          if (a.add_mask) {
            const bf16x8 mk = pmk[it];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)mk[e] > 0.f ? (float)ad[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)ad[e];
          }
        }
        bf16x8 zz;
        if constexpr (bwd) zz = pz[it];
        if (bwd && a.mscale != nullptr) {  // the mask the BN_ACT pass stored, recomputed from sz
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const __bf16 act = (__bf16)fmaxf(fmaf((float)zz[e], k.msc[e], k.msh[e]), 0.f);
            v[e] = (float)act > 0.f ? v[e] : 0.f;
          }
        } else if (mk_smask) {
          const bf16x8 mk = a.add && a.add_mask ? *reinterpret_cast<const bf16x8*>(a.smask + o) : pmk[it];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (float)mk[e] > 0.f ? v[e] : 0.f;
        }
        bf16x8 outv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (a.relu) v[e] = fmaxf(v[e], 0.f);
          outv[e] = (__bf16)v[e];
          v[e] = (float)outv[e];
        }
        *reinterpret_cast<bf16x8*>(a.y + o) = outv;
        if constexpr (bwd) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            k.s1[e] += v[e];
            k.s2[e] += v[e] * ((float)zz[e] - k.mu[e]) * k.rsd[e];
          }
          if (ds) {
            const bf16x8 zd = pzd[it];
#pragma unroll
            for (int e = 0; e < 8; ++e) k.s3[e] += v[e] * ((float)zd[e] - k.mud[e]) * k.rsdd[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            k.s1[e] += v[e];
            k.s2[e] += v[e] * v[e];
          }
        }
      }
    }
  }
}

// One tile's epilogue: the prefetching form (every global operand row of a half issued before the half is staged)
// where registers allow, else the row-by-row form (register-tight NBUF = 1 / 256-row kernels).
// Measured: ResNet1D-34 B=1024 3.87 -> 3.79 ms/step with the prefetching form (profiles/r3/resnet_epi_tail_ab.txt).
template <int BM, int BN, int EPI, int NWR = 2, bool PREF = true>
__device__ __forceinline__ void fwd_epi_tile(const FwdArgs& a, f32x4 (&acc)[BM / NWR / 16][BN / 32],
                                             unsigned char* smem, EpiConst& k, int m0, int n0, int Lrow, int M, int P,
                                             int ph) {
  if constexpr (PREF)
    fwd_epi_tile_pref<BM, BN, EPI, NWR>(a, acc, smem, k, m0, n0, Lrow, M, P, ph);
  else
    fwd_epi_tile_rowwise<BM, BN, EPI, NWR>(a, acc, smem, k, m0, n0, Lrow, M, P, ph);
}

// The lanes' running statistics -> one partial row ``row`` of ``nrows`` (columns n0 .. n0 + BN).  Block-uniform
// call (a.stats != null); ``smem``: the dead epilogue region.
template <int BM, int BN, int EPI, int NWR = 2>
__device__ __forceinline__ void fwd_epi_stats(const FwdArgs& a, unsigned char* smem, EpiConst& k, int n0, int row,
                                              int nrows) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WN = Cfg::WN, HR = Cfg::WM / 2, EP_LD = Cfg::EP_LD, CG = WN / 8;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1, cg = lane % CG;
  const bool ds = EPI == 1 && a.szd != nullptr;
  const int NS = ds ? 3 : 2;
#pragma unroll
  for (int off = CG; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      k.s1[e] += __shfl_xor(k.s1[e], off);
      k.s2[e] += __shfl_xor(k.s2[e], off);
      if (ds) k.s3[e] += __shfl_xor(k.s3[e], off);
    }
  float* sred = reinterpret_cast<float*>(smem) + Cfg::NW * HR * EP_LD;  // [wr][stat][BN]
  if (lane < CG) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sred[(wr * 3 + 0) * BN + wc * WN + cg * 8 + e] = k.s1[e];
      sred[(wr * 3 + 1) * BN + wc * WN + cg * 8 + e] = k.s2[e];
      sred[(wr * 3 + 2) * BN + wc * WN + cg * 8 + e] = k.s3[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < NS * BN; i += Cfg::NTHR) {
    const int st = i / BN, c = i % BN;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < NWR; ++r) v += sred[(3 * r + st) * BN + c];
    float* dst = a.stats + ((long)st * nrows + row) * a.Cout + n0 + c;
    if (a.tail)
      ecg::st_sc1(dst, v);  // handed to the tail's last arriver inside this launch (write-through)
    else
      *dst = v;
  }
}

template <int BM, int BN, int EPI, int NWR = 2, bool PREF = true>
__device__ __forceinline__ void fwd_epilogue(const FwdArgs& a, f32x4 (&acc)[BM / NWR / 16][BN / 32],
                                             unsigned char* smem, int m0, int n0, int mt, int MT, int Lrow, int M,
                                             int P, int ph) {
  EpiConst k;
  k.load<EPI == 1>(a, EpiLane<BN, NWR>::n(n0));
  fwd_epi_tile<BM, BN, EPI, NWR, PREF>(a, acc, smem, k, m0, n0, Lrow, M, P, ph);
  if (a.stats) fwd_epi_stats<BM, BN, EPI, NWR>(a, smem, k, n0, mt, MT);  // block-uniform
}

// NBUF = 2: double-buffered LDS, one barrier per K tile (2 workgroups / CU at 128x128).
// NBUF = 1: one LDS buffer, two barriers per K tile, half the LDS -> 3 workgroups / CU, i.e. 1.5x the
//           register-staged tiles in flight per CU for this HBM-latency-bound loop.
template <int BM, int BN, int EPI, int NBUF>
__global__ __launch_bounds__(THREADS, NBUF == 1 ? 3 : 2) void conv1d_nlc_fwd_kernel(FwdArgs a, int MT, int NT) {
  using Cfg = FwdCfg<BM, BN>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NA = Cfg::NA, NB = Cfg::NB;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __bf16* const lds = reinterpret_cast<__bf16*>(smem);  // [buf][A (BM rows) | B (BN rows)][LDS_ROW]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  // bijective XCD remap of the 1-D grid (blockIdx % 8 = blocks sharing an XCD)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int mt = wgid / NT, nt = wgid % NT;
  const int K = a.Kw * a.Cin;
  // Strided data-grad (in_dil = s > 1) is phase-decomposed: output rows u = i*s + ph of one phase share the
  // taps k = k0 + j*s (k0 = (pad - ph) mod s) that hit non-inserted input rows, so the zero half of the
  // dilated input is never multiplied.  M tiles are per phase; K tiles run over the phase's taps only.
  const int P = a.in_dil;
  const int ph = P > 1 ? mt / a.tpp : 0;
  const int m0 = (P > 1 ? mt - ph * a.tpp : mt) * BM, n0 = nt * BN;
  const int CB = a.Cin / BK;
  const int k0 = P > 1 ? ((a.pad - ph) % P + P) % P : 0;
  const int nk = P > 1 ? (k0 < a.Kw ? (a.Kw - k0 + P - 1) / P : 0) * CB : K / BK;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // One register set: tile t+1's global loads are in flight during tile t's MFMAs.  (Measured alternatives,
  // profiles/r1_resnet/conv_microbench_*: a second register set (tile t+2 in flight) costs occupancy and runs
  // 35 % slower; B fragments loaded straight from L2 into registers, bypassing LDS, 25-35 % slower.)
  uint4 ra0[NA], rb0[NB];
  // per-thread A rows are fixed across K tiles: precompute each row's sample base and first input position
  const int Lrow = P > 1 ? a.Lph : a.Lout;  // rows per sample in this kernel's (phase-local) M index
  const int M = a.B * Lrow;
  long abase[NA];
  int apos[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int e = tid + i * THREADS, m = m0 + (e >> 3);
    const int b = m / Lrow, t = m % Lrow;
    const int u = P > 1 ? t * P + ph : t;  // output position
    abase[i] = (long)b * a.Lin * a.Cin + (e & 7) * 8;
    apos[i] = (m < M && u < a.Lout) ? u * a.stride - a.pad : INT_MIN / 2;  // invalid rows never pass the check
  }
  const __bf16* wb = a.w + (long)(n0 + (tid >> 3)) * (a.Kw * a.Cin) + (tid & 7) * 8;
  const int Lext = a.in_dil > 1 ? (a.Lin - 1) * a.in_dil + 1 : a.Lin;  // extent of the (dilated) input
  const bool fold = a.ascale != nullptr;  // block-uniform
  unsigned aok = 0u;  // rows of the staged A set that are real input rows (fold: padding stays zero)
  float4 asc0, asc1, ash0, ash1;  // the staged set's 8 channels' BN scale / shift (fold)
  auto ld_set = [&](uint4* ra, uint4* rb, int t) {
    const int tc = t < nk ? t : nk - 1;
    const int k = k0 + (tc / CB) * P, c0 = (tc % CB) * BK;
    const int kk = k * a.Cin + c0;
    aok = 0u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int u = apos[i] + k;
      bool ok = u >= 0 && u < Lext;
      if (a.in_dil > 1) {
        ok = ok && (u % a.in_dil == 0);
        u /= a.in_dil;
      }
      aok |= (ok ? 1u : 0u) << i;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(a.x + abase[i] + (long)u * a.Cin + c0) : make_uint4(0u, 0u, 0u, 0u);
    }
    if (fold) {  // (every A piece of this thread covers channels c0 + (tid & 7) * 8 .. + 8)
      const float4* sp = reinterpret_cast<const float4*>(a.ascale + c0 + (tid & 7) * 8);
      const float4* hp = reinterpret_cast<const float4*>(a.ashift + c0 + (tid & 7) * 8);
      asc0 = sp[0];
      asc1 = sp[1];
      ash0 = hp[0];
      ash1 = hp[1];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = *reinterpret_cast<const uint4*>(wb + (long)i * (THREADS / 8) * (a.Kw * a.Cin) + kk);
  };
  auto st_set = [&](__bf16* base, const uint4* ra, const uint4* rb) {
    if (fold) {
      const float sc[8] = {asc0.x, asc0.y, asc0.z, asc0.w, asc1.x, asc1.y, asc1.z, asc1.w};
      const float sh[8] = {ash0.x, ash0.y, ash0.z, ash0.w, ash1.x, ash1.y, ash1.z, ash1.w};
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        bf16x8 v = __builtin_bit_cast(bf16x8, ra[i]);
        const bool ok = (aok >> i) & 1u;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok ? (__bf16)fmaxf(fmaf((float)v[e], sc[e], sh[e]), 0.f) : (__bf16)0.f;
        store_one(base, tid + i * THREADS, __builtin_bit_cast(uint4, v));
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) store_one(base, tid + i * THREADS, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) store_one(base + Cfg::A_EL, tid + i * THREADS, rb[i]);
  };
  auto mma = [&](const __bf16* As) {
    const __bf16* Bs = As + Cfg::A_EL;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wr * WM + i * 16 + (lane & 15)) * LDS_ROW + ks * 32 +
                                                 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wc * WN + j * 16 + (lane & 15)) * LDS_ROW + ks * 32 +
                                                  8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  __bf16* const L0 = lds;
  __bf16* const L1 = lds + (NBUF == 2 ? Cfg::A_EL + Cfg::B_EL : 0);
  if (nk > 0) {  // block-uniform (a phase without taps leaves acc = 0)
    ld_set(ra0, rb0, 0);
    st_set(L0, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      ld_set(ra0, rb0, kt + 1);
      if constexpr (NBUF == 2) {
        mma((kt & 1) ? L1 : L0);
        st_set((kt & 1) ? L0 : L1, ra0, rb0);
      } else {
        mma(L0);
        __syncthreads();  // every wave is done reading the buffer
        st_set(L0, ra0, rb0);
      }
      __syncthreads();
    }
  }
  fwd_epilogue<BM, BN, EPI, 2, (NBUF == 2)>(a, acc, smem, m0, n0, mt, MT, Lrow, M, P, ph);  // NBUF 1: 168 VGPRs
  if (a.tail && a.stats) ecg::bn_tail<THREADS>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, MT, a.Cout, mt, n0, BN, smem);
}

// LDS-DMA main loop (forward and non-dilated data-grad): every 16-byte piece of the A (activation rows) and B
// (weight rows) tiles goes global -> LDS with buffer_load ... lds (no register staging), two LDS stages, one
// barrier per 64-deep K step.  LDS image per operand: [row][64 bf16] (128-byte rows, no padding); 16-byte chunk
// cc of row r lives at chunk cc ^ ((r >> 1) & 7), so the 16 rows one ds_read_b128 lane group reads hit 16
// distinct 16-byte slots of the 256-byte bank row.  The DMA writes lane-linear (lane l -> row l/8, chunk l%8 of
// its 8-row piece), so the XOR is applied to the SOURCE chunk (MI355X guide rule 21).  Padding rows and the M
// tail use an out-of-range buffer offset: the range check lands zeros.
// The LDS-DMA goes through inline asm (buffer_load_dwordx4 ... offen lds, M0 = the wave's LDS destination):
// after a builtin LDS-DMA hipcc (ROCm 7.2) cannot tell a ring buffer's stages apart and waits vmcnt(0) before the
// next ds_read of ANY stage, draining every stage kept in flight (it defeated the 3-stage loops below).  From asm
// the loads are invisible to its wait-count pass: every loop here orders them with explicit (counted) vmcnt
// waits; compiler-placed waits for its own loads can only over-wait behind them (vmcnt retires in order).
typedef int srd_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ srd_t make_rsrc(const void* p, long bytes) {
  const unsigned long a = reinterpret_cast<unsigned long>(p);
  srd_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)((a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fff0000L ? bytes : 0x7fff0000L));  // num_records
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ unsigned lds_addr(const unsigned char* p) {
  return (unsigned)reinterpret_cast<unsigned long>((__attribute__((address_space(3))) const unsigned char*)p);
}
// one 16-B piece per lane into LDS at (wave-uniform) lds + 16 * lane; s_nop covers the M0 -> LDS-DMA hazard
__device__ __forceinline__ void dma16_at(srd_t r, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r),
               "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
__device__ __forceinline__ void dma16(srd_t r, unsigned voff, unsigned char* lds_piece) {
  dma16_at(r, voff, lds_addr(lds_piece));
}

// NWR = waves along M: 2 -> 4 waves (2x2), 4 -> 8 waves (4x2, 2 per SIMD at one workgroup per CU).  256-row
// tiles need one workgroup per CU (2 x 64 KB of stages at 256x256).  NST = LDS stages: 2 (one K step in flight
// while the MFMAs run) or 3 (two in flight; the 24 KB stages of the 128x64 tile still fit two workgroups per CU).
template <int BM, int BN, int EPI, int NWR, int NST = 2>
__global__ __launch_bounds__(128 * NWR, BM >= 256 ? 1 : 2) void conv1d_nlc_fwd_dma_kernel(FwdArgs a, int MT, int NT) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NW = Cfg::NW;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int AP = BM / (8 * NW), BP = BN / (8 * NW);  // 8-row DMA pieces per wave per stage
  static_assert(AP * 8 * NW == BM && BP * 8 * NW == BN, "tile rows must split into 8-row pieces over the waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int mt = wgid / NT, nt = wgid % NT;
  // Strided data-grad (in_dil = P > 1, stride 1): phase-decomposed as in conv1d_nlc_fwd_kernel - M tile mt belongs to
  // output phase ph (rows u = t * P + ph), whose taps k = k0 + j * P all hit real input rows t + j + (ph + k0 - pad) / P
  // (exact division), so the phase's K loop runs over its taps only and needs no per-row divisibility test.
  const int P = a.in_dil;
  const int ph = P > 1 ? mt / a.tpp : 0;
  const int m0 = (P > 1 ? mt - ph * a.tpp : mt) * BM, n0 = nt * BN;
  const int k0 = P > 1 ? ((a.pad - ph) % P + P) % P : 0;
  const int CB = a.Cin / BK, K = a.Kw * a.Cin;
  const int nk = (P > 1 ? (k0 < a.Kw ? (a.Kw - k0 + P - 1) / P : 0) : a.Kw) * CB;
  const int Lrow = P > 1 ? a.Lph : a.Lout;  // rows per sample of this kernel's (phase-local) M index
  const int M = a.B * Lrow;
  // The activation resource starts at the tile's first sample, so 32-bit offsets cover any batch size (the host
  // checks that one tile's sample span fits); records are capped below the out-of-range padding offset.
  const int b0 = m0 / Lrow;
  const long xrem = (long)(a.B - b0) * a.Lin * a.Cin * 2;
  const srd_t xr = make_rsrc(a.x + (long)b0 * a.Lin * a.Cin, xrem < 0x7fff0000L ? xrem : 0x7fff0000L);
  const srd_t wrs = make_rsrc(a.w, (long)a.Cout * K * 2);
  // this lane's rows: piece p = wv + 4*i covers tile rows 8p..8p+7; lane -> row 8p + lane/8, LDS chunk lane%8;
  // apos = the input row of tap step j = 0 (tap step j reads row apos + j)
  unsigned abase[AP];
  int apos[AP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int r = 8 * (wv + NW * i) + (lane >> 3), m = m0 + r;
    const int b = m / Lrow, t = m - b * Lrow;
    const int cs = (lane & 7) ^ ((r >> 1) & 7);  // source chunk landing in this lane's LDS slot
    const bool ok = m < M && (P == 1 || t * P + ph < a.Lout);
    abase[i] = ok ? (unsigned)(((long)(b - b0) * a.Lin * a.Cin + cs * 8) * 2) : 0u;
    apos[i] = ok ? (P > 1 ? t + (ph + k0 - a.pad) / P : t * a.stride - a.pad) : INT_MIN / 2;
  }
  unsigned wbase[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int r = 8 * (wv + NW * i) + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    wbase[i] = (unsigned)(((long)(n0 + r) * K + cs * 8) * 2);
  }
  auto issue = [&](int kt, int st) {
    const int j = kt / CB, c0 = (kt - j * CB) * BK;
    const int k = k0 + j * P;  // weight tap (P = 1: k = j)
    unsigned char* As = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int u = apos[i] + j;
      const unsigned voff = (u >= 0 && u < a.Lin) ? abase[i] + (unsigned)((u * a.Cin + c0) * 2) : 0x7ffffff0u;
      dma16(xr, voff, As + (wv + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i)
      dma16(wrs, wbase[i] + (unsigned)((k * a.Cin + c0) * 2), As + A_BYTES + (wv + NW * i) * 1024);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int st) {
    const unsigned char* As = smem + st * STAGE;
    const unsigned char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int cc = 4 * ks + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wr * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * 128 + ((cc ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = wc * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + n * 128 + ((cc ^ ((n >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (NST == 2) {
    if (nk > 0) {
      issue(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);  // lands during this step's MFMAs
        mma(kt & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next stage has landed (this wave's pieces) ...
        __syncthreads();                                  // ... for every wave, and nobody reads stage kt any more
      }
    }
  } else {
    // three stages: K steps kt+1 and kt+2 stream in while step kt's MFMAs run.  Each thread issues AP + BP
    // DMA loads per stage, so "stage kt landed" = at most one younger stage's loads still outstanding.
    constexpr int LPS = AP + BP;
    if (nk > 0) issue(0, 0);
    if (nk > 1) issue(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // stage kt landed for every wave; every wave is past mma(kt - 1).  A raw barrier: __syncthreads() would
      // emit vmcnt(0) and drain stage kt+1's DMA, which must stay in flight across it (guide: "Pipelining across
      // barriers"); the ds_reads of mma(kt - 1) retired with lgkmcnt(0)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) issue(kt + 2, (kt + 2) % 3);  // into the buffer mma(kt - 1) read
      mma(kt % 3);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();  // the epilogue reuses the stage buffers
  }
  fwd_epilogue<BM, BN, EPI, NWR, (BM < 256)>(a, acc, smem, m0, n0, mt, MT, Lrow, M, P, ph);
  if (a.tail && a.stats)
    ecg::bn_tail<Cfg::NTHR>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, MT, a.Cout, mt, n0, BN, smem);
}

// Multi-tile LDS-DMA forward (shapes with many more tiles than resident workgroups: the 64/128-channel ResNet
// stages, where one 128x64 tile is only 3-6 64-deep K steps).  Each workgroup walks M tiles mt = gm, gm + GM, ...
// of one column block as ONE stream of K steps: the next tile's first stage is DMA'd while this tile's last MFMAs
// and its epilogue run (the epilogue stages through an LDS region of its own), and the workgroup's statistics
// accumulate over its tiles into ONE partial row (row gm of GM) - so the BatchNorm tail's ticket, write-through
// drain and grid-wide hand-off are paid once per workgroup instead of once per tile.  Two workgroups per CU.
template <int BM, int BN, int EPI, int NWR = 2>
__global__ __launch_bounds__(128 * NWR, 2) void conv1d_nlc_fwd_dma_mt_kernel(FwdArgs a, int MT, int NT, int GM) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NW = Cfg::NW;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int AP = BM / (8 * NW), BP = BN / (8 * NW);
  static_assert(AP * 8 * NW == BM && BP * 8 * NW == BN, "tile rows must split into 8-row pieces over the waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* const eps = smem + 2 * STAGE;  // epilogue region (live while the next tile's stage lands)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int gm = wgid / NT, nt = wgid % NT;
  const int n0 = nt * BN;
  const int CB = a.Cin / BK, nk = a.Kw * CB, K = a.Kw * a.Cin;
  const int M = a.B * a.Lout;
  const int ntiles = gm < MT ? (MT - gm + GM - 1) / GM : 0;
  const int total = ntiles * nk;
  const srd_t wrs = make_rsrc(a.w, (long)a.Cout * K * 2);
  unsigned wbase[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int r = 8 * (wv + NW * i) + (lane >> 3);
    const int cs = (lane & 7) ^ ((r >> 1) & 7);
    wbase[i] = (unsigned)(((long)(n0 + r) * K + cs * 8) * 2);
  }
  // addressing of the tile being loaded (rebuilt when the K-step stream crosses into the next tile)
  int lt = -1;
  srd_t xr = wrs;
  unsigned abase[AP];
  int apos[AP];
  auto setup = [&](int j) {
    const int m0 = (gm + j * GM) * BM;
    const int b0 = m0 / a.Lout;
    const long xrem = (long)(a.B - b0) * a.Lin * a.Cin * 2;
    xr = make_rsrc(a.x + (long)b0 * a.Lin * a.Cin, xrem < 0x7fff0000L ? xrem : 0x7fff0000L);
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int r = 8 * (wv + NW * i) + (lane >> 3), m = m0 + r;
      const int b = m / a.Lout, t = m - b * a.Lout;
      const int cs = (lane & 7) ^ ((r >> 1) & 7);
      abase[i] = m < M ? (unsigned)(((long)(b - b0) * a.Lin * a.Cin + cs * 8) * 2) : 0u;
      apos[i] = m < M ? t * a.stride - a.pad : INT_MIN / 2;
    }
    lt = j;
  };
  auto issue = [&](int step, int st) {
    const int j = step / nk, kt = step - j * nk;
    if (j != lt) setup(j);
    const int k = kt / CB, c0 = (kt - k * CB) * BK;
    unsigned char* As = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int u = apos[i] + k;
      const unsigned voff = (u >= 0 && u < a.Lin) ? abase[i] + (unsigned)((u * a.Cin + c0) * 2) : 0x7ffffff0u;
      dma16(xr, voff, As + (wv + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i)
      dma16(wrs, wbase[i] + (unsigned)((k * a.Cin + c0) * 2), As + A_BYTES + (wv + NW * i) * 1024);
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int st) {
    const unsigned char* As = smem + st * STAGE;
    const unsigned char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int cc = 4 * ks + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wr * WM + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * 128 + ((cc ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = wc * WN + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + n * 128 + ((cc ^ ((n >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  EpiConst k;
  k.load<EPI == 1>(a, EpiLane<BN, NWR>::n(n0));
  if (total > 0) {  // block-uniform
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < total; ++s) {
      if (s + 1 < total) issue(s + 1, (s + 1) & 1);  // lands during this step's MFMAs (and epilogue)
      mma(s & 1);
      const int j = s / nk;
      if (s - j * nk == nk - 1) {  // tile j complete: store it (the epilogue region is not a stage)
        fwd_epi_tile<BM, BN, EPI, NWR>(a, acc, eps, k, (gm + j * GM) * BM, n0, a.Lout, M, 1, 0);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int q = 0; q < FN; ++q) acc[i][q] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (a.stats) {
    fwd_epi_stats<BM, BN, EPI, NWR>(a, eps, k, n0, gm, GM);
    if (a.tail) ecg::bn_tail<Cfg::NTHR>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, GM, a.Cout, gm, n0, BN, smem);
  }
}

inline bool conv_dma();
inline int conv_big();
inline int conv_mt();

// Tile choice: with the LDS-DMA loop (undilated input) 256x256 (8 waves of 64x128) when that gives >= 2 tiles
// per CU (one workgroup per CU; half the L2->LDS bytes per MAC of 128x128: 1.04 vs 0.87 PF/s on the
// ResNet layer4 shape, profiles/r1_resnet/cmb_p3_big*.log), [256x128 opt-in: measured slower], else 128x128 when that still gives >= 1 workgroup per CU (256 CUs), else 128x64,
// else 64x64.
inline void pick_fwd_tile(long M, int Cout, int in_dil, int* bm, int* bn) {
  // ECG_CONV_TILE=<bm>x<bn> forces one tile family wherever it applies (A/B experiments; read once)
  static int force_bm = -1, force_bn = 0;
  if (force_bm < 0) {
    const char* e = getenv("ECG_CONV_TILE");
    force_bm = 0;
    if (e && sscanf(e, "%dx%d", &force_bm, &force_bn) != 2) force_bm = 0;
  }
  if (force_bm > 0 && Cout % force_bn == 0 && (force_bm <= 128 || (in_dil == 1 && conv_dma()))) {
    *bm = force_bm;
    *bn = force_bn;
    return;
  }
  const long mt128 = (M + 127) / 128, mt256 = (M + 255) / 256;
  const int big = (in_dil == 1 && conv_dma()) ? conv_big() : 0;
  if (big >= 1 && Cout % 256 == 0 && mt256 * (Cout / 256) >= 512) {
    *bm = 256;
    *bn = 256;
  } else if (big >= 2 && Cout % 128 == 0 && mt256 * (Cout / 128) >= 512) {
    *bm = 256;
    *bn = 128;
  } else if (Cout == 128 && in_dil == 1 && conv_dma() && conv_mt() >= 2 && mt128 * 2 > 512) {
    *bm = 128;  // multi-tile 128x64 (ECG_CONV_MT=2)
    *bn = 64;
  } else if (Cout % 128 == 0 && mt128 * (Cout / 128) >= 256) {  // >= one tile per CU: 15.1 vs 17.7 us for 128x64
    *bm = 128;                                                      // at M=64512 C=128 (profiles/r2/conv_tiles.txt)
    *bn = 128;
  } else if (mt128 * (Cout / 64) >= 512) {
    *bm = 128;
    *bn = 64;
  } else {
    *bm = 64;
    *bn = 64;
  }
}

// ECG_CONV_MT=0|1|2: multi-tile forward workgroups (conv1d_nlc_fwd_dma_mt_kernel) for 128x64 tiles when the
// launch has more tiles than two resident workgroups per CU (1, default), and also for the 128-channel shapes
// that would otherwise take 128x128 tiles (2); 0 = one tile per workgroup.  Read once.
int g_conv_mt = -1;
inline int conv_mt() {
  if (g_conv_mt < 0) {
    const char* e = getenv("ECG_CONV_MT");
    g_conv_mt = e ? atoi(e) : 1;
  }
  return g_conv_mt;
}

// Workgroups along M of the multi-tile forward (0: the one-tile-per-workgroup kernels run).  A function of the
// shape and the tile alone, so the host can size the BatchNorm partial rows (ecg_conv1d_nlc_fwd_stat_tiles).
inline int fwd_mt_groups(long M, int Cout, int in_dil, int bm, int bn) {
  if (in_dil != 1 || !conv_dma() || conv_mt() == 0 || bm != 128 || bn != 64) return 0;
  const long MT = (M + bm - 1) / bm, NT = Cout / bn;
  const long slots = 2L * 256;  // two workgroups per CU
  if (MT * NT <= slots) return 0;
  const long tpw = (MT * NT + slots - 1) / slots;
  return (int)((MT + tpw - 1) / tpw);
}

// ECG_CONV_NBUF=1|2 selects the LDS buffering of the forward/data-grad kernel (read once; default 1).
inline int conv_nbuf() {
  static int nb = -1;
  if (nb < 0) {
    const char* e = getenv("ECG_CONV_NBUF");
    nb = (e && atoi(e) == 2) ? 2 : 1;
  }
  return nb;
}

// ECG_CONV_DMA=0 selects the register-staged main loop for every conv (read once; default: LDS-DMA loop when
// the input is not dilated).
inline bool conv_dma() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_CONV_DMA");
    v = (e && atoi(e) == 0) ? 0 : 1;
  }
  return v == 1;
}

// ECG_CONV_BIG=0|1|2: 256-row tiles (0: 128-row tiles only, 1 (default): + 256x256 forward, 2: + 256x128 forward
// and 256x256 weight-gradient); read
// once, overridable with ecg_conv1d_nlc_set_big (tests; plans built before a change keep their tiling).
int g_conv_big = -1;
inline int conv_big() {
  if (g_conv_big < 0) {
    const char* e = getenv("ECG_CONV_BIG");
    g_conv_big = e ? atoi(e) : 1;
  }
  return g_conv_big;
}

// ECG_CONV_NST=3 gives the 64-column tiles a three-stage loop (opt-in: ResNet1D-34 B=1024 4.64-4.66 vs 4.61
// ms/step with two stages, profiles/r2/resnet_conv_ab.txt - the K loops are not bound by DMA latency alone).
inline int conv_nst64() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_CONV_NST");
    v = (e && atoi(e) == 3) ? 3 : 2;
  }
  return v;
}

template <int BM, int BN, int EPI, int NST, int NWR = (BM >= 256 ? 4 : 2)>  // 256-row tiles: 8 waves of 64 x BN/2
int launch_fwd_dma_st(const FwdArgs& a, hipStream_t stream) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int STAGE_BYTES = NST * (BM + BN) * 128;
  constexpr int SMEM = STAGE_BYTES > Cfg::EP_BYTES ? STAGE_BYTES : Cfg::EP_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_dma_kernel<BM, BN, EPI, NWR, NST>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  FwdArgs b = a;
  int MT;
  if (a.in_dil > 1) {  // phase-decomposed strided data-grad (see the kernel)
    b.Lph = (a.Lout + a.in_dil - 1) / a.in_dil;
    b.tpp = (int)(((long)a.B * b.Lph + BM - 1) / BM);
    MT = a.in_dil * b.tpp;
  } else {
    MT = (int)(((long)a.B * a.Lout + BM - 1) / BM);
  }
  const int NT = a.Cout / BN;
  hipLaunchKernelGGL((conv1d_nlc_fwd_dma_kernel<BM, BN, EPI, NWR, NST>), dim3((unsigned)(MT * NT)), dim3(Cfg::NTHR),
                     SMEM, stream, b, MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

// ECG_CONV_NST=3: 64-column tiles take three LDS stages (two workgroups per CU still fit: 2 x 72 KB at 128x64).
// ECG_CONV_V128=1|2|3: the 128x128 tile with three stages (one workgroup per CU) | eight waves of 32x64 | both.
inline int conv_v128() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_CONV_V128");
    v = e ? atoi(e) : 0;
  }
  return v;
}

template <int BM, int BN, int EPI>
int launch_fwd_dma_mt(const FwdArgs& a, int GM, hipStream_t stream) {
  using Cfg = FwdCfg<BM, BN, 2>;
  constexpr int SMEM = 2 * (BM + BN) * 128 + Cfg::EP_BYTES;
  static_assert(2 * SMEM <= 160 * 1024, "two workgroups per CU");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_dma_mt_kernel<BM, BN, EPI, 2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int MT = (int)(((long)a.B * a.Lout + BM - 1) / BM), NT = a.Cout / BN;
  hipLaunchKernelGGL((conv1d_nlc_fwd_dma_mt_kernel<BM, BN, EPI, 2>), dim3((unsigned)(GM * NT)), dim3(Cfg::NTHR), SMEM,
                     stream, a, MT, NT, GM);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

template <int BM, int BN, int EPI>
int launch_fwd_dma(const FwdArgs& a, hipStream_t stream) {
  if constexpr (BM == 128 && BN == 64) {
    const int GM = fwd_mt_groups((long)a.B * a.Lout, a.Cout, a.in_dil, BM, BN);
    if (GM > 0) return launch_fwd_dma_mt<BM, BN, EPI>(a, GM, stream);
  }
  if constexpr (BN == 64 && BM <= 128) {
    if (conv_nst64() == 3) return launch_fwd_dma_st<BM, BN, EPI, 3>(a, stream);
  }
  if constexpr (BM == 256 && BN == 128) {  // ECG_CONV_NST256=3: three LDS stages (3 x 48 KB) for the 8-wave tile
    static const int nst = [] {
      const char* e = getenv("ECG_CONV_NST256");
      return e && atoi(e) == 3 ? 3 : 2;
    }();
    if (nst == 3) return launch_fwd_dma_st<BM, BN, EPI, 3>(a, stream);
  }
  if constexpr (BN == 128 && BM == 128) {
    switch (conv_v128()) {
      case 1: return launch_fwd_dma_st<BM, BN, EPI, 3, 2>(a, stream);
      case 2: return launch_fwd_dma_st<BM, BN, EPI, 2, 4>(a, stream);
      case 3: return launch_fwd_dma_st<BM, BN, EPI, 3, 4>(a, stream);
      default: break;
    }
  }
  return launch_fwd_dma_st<BM, BN, EPI, 2>(a, stream);
}

template <int BM, int BN, int EPI, int NBUF>
int launch_fwd_cfg(const FwdArgs& a, hipStream_t stream) {
  using Cfg = FwdCfg<BM, BN>;
  constexpr int SMEM = Cfg::smem(NBUF);
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_kernel<BM, BN, EPI, NBUF>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  FwdArgs b = a;
  int MT;
  if (a.in_dil > 1) {
    b.Lph = (a.Lout + a.in_dil - 1) / a.in_dil;
    b.tpp = (int)(((long)a.B * b.Lph + BM - 1) / BM);
    MT = a.in_dil * b.tpp;
  } else {
    MT = (int)(((long)a.B * a.Lout + BM - 1) / BM);
  }
  const int NT = a.Cout / BN;
  hipLaunchKernelGGL((conv1d_nlc_fwd_kernel<BM, BN, EPI, NBUF>), dim3((unsigned)(MT * NT)), dim3(THREADS), SMEM,
                     stream, b, MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

// ECG_CONV_DMA_DIL=0 keeps the strided (phase-decomposed) data-grads on the register-staged loop (read once;
// default: LDS-DMA loop, two stages).
int g_conv_dma_dil = -1;
inline bool conv_dma_dil() {
  if (g_conv_dma_dil < 0) {
    const char* e = getenv("ECG_CONV_DMA_DIL");
    g_conv_dma_dil = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_conv_dma_dil == 1;
}

template <int BM, int BN>
int launch_fwd(const FwdArgs& a, hipStream_t stream) {
  // the DMA loop addresses bytes with 32-bit buffer offsets from the tile's first sample
  const int Lrow = a.in_dil > 1 ? (a.Lout + a.in_dil - 1) / a.in_dil : a.Lout;
  const bool dma_ok = (a.in_dil == 1 || (conv_dma_dil() && a.stride == 1 && BM <= 128)) &&
                      (long)(BM / Lrow + 2) * a.Lin * a.Cin * 2 < 0x7fff0000L &&
                      (long)a.Cout * a.Kw * a.Cin * 2 < 0x7fff0000L;
  if (conv_dma() && dma_ok && a.in_dil > 1)  // two stages, one tile per workgroup
    return a.stat_mode == 1 ? launch_fwd_dma_st<BM, BN, 1, 2>(a, stream) : launch_fwd_dma_st<BM, BN, 0, 2>(a, stream);
  if (conv_dma() && dma_ok)
    return a.stat_mode == 1 ? launch_fwd_dma<BM, BN, 1>(a, stream) : launch_fwd_dma<BM, BN, 0>(a, stream);
  if (a.stats && fwd_mt_groups((long)a.B * a.Lout, a.Cout, a.in_dil, BM, BN) > 0)
    return ecg::kBadArg;  // the host sized the partial rows for the multi-tile kernel
  if constexpr (BM > 128) return ecg::kBadArg;  // 256-row tiles exist only as DMA kernels (the picker ensures it)
  else {
    if (conv_nbuf() == 2)
      return a.stat_mode == 1 ? launch_fwd_cfg<BM, BN, 1, 2>(a, stream) : launch_fwd_cfg<BM, BN, 0, 2>(a, stream);
    return a.stat_mode == 1 ? launch_fwd_cfg<BM, BN, 1, 1>(a, stream) : launch_fwd_cfg<BM, BN, 0, 1>(a, stream);
  }
}

// ------------------------------------------------------------------------------------------- weight grad
// Division by a runtime-invariant divisor without the ~40-instruction integer divide (Granlund-Montgomery):
// q = (umulhi(n, m) + n) >> s, exact for 0 <= n < 2^31.
struct FastDiv {
  uint32_t m;
  int s;
  int d;
};
inline FastDiv make_fastdiv(int d) {
  int s = 0;
  while ((1u << s) < (uint32_t)d) ++s;
  const uint64_t m = ((uint64_t)1 << 32) * (((uint64_t)1 << s) - (uint64_t)d) / (uint64_t)d + 1;
  return FastDiv{(uint32_t)m, s, d};
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)(((uint64_t)__umulhi((uint32_t)n, f.m) + (uint32_t)n) >> f.s);
}

struct WgradArgs {
  const __bf16* dy;  // [B][Lout][Cout]
  const __bf16* x;   // [B][Lin][Cin]
  float* part;       // [splits][Cout][Kw*Cin] fp32 partials
  int B, Lin, Cin, Lout, Cout, Kw, stride, pad, chunks_per_split;
  FastDiv lout;  // r -> (b, t) = divmod(r, Lout)
};


__device__ __forceinline__ s16x4 tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// Tiles BM (C_out) x BN (taps*C_in), reduction over 64-row chunks of (b,t); both LDS images are [r][col] and
// the MFMA fragments come out of them with transposing reads.  Register prefetch (the next chunk's global
// loads are in flight during this chunk's MFMAs) into ONE LDS buffer (two barriers per chunk), which keeps
// three workgroups resident per CU; 1-D grid, split-major so the workgroups on one XCD share the same
// activation rows; partial tiles leave through an LDS-staged float4 epilogue.
// NWR = waves along C_out (2 x NWR waves): 2 for the 128/64 tiles (3 workgroups / CU), 4 for 256x256 (8 waves of
// 64 x 128, one workgroup / CU, half the L2->LDS bytes per MAC).
template <int BM, int BN, int NWR = 2>
struct WgCfg {
  static constexpr int NW = 2 * NWR, NTHR = 64 * NW;
  static constexpr int WM = BM / NWR, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  static constexpr int ROW_A = BM + 4, ROW_B = BN + 4;     // bf16 per LDS row (8-B aligned tr reads)
  static constexpr int NA = 8 * BM / NTHR, NB = 8 * BN / NTHR;  // 16-B loads per thread per chunk
  static constexpr int A_EL = 64 * ROW_A, B_EL = 64 * ROW_B;
  static constexpr int STAGE_BYTES = (A_EL + B_EL) * 2;  // one buffer (two barriers per chunk)
  static constexpr int EP_LD = WN + 4;
  static constexpr int EP_BYTES = NW * (WM / 2) * EP_LD * 4;  // epilogue staged in two halves
  static constexpr int SMEM = STAGE_BYTES > EP_BYTES ? STAGE_BYTES : EP_BYTES;
};

__device__ __forceinline__ void st_split(__bf16* p, uint4 v) {  // 8-B aligned 16-B store
  *reinterpret_cast<uint2*>(p) = make_uint2(v.x, v.y);
  *reinterpret_cast<uint2*>(p + 4) = make_uint2(v.z, v.w);
}

// Weight-gradient epilogue shared by both main loops: partial[split][co][n] through an LDS fp32 image (two halves
// of WM/2 rows per wave), float4 row stores.  Starts with a barrier: the main loop's LDS may still be read.
template <int BM, int BN, int NWR>
__device__ __forceinline__ void wgrad_epilogue(const WgradArgs& a, f32x4 (&acc)[BM / NWR / 16][BN / 32],
                                               unsigned char* smem, int split, int co0, int n0) {
  using Cfg = WgCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  constexpr int EP_LD = Cfg::EP_LD, HR = WM / 2;
  float* ep = reinterpret_cast<float*>(smem) + wv * HR * EP_LD;
  constexpr int C4 = WN / 4, RSTEP = 64 / C4;
  const int c4 = lane % C4, rs = lane / C4;
  const long N = (long)a.Kw * a.Cin;
  float* out = a.part + (long)split * a.Cout * N;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();  // main loop / previous half done with the LDS
#pragma unroll
    for (int i = 0; i < FM / 2; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          ep[(i * 16 + 4 * (lane >> 4) + qq) * EP_LD + j * 16 + (lane & 15)] = acc[h * (FM / 2) + i][j][qq];
    __syncthreads();
#pragma unroll 4
    for (int r = rs; r < HR; r += RSTEP) {
      const float4 v = *reinterpret_cast<const float4*>(ep + r * EP_LD + c4 * 4);
      *reinterpret_cast<float4*>(out + (long)(co0 + wr * WM + h * HR + r) * N + n0 + wc * WN + c4 * 4) = v;
    }
  }
}

template <int BM, int BN, int NWR>
__global__ __launch_bounds__(128 * NWR, NWR == 2 ? 3 : 1) void conv1d_nlc_wgrad_kernel(WgradArgs a, int TM, int TN,
                                                                                       int splits) {
  using Cfg = WgCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NA = Cfg::NA, NB = Cfg::NB;
  constexpr int THREADS = Cfg::NTHR;  // shadows the 4-wave default
  constexpr int ROW_A = Cfg::ROW_A, ROW_B = Cfg::ROW_B;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __bf16* const lds = reinterpret_cast<__bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tiles = TM * TN;
  const int split = wgid / tiles, tile = wgid % tiles;
  const int co0 = (tile / TN) * BM, n0 = (tile % TN) * BN;
  const int k = n0 / a.Cin, c0 = n0 % a.Cin;  // the BN columns lie inside one tap
  const int R = a.B * a.Lout;
  const int nchunks = (R + 63) / 64;
  const int ch0 = split * a.chunks_per_split;
  const int ch1 = min(nchunks, ch0 + a.chunks_per_split);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_a = [&](int ch, int e) -> uint4 {  // dy[r][co0 + 8*part]
    const int row = e / (BM / 8), part = e % (BM / 8);
    const int r = ch * 64 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < R) v = *reinterpret_cast<const uint4*>(a.dy + (long)r * a.Cout + co0 + part * 8);
    return v;
  };
  auto load_b = [&](int ch, int e) -> uint4 {  // x[b, t*s + k - p][c0 + 8*part]
    const int row = e / (BN / 8), part = e % (BN / 8);
    const int r = ch * 64 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < R) {
      const int b = fdiv(r, a.lout), t = r - b * a.Lout;
      const int u = t * a.stride + k - a.pad;
      if (u >= 0 && u < a.Lin) v = *reinterpret_cast<const uint4*>(a.x + ((long)b * a.Lin + u) * a.Cin + c0 + part * 8);
    }
    return v;
  };
  auto store_ab = [&](__bf16* base, const uint4* ra, const uint4* rb) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = tid + i * THREADS;
      st_split(base + (e / (BM / 8)) * ROW_A + (e % (BM / 8)) * 8, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = tid + i * THREADS;
      st_split(base + Cfg::A_EL + (e / (BN / 8)) * ROW_B + (e % (BN / 8)) * 8, rb[i]);
    }
  };

  if (ch0 < ch1) {  // block-uniform
    uint4 ra[NA], rb[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = load_a(ch0, tid + i * THREADS);
#pragma unroll
    for (int i = 0; i < NB; ++i) rb[i] = load_b(ch0, tid + i * THREADS);
    store_ab(lds, ra, rb);
    __syncthreads();
    const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, h = lane >> 4;
    for (int ch = ch0; ch < ch1; ++ch) {
      const int cn = ch + 1 < ch1 ? ch + 1 : ch;
#pragma unroll
      for (int i = 0; i < NA; ++i) ra[i] = load_a(cn, tid + i * THREADS);
#pragma unroll
      for (int i = 0; i < NB; ++i) rb[i] = load_b(cn, tid + i * THREADS);
      const __bf16* As = lds;
      const __bf16* Bs = As + Cfg::A_EL;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {  // two 32-deep k-steps over r
        typedef short s16x8v __attribute__((ext_vector_type(8)));
        bf16x8 af[FM], bfr[FN];
        const int rr = ks * 32 + 8 * h + q;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int col = wr * WM + i * 16 + p4;
          const s16x4 lo = tr16(As + rr * ROW_A + col);
          const s16x4 hi = tr16(As + (rr + 4) * ROW_A + col);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wc * WN + j * 16 + p4;
          const s16x4 lo = tr16(Bs + rr * ROW_B + col);
          const s16x4 hi = tr16(Bs + (rr + 4) * ROW_B + col);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();  // every wave is done reading the buffer
      store_ab(lds, ra, rb);
      __syncthreads();
    }
  }
  wgrad_epilogue<BM, BN, NWR>(a, acc, smem, split, co0, n0);
}

// LDS-DMA weight-gradient main loop (128x128 tiles, 4 waves): both 64-row operand images go global -> LDS with
// buffer_load ... lds (no VGPR staging: the register-staged loop spends more LDS cycles on its ds_write_b64
// stores than on the MFMA operand reads), two stages, one barrier per 64-row chunk.  Images are dense
// [r][128] bf16 (256-B rows); 16-B chunk c of row r is stored at chunk c ^ swz(r), swz(r) = 2 * ((r & 3) |
// ((r >> 3) & 1) << 2), so the 8 rows {q, 8+q} x 32 B one 32-lane ds_read_b64_tr_b16 group touches land on 16
// distinct 16-B slots of the 256-B bank row.  The DMA writes lane-linear, so the XOR is applied to the SOURCE
// chunk.  Rows past R and out-of-range taps use an out-of-range buffer offset (zeros land).  Resources are
// rebased at the split's first row / sample: 32-bit offsets cover any batch (the host checks the span).
__device__ __forceinline__ int wg_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

template <int BM, int BN, int NWR>
__global__ __launch_bounds__(128 * NWR, NWR == 2 ? 2 : 1) void conv1d_nlc_wgrad_dma_kernel(WgradArgs a, int TM, int TN,
                                                                                           int splits) {
  static_assert(BM == BN && (BM == 128 || BM == 256), "square tiles with >= 16 chunks per row");
  using Cfg = WgCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NW = Cfg::NW;
  constexpr int RA = BM * 2, RB = BN * 2;  // bytes per image row
  constexpr int A_BYTES = 64 * RA, STAGE = 64 * (RA + RB);
  constexpr int AP = A_BYTES / 1024 / NW, BP = 64 * RB / 1024 / NW;  // 1-KB DMA pieces per wave per stage
  constexpr int RPP = 1024 / RA;                                      // rows per piece (4 or 2)
  constexpr int SH = RA == 256 ? 4 : 5, SLOT = RA / 16 - 1;           // lane -> (row in piece, 16-B slot)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tiles = TM * TN;
  const int split = wgid / tiles, tile = wgid % tiles;
  const int co0 = (tile / TN) * BM, n0 = (tile % TN) * BN;
  const int k = n0 / a.Cin, c0 = n0 % a.Cin;  // the BN columns lie inside one tap
  const int R = a.B * a.Lout;
  const int nchunks = (R + 63) / 64;
  const int ch0 = split * a.chunks_per_split;
  const int ch1 = min(nchunks, ch0 + a.chunks_per_split);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (ch0 < ch1) {  // block-uniform
    const int r0 = ch0 * 64, b0 = r0 / a.Lout;
    const long dyrem = (long)(R - r0) * a.Cout * 2, xrem = (long)(a.B - b0) * a.Lin * a.Cin * 2;
    const srd_t dyr = make_rsrc(a.dy + (long)r0 * a.Cout, dyrem < 0x7fff0000L ? dyrem : 0x7fff0000L);
    const srd_t xr = make_rsrc(a.x + (long)b0 * a.Lin * a.Cin, xrem < 0x7fff0000L ? xrem : 0x7fff0000L);
    // this lane's image rows and source chunks (piece p = wv + 4*i covers rows RPP*p .. RPP*p + RPP-1)
    int arow[AP], asrc[BP > AP ? BP : AP], brow[BP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      arow[i] = RPP * (wv + NW * i) + (lane >> SH);
      asrc[i] = (lane & SLOT) ^ wg_swz(arow[i]);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) brow[i] = RPP * (wv + NW * i) + (lane >> SH);
    auto issue = [&](int ch, int st) {
      unsigned char* As = smem + st * STAGE;
      const int rel = (ch - ch0) * 64;
#pragma unroll
      for (int i = 0; i < AP; ++i) {
        const int r = rel + arow[i];
        const unsigned voff = r0 + r < R ? (unsigned)(((long)r * a.Cout + co0 + asrc[i] * 8) * 2) : 0x7ffffff0u;
        dma16(dyr, voff, As + (wv + NW * i) * 1024);
      }
#pragma unroll
      for (int i = 0; i < BP; ++i) {
        const int rg = r0 + rel + brow[i];
        const int b = fdiv(rg, a.lout), t = rg - b * a.Lout;
        const int u = t * a.stride + k - a.pad;
        const int src = (lane & SLOT) ^ wg_swz(brow[i]);
        const unsigned voff = (rg < R && u >= 0 && u < a.Lin)
                                  ? (unsigned)((((long)(b - b0) * a.Lin + u) * a.Cin + c0 + src * 8) * 2)
                                  : 0x7ffffff0u;
        dma16(xr, voff, As + A_BYTES + (wv + NW * i) * 1024);
      }
    };
    const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, h = lane >> 4;
    auto tr_at = [&](const unsigned char* img, int RB_, int rr, int col) -> s16x4 {
      return tr16(reinterpret_cast<const __bf16*>(img + rr * RB_ + ((((col >> 3) ^ wg_swz(rr))) << 4) +
                                                  ((col & 7) << 1)));
    };
    auto mma = [&](int st) {
      const unsigned char* As = smem + st * STAGE;
      const unsigned char* Bs = As + A_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {  // two 32-deep k-steps over r
        typedef short s16x8v __attribute__((ext_vector_type(8)));
        bf16x8 af[FM], bfr[FN];
        const int rr = ks * 32 + 8 * h + q;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int col = wr * WM + i * 16 + p4;
          const s16x4 lo = tr_at(As, RA, rr, col), hi = tr_at(As, RA, rr + 4, col);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wc * WN + j * 16 + p4;
          const s16x4 lo = tr_at(Bs, RB, rr, col), hi = tr_at(Bs, RB, rr + 4, col);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    issue(ch0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = ch0; ch < ch1; ++ch) {
      const int st = (ch - ch0) & 1;
      if (ch + 1 < ch1) issue(ch + 1, st ^ 1);  // lands during this chunk's MFMAs
      mma(st);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  wgrad_epilogue<BM, BN, NWR>(a, acc, smem, split, co0, n0);
}

// ------------------------------------------------------------------ weight-resident tap-shared forward (WR)
// Stride-1, pad-1, 3-tap convs with C_in in {64, 128, 256} (the forward and the data-grad of every 3-tap conv of a
// ResNet stage except its strided first one: in_dil 1, Lin == Lout).  One workgroup per CU (4 waves):
//   * the weights of its BN output channels, all 3 taps x C_in, stay resident in LDS for the workgroup's life
//     (loaded once; the one-tap kernels restream a weight tile per 64-deep K step of every M tile);
//   * per 128-row M tile and 64-channel chunk it stages x[m0 - 1, m0 + 135) ONCE (LDS-DMA, 3-stage ring, counted
//     vmcnt, raw barriers); the 3 taps read that image at row offsets 0, 1, 2.
// So a CU moves ~17 KB of activations per 128 x BN x 192 MACs instead of 32 KB per 128 x 128 x 64.
// Orientation out^T[co][m] = W[co][kk] x X^T[kk][m] (A = weights, B = activations): a lane's accumulator holds 4
// consecutive channels of ONE output row, so the epilogue is 8-byte loads / stores straight from registers and
// the BatchNorm partials reduce over rows with DPP - the LDS holds only the weights and the activation ring.
// Sample boundaries: a lane's B fragment is one output row; it is zeroed for tap 0 at t == 0 and for tap 2 at
// t == L - 1 (the shifted row belongs to the neighbouring sample).
// Work split: workgroup (gm, nt) of a GM x NT grid owns channels [nt * BN, + BN) and M tiles gm, gm + GM, ...; its
// statistics accumulate over those tiles into partial row gm of GM (the rows the BatchNorm tail reduces).
// Weight image: row co = 3 * C_in bf16 (tap-major), padded to a multiple of 256 B; 16-B chunk ch of row co is
// stored at (ch & ~15) | ((ch & 15) ^ (co & 15)), so the 16 rows x 2 chunk offsets of a ds_read_b128 lane group
// land on 16 distinct slots.  Activation image: [136 rows][64] bf16, chunk cc of row r at cc ^ ((r >> 1) & 7).
__device__ __forceinline__ float wr_row16_sum(float v) {  // lane 15 of each 16-lane DPP row ends with the row sum
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

constexpr int WR_BM = 128;
constexpr int WR_XSTAGE = 136 * 128;  // activation image bytes per stage (rows m0-1 .. m0+134, 130 used)

template <int BN, int NCH>
struct WrCfg {
  static constexpr int CIN = 64 * NCH;
  static constexpr int WROW = (3 * CIN * 2 + 255) / 256 * 256;  // weight-image row bytes
  static constexpr int W_BYTES = BN * WROW;
  static constexpr int FI = BN / 16;                             // co fragments per wave
  static constexpr int SRED_BYTES = 4 * 3 * BN * 4;              // [wave][stat][BN] partials
  static constexpr int smem(int nst) { return W_BYTES + nst * WR_XSTAGE + SRED_BYTES; }
};

template <int BN, int NCH, int EPI, int NST>
__global__ __launch_bounds__(256, 1) void conv1d_nlc_fwd_wr_kernel(FwdArgs a, int MT, int NT, int GM) {
  using Cfg = WrCfg<BN, NCH>;
  constexpr int CIN = Cfg::CIN, WROW = Cfg::WROW, FI = Cfg::FI;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* const wimg = smem;
  unsigned char* const xring = smem + Cfg::W_BYTES;
  float* const sred = reinterpret_cast<float*>(smem + Cfg::W_BYTES + NST * WR_XSTAGE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, ml = lane & 15;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int gm = wgid / NT, nt = wgid % NT;  // the NT workgroups of one gm (same activation rows) share an XCD
  const int n0 = nt * BN;
  const int L = a.Lout;
  const int M = a.B * L;
  const int ntiles = gm < MT ? (MT - gm + GM - 1) / GM : 0;
  const int total = ntiles * NCH;
  const srd_t xr = make_rsrc(a.x, (long)M * CIN * 2);
  const unsigned ring0 = lds_addr(xring);
  const int prow = lane >> 3;
  // stage s = (tile j, chunk c): rows m0 - 1 + [0, 136) of channels [64c, 64c + 64); 5 DMA instructions per wave
  auto issue = [&](int s, int st) {
    const int j = s / NCH, c = s - j * NCH;
    const int m0 = (gm + j * GM) * WR_BM;
    const unsigned base = ring0 + st * WR_XSTAGE;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = wv + 4 * u, row = 8 * p + prow, r = m0 - 1 + row;
      const int src = (lane & 7) ^ ((row >> 1) & 7);
      dma16_at(xr, (r >= 0 && r < M) ? (unsigned)((r * CIN + c * 64 + src * 8) * 2) : 0x7ffffff0u, base + p * 1024);
    }
    {  // piece 16 (rows 128..135): lanes 16w .. 16w + 15 of wave w write rows 128 + 2w, 129 + 2w
      const int row = 128 + prow, r = m0 - 1 + row;
      const int src = (lane & 7) ^ ((row >> 1) & 7);
      if ((lane >> 4) == wv)
        dma16_at(xr, (r >= 0 && r < M) ? (unsigned)((r * CIN + c * 64 + src * 8) * 2) : 0x7ffffff0u,
                 base + 16 * 1024);
    }
  };
#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < total) issue(i, i);
  // resident weights (plain 16-B loads -> swizzled ds_write_b128; once per workgroup)
  {
    constexpr int RCH = 3 * CIN / 8;  // 16-B chunks per weight row
    constexpr int LPT = BN * RCH / 256;
    static_assert(LPT * 256 == BN * RCH, "weight image must split evenly over the threads");
    uint4 wv4[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int q = tid + 256 * u, co = q / RCH, ch = q - co * RCH;
      wv4[u] = *reinterpret_cast<const uint4*>(a.w + (long)(n0 + co) * (3 * CIN) + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int q = tid + 256 * u, co = q / RCH, ch = q - co * RCH;
      const int phys = (ch & ~15) | ((ch & 15) ^ (co & 15));
      *reinterpret_cast<uint4*>(wimg + co * WROW + phys * 16) = wv4[u];
    }
  }
  __syncthreads();
  f32x4 acc[FI][2];
#pragma unroll
  for (int i = 0; i < FI; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float st1[FI][4], st2[FI][4], st3[FI][4];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) st1[i][q] = st2[i][q] = st3[i][q] = 0.f;
  const bool ds = EPI == 1 && a.szd != nullptr;
  bool v0[2] = {true, true}, v2[2] = {true, true};  // this lane's rows: tap 0 / tap 2 inside the sample
  for (int s = 0; s < total; ++s) {
    const int ahead = min(NST - 2, total - 1 - s);
    if constexpr (NST >= 4) {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (NST == 3) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NST - 1 < total) issue(s + NST - 1, (s + NST - 1) % NST);  // into the stage read at s - 1
    const int j = s / NCH, c = s - j * NCH;
    const int m0 = (gm + j * GM) * WR_BM;
    if (c == 0) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int m = m0 + 32 * wv + 16 * jj + ml;
        const int t = m - (m / L) * L;
        v0[jj] = t != 0;
        v2[jj] = t != L - 1;
      }
    }
    const unsigned char* ximg = xring + (s % NST) * WR_XSTAGE;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 wf[FI], xf[2];
        const int ch = k * 8 * NCH + c * 8 + ks * 4 + h;
#pragma unroll
        for (int i = 0; i < FI; ++i) {
          const int co = 16 * i + ml;
          const int phys = (ch & ~15) | ((ch & 15) ^ (co & 15));
          wf[i] = *reinterpret_cast<const bf16x8*>(wimg + co * WROW + phys * 16);
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int row = 32 * wv + 16 * jj + ml + k;
          const int cc = (ks * 4 + h) ^ ((row >> 1) & 7);
          uint4 v = *reinterpret_cast<const uint4*>(ximg + row * 128 + cc * 16);
          const bool ok = k == 1 || (k == 0 ? v0[jj] : v2[jj]);
          if (!ok) v = make_uint4(0u, 0u, 0u, 0u);
          xf[jj] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[jj], acc[i][jj], 0, 0, 0);
      }
    }
    if (c == NCH - 1) {  // tile j complete: epilogue from registers (rows m, 4 channels per lane and fragment)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int m = m0 + 32 * wv + 16 * jj + ml;
        if (m < M) {
#pragma unroll
          for (int i = 0; i < FI; ++i) {
            const int co = n0 + 16 * i + 4 * h;
            const long o = (long)m * a.Cout + co;
            float v[4] = {acc[i][jj][0], acc[i][jj][1], acc[i][jj][2], acc[i][jj][3]};
            if (a.bias) {
              const float4 b4 = *reinterpret_cast<const float4*>(a.bias + co);
              v[0] += b4.x; v[1] += b4.y; v[2] += b4.z; v[3] += b4.w;
            }
            if (a.add) {
              const bf16x4 ad = *reinterpret_cast<const bf16x4*>(a.add + o);
              if (a.add_mask) {
                const bf16x4 mk = *reinterpret_cast<const bf16x4*>(a.add_mask + o);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)mk[e] > 0.f ? (float)ad[e] : 0.f;
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)ad[e];
              }
            }
            bf16x4 zz;
            if constexpr (EPI == 1) {
              zz = *reinterpret_cast<const bf16x4*>(a.sz + o);
              if (a.mscale != nullptr) {  // the mask the BN_ACT pass stored, recomputed from sz
                const float4 sc = *reinterpret_cast<const float4*>(a.mscale + co);
                const float4 sh = *reinterpret_cast<const float4*>(a.mshift + co);
                const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const __bf16 act = (__bf16)fmaxf(fmaf((float)zz[e], scv[e], shv[e]), 0.f);
                  v[e] = (float)act > 0.f ? v[e] : 0.f;
                }
              } else if (a.smask != nullptr) {
                const bf16x4 mk = *reinterpret_cast<const bf16x4*>(a.smask + o);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (float)mk[e] > 0.f ? v[e] : 0.f;
              }
            }
            bf16x4 outv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (a.relu) v[e] = fmaxf(v[e], 0.f);
              outv[e] = (__bf16)v[e];
              v[e] = (float)outv[e];
            }
            *reinterpret_cast<bf16x4*>(a.y + o) = outv;
            if (a.stats) {
              if constexpr (EPI == 1) {
                const float4 mu4 = *reinterpret_cast<const float4*>(a.smean + co);
                const float4 rs4 = *reinterpret_cast<const float4*>(a.srstd + co);
                const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, rs[4] = {rs4.x, rs4.y, rs4.z, rs4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  st1[i][e] += v[e];
                  st2[i][e] += v[e] * ((float)zz[e] - mu[e]) * rs[e];
                }
                if (ds) {
                  const bf16x4 zd = *reinterpret_cast<const bf16x4*>(a.szd + o);
                  const float4 md4 = *reinterpret_cast<const float4*>(a.smean_d + co);
                  const float4 rd4 = *reinterpret_cast<const float4*>(a.srstd_d + co);
                  const float md[4] = {md4.x, md4.y, md4.z, md4.w}, rd[4] = {rd4.x, rd4.y, rd4.z, rd4.w};
#pragma unroll
                  for (int e = 0; e < 4; ++e) st3[i][e] += v[e] * ((float)zd[e] - md[e]) * rd[e];
                }
              } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  st1[i][e] += v[e];
                  st2[i][e] += v[e] * v[e];
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < FI; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the activation ring is dead from here (bn_tail scratch)
  if (a.stats) {  // block-uniform
    const int NS = ds ? 3 : 2;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float s1 = wr_row16_sum(st1[i][e]), s2 = wr_row16_sum(st2[i][e]);
        const float s3 = ds ? wr_row16_sum(st3[i][e]) : 0.f;
        if (ml == 15) {
          sred[(wv * 3 + 0) * BN + 16 * i + 4 * h + e] = s1;
          sred[(wv * 3 + 1) * BN + 16 * i + 4 * h + e] = s2;
          sred[(wv * 3 + 2) * BN + 16 * i + 4 * h + e] = s3;
        }
      }
    __syncthreads();
    for (int p = tid; p < NS * BN; p += 256) {
      const int st = p / BN, cl = p - st * BN;
      const float v = ((sred[(0 * 3 + st) * BN + cl] + sred[(1 * 3 + st) * BN + cl]) + sred[(2 * 3 + st) * BN + cl]) +
                      sred[(3 * 3 + st) * BN + cl];
      float* dst = a.stats + ((long)st * GM + gm) * a.Cout + n0 + cl;
      if (a.tail)
        ecg::st_sc1(dst, v);  // handed to the tail's last arriver inside this launch (write-through)
      else
        *dst = v;
    }
    if (a.tail) ecg::bn_tail<256>(a.tail, a.stats, NS, GM, a.Cout, gm, n0, BN, xring);
  }
}

// ECG_CONV_WR = largest C_in that takes the weight-resident tap-shared forward (read once; default 0 = off).
// Measured on MI355X (profiles/r3/conv_wr_ab.txt): in isolation 13.2 vs 15.6 us at 64 channels but 18.2 vs 15.6
// (128) and 31.7 vs 22.0 (256) - one 4-wave workgroup per CU leaves the LDS-read -> MFMA latency of each k-step
// exposed - and inside the ResNet1D-34 step 3.84-4.35 vs 3.75-3.77 ms: its CU-filling persistent grid also
// crowds out the side-lane weight gradients.  Kept as an opt-in variant.
inline int conv_wr() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_CONV_WR");
    v = e ? atoi(e) : 0;
  }
  return v;
}
inline int wr_bn(int Cin) { return Cin == 128 ? 128 : 64; }
inline bool wr_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad, int in_dil) {
  return Cin <= conv_wr() && Kw == 3 && stride == 1 && pad == 1 && in_dil == 1 && Lin == Lout && Lout >= 2 &&
         (Cin == 64 || Cin == 128 || Cin == 256) && Cout % wr_bn(Cin) == 0 &&
         (long)B * Lout * Cin * 2 < 0x7fff0000L;
}
// M-tile groups of the WR grid (= BatchNorm partial rows): about one workgroup per CU in all
inline int wr_groups(long M, int Cout, int Cin) {
  const int NT = Cout / wr_bn(Cin);
  const long MT = (M + WR_BM - 1) / WR_BM;
  long gm = 256 / NT;
  if (gm < 1) gm = 1;
  return (int)(gm < MT ? gm : MT);
}

template <int BN, int NCH, int EPI>
int launch_fwd_wr_t(const FwdArgs& a, hipStream_t stream) {
  constexpr int NST = 3;
  constexpr int SMEM = WrCfg<BN, NCH>::smem(NST);
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_wr_kernel<BN, NCH, EPI, NST>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const long M = (long)a.B * a.Lout;
  const int MT = (int)((M + WR_BM - 1) / WR_BM), NT = a.Cout / BN;
  const int GM = wr_groups(M, a.Cout, a.Cin);
  hipLaunchKernelGGL((conv1d_nlc_fwd_wr_kernel<BN, NCH, EPI, NST>), dim3((unsigned)(GM * NT)), dim3(256), SMEM, stream,
                     a, MT, NT, GM);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int launch_fwd_wr(const FwdArgs& a, hipStream_t stream) {
  const bool b = a.stat_mode == 1;
  switch (a.Cin) {
    case 64: return b ? launch_fwd_wr_t<64, 1, 1>(a, stream) : launch_fwd_wr_t<64, 1, 0>(a, stream);
    case 128: return b ? launch_fwd_wr_t<128, 2, 1>(a, stream) : launch_fwd_wr_t<128, 2, 0>(a, stream);
    case 256: return b ? launch_fwd_wr_t<64, 4, 1>(a, stream) : launch_fwd_wr_t<64, 4, 0>(a, stream);
    default: return ecg::kBadArg;
  }
}

// ------------------------------------------------------------------------------ tap-shared weight gradient
// Stride-1, pad-1, 3-tap convs (Lin == Lout = L, every 3-tap conv of a ResNet stage except its first):
//   dw[co][k][ci] = sum_r dy[r][co] * x[r + k - 1][ci]   over rows r = (b, t), the shifted row inside sample b.
// One workgroup owns a 64 (co) x 64 (ci) x 3 (taps) block of dw and a range of 64-row chunks of r.  Per chunk it
// stages dy[r0, r0 + 64) and x[r0 - 1, r0 + 65) ONCE into LDS (LDS-DMA): the three taps read the x image at row
// offsets 0, 1, 2.  Against the one-tap kernel (a 128 x 128 tile of one tap per workgroup) that moves 17 KB instead
// of 32 KB per 0.8 M MACs ... per CU: 46 vs 32 MAC per staged byte, 3 x the MFMAs per barrier, and a 12 K-element
// output block instead of 16 K, so the split-K partial slabs (S x |dw|) shrink at equal workgroup counts.
// Sample boundaries: where t = 0 (tap 0) or t = L - 1 (tap 2) the shifted x row belongs to the neighbouring sample,
// so the dy operand of that tap is zeroed at those rows (a per-lane dword mask on the MFMA fragment).
// LDS images: [row][64] bf16 (128-B rows); 16-B chunk c of row j lives at chunk c ^ tsw(j), tsw(j) =
// 2 * (((j >> 1) & 1) | ((j >> 3) & 1) << 1): the 8 rows x 32 B one 32-lane ds_read_b64_tr_b16 group reads (rows
// {0..3, 8..11} + any shift) hit all 64 banks once.  The DMA writes lane-linear, so the XOR goes on the SOURCE chunk.
// Waves: wave w owns ci columns [16w, 16w + 16) for all 64 co and 3 taps (acc[4 co frags][3 taps]).
__device__ __forceinline__ int tsw(int j) { return 2 * (((j >> 1) & 1) | (((j >> 3) & 1) << 1)); }

constexpr int TSW_DY = 64 * 128;              // dy image bytes per stage
constexpr int TSW_STAGE = TSW_DY + 72 * 128;  // + x image rows r0-1 .. r0+70 (66 used)

template <int NST>
__global__ __launch_bounds__(256, 2) void conv1d_nlc_wgrad_ts_kernel(WgradArgs a, int TM, int TN, int splits) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): the DMA destinations are scalar
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tiles = TM * TN;
  const int split = wgid / tiles, tile = wgid % tiles;  // the tiles of one split (same rows) share an XCD
  const int co0 = (tile / TN) * 64, ci0 = (tile % TN) * 64;
  const int L = a.Lout;
  const int R = a.B * L;
  const int nchunks = (R + 63) / 64;
  const int ch0 = split * a.chunks_per_split;
  const int ch1 = min(nchunks, ch0 + a.chunks_per_split);
  f32x4 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (ch0 < ch1) {  // block-uniform
    const srd_t dyr = make_rsrc(a.dy, (long)R * a.Cout * 2);
    const srd_t xr = make_rsrc(a.x, (long)R * a.Cin * 2);
    const unsigned lds0 = lds_addr(smem);
    const int prow = lane >> 3;  // row inside an 8-row DMA piece
    // issue: dy pieces wv, wv + 4; x pieces wv, wv + 4, and x piece 8 split over the waves (16 lanes = 2 rows each)
    auto issue = [&](int ch, int st) {
      const unsigned dimg = lds0 + st * TSW_STAGE;
      const unsigned ximg = dimg + TSW_DY;
      const int r0 = ch * 64;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = wv + 4 * u, row = 8 * p + prow, r = r0 + row;
        const int src = (lane & 7) ^ tsw(row);
        dma16_at(dyr, r < R ? (unsigned)(((long)r * a.Cout + co0 + src * 8) * 2) : 0x7ffffff0u, dimg + p * 1024);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = wv + 4 * u, row = 8 * p + prow, r = r0 - 1 + row;
        const int src = (lane & 7) ^ tsw(row);
        dma16_at(xr, (r >= 0 && r < R) ? (unsigned)(((long)r * a.Cin + ci0 + src * 8) * 2) : 0x7ffffff0u,
              ximg + p * 1024);
      }
      {  // piece 8 (rows 64..71): lanes 16w .. 16w + 15 of wave w write rows 64 + 2w, 65 + 2w
        const int row = 64 + prow, r = r0 - 1 + row;
        const int src = (lane & 7) ^ tsw(row);
        if ((lane >> 4) == wv)
          dma16_at(xr, (r >= 0 && r < R) ? (unsigned)(((long)r * a.Cin + ci0 + src * 8) * 2) : 0x7ffffff0u,
                ximg + 8 * 1024);
      }
    };
    const int h = lane >> 4, q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
    auto tr_img = [&](const unsigned char* img, int row, int col) -> s16x4 {
      return tr16(reinterpret_cast<const __bf16*>(img + row * 128 + (((col >> 3) ^ tsw(row)) << 4) + ((col & 7) << 1)));
    };
    auto mma = [&](int st, int ch) {
      const unsigned char* dimg = smem + st * TSW_STAGE;
      const unsigned char* ximg = dimg + TSW_DY;
      const int r0 = ch * 64;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        typedef short s16x8v __attribute__((ext_vector_type(8)));
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const int rr = ks * 32 + 8 * h + q;
        // this lane's 8 reduction rows r0 + ks*32 + 8h + j: tap 0 drops t == 0, tap 2 drops t == L - 1 (L >= 8:
        // one wrap at most)
        const int rb = r0 + ks * 32 + 8 * h;
        const int tb = rb - fdiv(rb, a.lout) * L;
        u32x4 m0, m2;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          unsigned v0 = 0u, v2 = 0u;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            int t = tb + 2 * d + e;
            t -= t >= L ? L : 0;
            v0 |= (t != 0 ? 0xffffu : 0u) << (16 * e);
            v2 |= (t != L - 1 ? 0xffffu : 0u) << (16 * e);
          }
          m0[d] = v0;
          m2[d] = v2;
        }
        bf16x8 bx[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const s16x4 lo = tr_img(ximg, rr + k, 16 * wv + p4), hi = tr_img(ximg, rr + k + 4, 16 * wv + p4);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bx[k] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const s16x4 lo = tr_img(dimg, rr, 16 * i + p4), hi = tr_img(dimg, rr + 4, 16 * i + p4);
          s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const u32x4 ad = __builtin_bit_cast(u32x4, v);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ad), bx[1], acc[i][1], 0, 0, 0);
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ad & m0), bx[0], acc[i][0], 0,
                                                              0, 0);
          acc[i][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ad & m2), bx[2], acc[i][2], 0,
                                                              0, 0);
        }
      }
    };
    // NST-stage ring: chunks ch+1 .. ch+NST-2 stay in flight while chunk ch's MFMAs run.  Every wave issues exactly
    // 5 DMA instructions per chunk, so "chunk ch landed" = at most 5 x (younger chunks issued) outstanding; raw
    // s_barrier (a __syncthreads() would emit vmcnt(0) and drain the younger chunks: guide, "Pipelining across
    // barriers"); lgkmcnt(0) before it retires this wave's ds_reads of the buffer the next issue overwrites.
    const int n = ch1 - ch0;
#pragma unroll
    for (int i = 0; i < NST - 1; ++i)
      if (i < n) issue(ch0 + i, i);
    for (int i = 0; i < n; ++i) {
      const int ahead = min(NST - 2, n - 1 - i);  // younger chunks already issued
      if constexpr (NST >= 4) {
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if constexpr (NST == 3) {
        if (ahead >= 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (i + NST - 1 < n) issue(ch0 + i + NST - 1, (i + NST - 1) % NST);  // into the buffer mma(i - 1) read
      mma(i % NST, ch0 + i);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  }
  // partial[split][co][k * Cin + ci]: lane holds co = 16i + 4h + e, ci = 16 wv + (lane & 15) -> 64-B row segments
  const long N = 3L * a.Cin;
  float* out = a.part + (long)split * a.Cout * N + (long)co0 * N + ci0 + 16 * wv + (lane & 15);
  const int hq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(long)(16 * i + hq + e) * N + (long)k * a.Cin] = acc[i][k][e];
}

// The tap-shared kernel applies (stride 1, pad 1, 3 taps, same length, whole tensors addressable with 32-bit
// offsets) up to ECG_WGRAD_TS channels (read once; default 64: measured on MI355X, B=1024 ResNet1D-34 shapes,
// scripts/wgrad_micro.py, profiles/r3/wgrad_ts_ab.txt - 14.1 vs 21.6 us at 64 channels, where the one-tap path
// is the register-staged 64x64 kernel; slower than the one-tap 128x128 LDS-DMA kernel at 128-512 channels).
// 0 disables it.
inline bool wgrad_ts_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_WGRAD_TS");
    v = e ? atoi(e) : 64;
  }
  const long R = (long)B * Lout;
  return Cin <= v && Cout <= v && Kw == 3 && stride == 1 && pad == 1 && Lin == Lout && Lout >= 8 && Cin % 64 == 0 && Cout % 64 == 0 &&
         R * Cout * 2 < 0x7fff0000L && R * Cin * 2 < 0x7fff0000L;
}

// Workgroups the tap-shared launch aims for (ECG_WGRAD_TS_WGS, default 256: one per CU; the split-K partials are
// workgroups x 48 KB).
inline int wgrad_ts_target() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_WGRAD_TS_WGS");
    v = e ? atoi(e) : 256;
    if (v < 8) v = 8;
  }
  return v;
}

// ECG_WGRAD_TS_NST = LDS stages of the tap-shared loop (2..4, default 4: two chunks in flight); read once.
inline int wgrad_ts_nst() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_WGRAD_TS_NST");
    v = e ? atoi(e) : 4;
    if (v < 2 || v > 4) v = 4;
  }
  return v;
}

template <int NST>
int launch_wgrad_ts_n(const WgradArgs& a, int splits, hipStream_t stream) {
  constexpr int SMEM = NST * TSW_STAGE;
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_wgrad_ts_kernel<NST>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int TM = a.Cout / 64, TN = a.Cin / 64;
  hipLaunchKernelGGL(conv1d_nlc_wgrad_ts_kernel<NST>, dim3((unsigned)(TM * TN * splits)), dim3(256), SMEM, stream, a,
                     TM, TN, splits);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int launch_wgrad_ts(const WgradArgs& a, int splits, hipStream_t stream) {
  switch (wgrad_ts_nst()) {
    case 2: return launch_wgrad_ts_n<2>(a, splits, stream);
    case 3: return launch_wgrad_ts_n<3>(a, splits, stream);
    default: return launch_wgrad_ts_n<4>(a, splits, stream);
  }
}

template <int BM, int BN>
int launch_wgrad(const WgradArgs& a, int splits, hipStream_t stream) {
  constexpr int NWR = BM >= 256 ? 4 : 2;
  using Cfg = WgCfg<BM, BN, NWR>;
  static_assert(Cfg::SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_wgrad_kernel<BM, BN, NWR>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::SMEM));
    attr = true;
  }
  const int TM = a.Cout / BM, TN = a.Kw * a.Cin / BN;
  hipLaunchKernelGGL((conv1d_nlc_wgrad_kernel<BM, BN, NWR>), dim3((unsigned)(TM * TN * splits)), dim3(Cfg::NTHR),
                     Cfg::SMEM, stream, a, TM, TN, splits);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

// ECG_WGRAD_DMA=0 selects the register-staged weight-gradient loop (read once; default: LDS-DMA for 128x128).
inline bool wgrad_dma() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ECG_WGRAD_DMA");
    v = (e && atoi(e) == 0) ? 0 : 1;
  }
  return v == 1;
}

template <int BM, int BN>
int launch_wgrad_dma(const WgradArgs& a, int splits, hipStream_t stream) {
  constexpr int NWR = BM >= 256 ? 4 : 2;
  using Cfg = WgCfg<BM, BN, NWR>;
  constexpr int STAGES = 2 * 64 * (BM + BN) * 2;
  constexpr int SMEM = STAGES > Cfg::EP_BYTES ? STAGES : Cfg::EP_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_wgrad_dma_kernel<BM, BN, NWR>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int TM = a.Cout / BM, TN = a.Kw * a.Cin / BN;
  hipLaunchKernelGGL((conv1d_nlc_wgrad_dma_kernel<BM, BN, NWR>), dim3((unsigned)(TM * TN * splits)), dim3(Cfg::NTHR),
                     SMEM, stream, a, TM, TN, splits);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

// 256x256 weight-gradient tiles (opt-in, ECG_CONV_BIG >= 2, both channel counts multiples of 256): register-staged
// -6 %..+6 % against 128x128 (profiles/r1_resnet/cmb_p4_big*.log); with the LDS-DMA loop 1-14 % slower than the
// 128x128 DMA tiles (profiles/r1_resnet/wgrad_dma_256_*.log).
inline bool wgrad_big(int Cout, int Cin) { return conv_big() >= 2 && Cout % 256 == 0 && Cin % 256 == 0; }

}  // namespace

// y = conv(x) (+bias)(+ReLU); x [B][Lin][Cin] bf16, w [Cout][Kw][Cin] bf16, y [B][Lout][Cout] bf16.
// in_dil > 1 reads x as zero-inserted with that dilation (used for the data-gradient of strided convs).
// Extended form used by the ResNet step plan: ``stats`` receives [2][ceil(B*Lout/64)][Cout] BN partials;
// ``add`` (optionally masked by ``add_mask`` > 0) is added to the output before rounding.
// ``bnb`` (optional, stat_mode 1): {smask, sz, smean, srstd, szd, smean_d, srstd_d, mscale, mshift} of the
// BatchNorm whose backward statistics the data-grad epilogue produces ([2 or 3][M tiles][Cout] into ``stats``);
// mscale / mshift (both or neither) re-derive the ReLU mask from sz instead of reading smask.
// Register-staged launch for a forward conv with the A-operand BN+ReLU fold (fold_scale/shift): the tile family
// the picker gives a dilated input (no LDS-DMA, no 256-row tiles, no multi-tile workgroups).
namespace {
int launch_fwd_fold(const FwdArgs& a, hipStream_t stream) {
  int bm, bn;
  pick_fwd_tile((long)a.B * a.Lout, a.Cout, 2, &bm, &bn);
  const bool nb2 = conv_nbuf() == 2;
#define ECG_FOLD(BM_, BN_)                                                                                     \
  return a.stat_mode == 1 ? (nb2 ? launch_fwd_cfg<BM_, BN_, 1, 2>(a, stream) : launch_fwd_cfg<BM_, BN_, 1, 1>(a, stream)) \
                          : (nb2 ? launch_fwd_cfg<BM_, BN_, 0, 2>(a, stream) : launch_fwd_cfg<BM_, BN_, 0, 1>(a, stream))
  if (bm == 128 && bn == 128) ECG_FOLD(128, 128);
  if (bm == 128) ECG_FOLD(128, 64);
  ECG_FOLD(64, 64);
#undef ECG_FOLD
}
}  // namespace

ECG_API int ecg_conv1d_nlc_fwd_ex2(const void* x, const void* w, const float* bias, void* y, float* stats,
                                   const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                   int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                   const void* tail, const float* fold_scale, const float* fold_shift,
                                   hipStream_t stream);

ECG_API int ecg_conv1d_nlc_fwd_ex(const void* x, const void* w, const float* bias, void* y, float* stats,
                                  const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                  int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                  const void* tail, hipStream_t stream) {
  return ecg_conv1d_nlc_fwd_ex2(x, w, bias, y, stats, add, add_mask, B, Lin, Cin, Lout, Cout, Kw, stride, pad,
                                in_dil, relu, bnb, tail, nullptr, nullptr, stream);
}

// ecg_conv1d_nlc_fwd_ex plus the A-operand fold: with fold_scale / fold_shift (both or neither; in_dil == 1) the
// conv reads x = z and stages bf16(max(z * fold_scale[c] + fold_shift[c], 0)) - the BN_ACT output it replaces,
// bitwise - on the register-staged loop.  Its BatchNorm partial rows: ecg_conv1d_nlc_fwd_stat_tiles_fold.
ECG_API int ecg_conv1d_nlc_fwd_ex2(const void* x, const void* w, const float* bias, void* y, float* stats,
                                   const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                   int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                   const void* tail, const float* fold_scale, const float* fold_shift,
                                   hipStream_t stream) {
  if (!fold_scale != !fold_shift || (fold_scale && in_dil != 1)) return ecg::kBadArg;
  if (!x || !w || !y || B <= 0 || Lin <= 0 || Lout <= 0 || Kw <= 0 || stride <= 0 || in_dil <= 0 || pad < 0)
    return ecg::kBadArg;
  if (Cin % BK != 0 || Cout % 64 != 0 || (add_mask && !add)) return ecg::kBadArg;
  if (bnb && (!stats || !bnb[1] || !bnb[2] || !bnb[3] || (bnb[4] && (!bnb[5] || !bnb[6])) || (!bnb[7] != !bnb[8])))
    return ecg::kBadArg;
  if (tail && !stats) return ecg::kBadArg;
  FwdArgs a{static_cast<const __bf16*>(x), static_cast<const __bf16*>(w), bias, static_cast<__bf16*>(y), stats,
            static_cast<const __bf16*>(add), static_cast<const __bf16*>(add_mask),
            B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil, relu, bnb ? 1 : 0};
  if (bnb) {
    a.mscale = static_cast<const float*>(bnb[7]);
    a.mshift = static_cast<const float*>(bnb[8]);
    a.smask = static_cast<const __bf16*>(bnb[0]);
    a.sz = static_cast<const __bf16*>(bnb[1]);
    a.smean = static_cast<const float*>(bnb[2]);
    a.srstd = static_cast<const float*>(bnb[3]);
    a.szd = static_cast<const __bf16*>(bnb[4]);
    a.smean_d = static_cast<const float*>(bnb[5]);
    a.srstd_d = static_cast<const float*>(bnb[6]);
  }
  a.tail = static_cast<const ecg::BnTail*>(tail);
  a.ascale = fold_scale;
  a.ashift = fold_shift;
  if (fold_scale) return launch_fwd_fold(a, stream);
  if (wr_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return launch_fwd_wr(a, stream);
  int bm, bn;
  pick_fwd_tile((long)B * Lout, Cout, in_dil, &bm, &bn);
  if (bm == 256 && bn == 256) return launch_fwd<256, 256>(a, stream);
  if (bm == 256) return launch_fwd<256, 128>(a, stream);
  if (bm == 128 && bn == 128) return launch_fwd<128, 128>(a, stream);
  if (bm == 128) return launch_fwd<128, 64>(a, stream);
  return launch_fwd<64, 64>(a, stream);
}

// Select the forward tile family (see conv_big); returns the previous setting.
// Strided data-grads on the LDS-DMA loop (1) or the register-staged loop (0); returns the previous setting (tests).
ECG_API int ecg_conv1d_nlc_set_dma_dil(int on) {
  const int prev = conv_dma_dil() ? 1 : 0;
  g_conv_dma_dil = on ? 1 : 0;
  return prev;
}

ECG_API int ecg_conv1d_nlc_set_big(int big) {
  const int prev = conv_big();
  g_conv_big = big < 0 ? 0 : (big > 2 ? 2 : big);
  return prev;
}

// Select the multi-tile forward mode (see conv_mt); returns the previous setting.  Plans built before a change
// keep their BatchNorm partial-row counts: build them after setting the mode.
ECG_API int ecg_conv1d_nlc_set_mt(int mode) {
  const int prev = conv_mt();
  g_conv_mt = mode < 0 ? 0 : (mode > 2 ? 2 : mode);
  return prev;
}

// Number of M tiles (rows of the BN-statistics partials) the forward kernel uses for this shape.
ECG_API int ecg_conv1d_nlc_fwd_stat_tiles(long M, int Cout) {
  int bm, bn;
  pick_fwd_tile(M, Cout, 1, &bm, &bn);
  const int gm = fwd_mt_groups(M, Cout, 1, bm, bn);
  return gm > 0 ? gm : (int)((M + bm - 1) / bm);
}

// Partial rows of a forward with the A-operand fold (register-staged tiles, one per M tile).
ECG_API int ecg_conv1d_nlc_fwd_stat_tiles_fold(long M, int Cout) {
  int bm, bn;
  pick_fwd_tile(M, Cout, 2, &bm, &bn);
  return (int)((M + bm - 1) / bm);
}

// Rows of BatchNorm partials for the kernel that runs this exact conv (any stride / taps / dilation): the
// weight-resident kernel's M-tile groups where it applies, else the tile-family rows below.
ECG_API int ecg_conv1d_nlc_fwd_stat_tiles_ex(int B, int Lout, int Cout, int in_dil);
ECG_API int ecg_conv1d_nlc_fwd_stat_rows(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad,
                                         int in_dil) {
  if (wr_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return wr_groups((long)B * Lout, Cout, Cin);
  return ecg_conv1d_nlc_fwd_stat_tiles_ex(B, Lout, Cout, in_dil);
}

// Same for a call with batch B, output length Lout and input dilation in_dil (phase-decomposed data-grad).
ECG_API int ecg_conv1d_nlc_fwd_stat_tiles_ex(int B, int Lout, int Cout, int in_dil) {
  int bm, bn;
  pick_fwd_tile((long)B * Lout, Cout, in_dil, &bm, &bn);
  if (in_dil <= 1) return ecg_conv1d_nlc_fwd_stat_tiles((long)B * Lout, Cout);
  const int Lph = (Lout + in_dil - 1) / in_dil;
  return in_dil * (int)(((long)B * Lph + bm - 1) / bm);
}

ECG_API int ecg_conv1d_nlc_fwd(const void* x, const void* w, const float* bias, void* y, int B, int Lin, int Cin,
                               int Lout, int Cout, int Kw, int stride, int pad, int in_dil, int relu,
                               hipStream_t stream) {
  return ecg_conv1d_nlc_fwd_ex(x, w, bias, y, nullptr, nullptr, nullptr, B, Lin, Cin, Lout, Cout, Kw, stride, pad,
                               in_dil, relu, nullptr, nullptr, stream);
}

// Partial weight gradients: part[splits][Cout][Kw*Cin] fp32 (sum over dim 0 = dw in [Cout][Kw][Cin]).
// ``splits`` workgroup slices of the (b,t) reduction; returns kBadArg unless Cin, Cout % 64 == 0.
ECG_API int ecg_conv1d_nlc_wgrad(const void* dy, const void* x, float* part, int splits, int B, int Lin, int Cin,
                                 int Lout, int Cout, int Kw, int stride, int pad, hipStream_t stream) {
  if (!dy || !x || !part || splits <= 0 || B <= 0 || Kw <= 0 || stride <= 0 || pad < 0) return ecg::kBadArg;
  if (Cin % 64 != 0 || Cout % 64 != 0) return ecg::kBadArg;
  const long R = (long)B * Lout;
  const int nchunks = (int)((R + 63) / 64);
  const int cps = (nchunks + splits - 1) / splits;
  WgradArgs a{static_cast<const __bf16*>(dy), static_cast<const __bf16*>(x), part, B, Lin, Cin, Lout, Cout, Kw,
              stride, pad, cps, make_fastdiv(Lout)};
  if (wgrad_ts_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad)) return launch_wgrad_ts(a, splits, stream);
  const bool bm128 = Cout % 128 == 0, bn128 = Cin % 128 == 0;
  // LDS-DMA loops: 32-bit buffer offsets from the split's first row / sample
  const long rows = (long)cps * 64;
  const bool dma_ok = wgrad_dma() && rows * Cout * 2 < 0x7fff0000L &&
                      (rows / Lout + 2) * (long)Lin * Cin * 2 < 0x7fff0000L;
  if (wgrad_big(Cout, Cin)) return dma_ok ? launch_wgrad_dma<256, 256>(a, splits, stream)
                                          : launch_wgrad<256, 256>(a, splits, stream);
  if (bm128 && bn128 && dma_ok) return launch_wgrad_dma<128, 128>(a, splits, stream);
  if (bm128 && bn128) return launch_wgrad<128, 128>(a, splits, stream);
  if (bm128) return launch_wgrad<128, 64>(a, splits, stream);
  if (bn128) return launch_wgrad<64, 128>(a, splits, stream);
  return launch_wgrad<64, 64>(a, splits, stream);
}

// Workgroup tiles (C_out tiles x tap*C_in tiles) the weight-gradient kernel uses for this shape (split sizing).
ECG_API int ecg_conv1d_nlc_wgrad_tiles(int Cout, int Kw, int Cin) {
  const bool big = wgrad_big(Cout, Cin);
  const int bm = big ? 256 : (Cout % 128 == 0 ? 128 : 64), bn = big ? 256 : (Cin % 128 == 0 ? 128 : 64);
  return (Cout / bm) * (Kw * Cin / bn);
}

// Split count for the tap-shared weight-gradient kernel (64 x 64 x 3 output blocks, ~ECG_WGRAD_TS_WGS workgroups,
// >= 4 row chunks each), or 0 when this conv takes the one-tap kernels (the caller then sizes its own splits).
ECG_API int ecg_conv1d_nlc_wgrad_splits(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad) {
  if (!wgrad_ts_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad)) return 0;
  const long chunks = ((long)B * Lout + 63) / 64;
  const int tiles = (Cout / 64) * (Cin / 64);
  long s = (wgrad_ts_target() + tiles - 1) / tiles;
  s = s < chunks / 4 ? s : chunks / 4;
  return (int)(s < 1 ? 1 : (s > 1024 ? 1024 : s));
}

// Workgroups the weight-gradient launch should aim for (tiles x splits): ~4 resident per CU for the 4-wave
// tiles, ~2 rounds of one per CU for the 8-wave 256x256 tile.
ECG_API int ecg_conv1d_nlc_wgrad_target_wgs(int Cout, int Kw, int Cin) {
  (void)Kw;
  return wgrad_big(Cout, Cin) ? 512 : 1024;
}
