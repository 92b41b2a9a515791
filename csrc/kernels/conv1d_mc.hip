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
  const ecg::BnTail* tail;  // BatchNorm finalize fused into this launch's tail (bn_tail.h), or null
  // ReLU mask as bits (stat_mode 1, instead of smask): byte i of smask_bits holds (smask[8i + e] > 0) in bit e, one
  // byte per 8-channel vector - what the block-output BN_ACT pass writes beside its output (1/16 of the bytes)
  const uint8_t* smask_bits;
  // Input pre-activation (pa_scale != null; forward convs on the tap-shared kernels only): the GEMM operand is
  // bf16(relu(fmaf(x, pa_scale, pa_shift))) per input channel - the BatchNorm + ReLU of the conv that produced x,
  // bitwise the BN_ACT pass - applied to the staged A' image; nt == 0 workgroups store the activated rows of their
  // tile to pa_out (the weight gradient's operand).
  const float* pa_scale;
  const float* pa_shift;
  __bf16* pa_out;
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
  // ph < 0: the strided tap data-grad's layout - wave row wr holds phase wr >> 1, rows (wr & 1) * WM of the phase
  const int wph = ph < 0 ? wr >> 1 : ph, wrow = ph < 0 ? (wr & 1) * WM : wr * WM;
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
      const int m = m0 + wrow + r;
      const int bb = m / Lrow, tt = m - bb * Lrow;
      const int uu = P > 1 ? tt * P + wph : tt;
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
        } else if (bwd && a.smask_bits != nullptr) {
          const unsigned mb = a.smask_bits[o >> 3];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (mb >> e) & 1u ? v[e] : 0.f;
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
  const int wph = ph < 0 ? wr >> 1 : ph, wrow = ph < 0 ? (wr & 1) * WM : wr * WM;  // (ph < 0: see the rowwise form)
  constexpr int EP_LD = Cfg::EP_LD, HR = WM / 2;
  float* ep = reinterpret_cast<float*>(smem) + wv * HR * EP_LD;
  constexpr int CG = WN / 8, RSTEP = 64 / CG, ITEMS = HR / RSTEP;
  const int cg = lane % CG, rs = lane / CG;
  const int n = EpiLane<BN, NWR>::n(n0);
  constexpr bool bwd = EPI == 1;  // compile-time: the forward epilogue carries none of the backward code
  const bool ds = bwd && a.szd != nullptr;
  const bool mk_bits = bwd && a.mscale == nullptr && a.smask_bits != nullptr;
  const bool mk_smask = bwd && a.mscale == nullptr && !mk_bits && a.smask != nullptr;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // The half's global operands (z, z_d, residual gradient and its mask) for all ITEMS rows are issued before the
    // accumulators are staged, so the half costs ONE load round trip instead of one per row pair.  Rows outside
    // the output read offset 0 (valid memory, value unused).
    long po[ITEMS];
    bool pv[ITEMS];
    bf16x8 pz[ITEMS], pzd[ITEMS], pad[ITEMS], pmk[ITEMS];
    unsigned pmb[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
      const int r = h * HR + rs + it * RSTEP;
      const int m = m0 + wrow + r;
      const int bb = m / Lrow, tt = m - bb * Lrow;
      const int uu = P > 1 ? tt * P + wph : tt;
      pv[it] = m < M && uu < a.Lout;
      po[it] = pv[it] ? ((long)bb * a.Lout + uu) * a.Cout + n : 0;
      if constexpr (bwd) pz[it] = *reinterpret_cast<const bf16x8*>(a.sz + po[it]);
      if (ds) pzd[it] = *reinterpret_cast<const bf16x8*>(a.szd + po[it]);
      if (a.add) pad[it] = *reinterpret_cast<const bf16x8*>(a.add + po[it]);
      if (a.add && a.add_mask) pmk[it] = *reinterpret_cast<const bf16x8*>(a.add_mask + po[it]);
      else if (mk_smask) pmk[it] = *reinterpret_cast<const bf16x8*>(a.smask + po[it]);
      if (mk_bits) pmb[it] = a.smask_bits[po[it] >> 3];
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
        } else if (mk_bits) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (pmb[it] >> e) & 1u ? v[e] : 0.f;
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

// Register-staged forward / data-grad, the fallback of the LDS-DMA loops (operands beyond 32-bit buffer offsets):
// one LDS buffer, two barriers per K tile, three workgroups per CU; tile t+1's global loads are in flight during
// tile t's MFMAs.
template <int BM, int BN, int EPI>
__global__ __launch_bounds__(THREADS, 3) void conv1d_nlc_fwd_kernel(FwdArgs a, int MT, int NT) {
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
  auto ld_set = [&](uint4* ra, uint4* rb, int t) {
    const int tc = t < nk ? t : nk - 1;
    const int k = k0 + (tc / CB) * P, c0 = (tc % CB) * BK;
    const int kk = k * a.Cin + c0;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int u = apos[i] + k;
      bool ok = u >= 0 && u < Lext;
      if (a.in_dil > 1) {
        ok = ok && (u % a.in_dil == 0);
        u /= a.in_dil;
      }
      ra[i] = ok ? *reinterpret_cast<const uint4*>(a.x + abase[i] + (long)u * a.Cin + c0) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rb[i] = *reinterpret_cast<const uint4*>(wb + (long)i * (THREADS / 8) * (a.Kw * a.Cin) + kk);
  };
  auto st_set = [&](__bf16* base, const uint4* ra, const uint4* rb) {
#pragma unroll
    for (int i = 0; i < NA; ++i) store_one(base, tid + i * THREADS, ra[i]);
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
  if (nk > 0) {  // block-uniform (a phase without taps leaves acc = 0)
    ld_set(ra0, rb0, 0);
    st_set(lds, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      ld_set(ra0, rb0, kt + 1);
      mma(lds);
      __syncthreads();  // every wave is done reading the buffer
      st_set(lds, ra0, rb0);
      __syncthreads();
    }
  }
  fwd_epilogue<BM, BN, EPI, 2, false>(a, acc, smem, m0, n0, mt, MT, Lrow, M, P, ph);  // row-wise form: 168 VGPRs
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
// one 16-B piece per lane into LDS at (wave-uniform) lds + 16 * lane; s_nop covers the M0 -> LDS-DMA hazard.
// M0 is compiler-reserved and assumed unchanged across an asm statement, so the statement restores it (a "m0"
// clobber is not honoured: MI355X guide §5.7) - any compiler use of M0 around these loops stays correct.
__device__ __forceinline__ void dma16_at(srd_t r, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
__device__ __forceinline__ void dma16(srd_t r, unsigned voff, unsigned char* lds_piece) {
  dma16_at(r, voff, lds_addr(lds_piece));
}
// 16-byte vector store through a buffer resource (out-of-range offsets are dropped by the range check), from asm so
// that it is always issued - one vmcnt entry per call, which the counted waits of the tap loop rely on.  The s_nop
// is the wait state a VALU write of the store's data VGPRs needs after a >8-byte buffer store (hipcc does not pad
// hazards of an asm statement, MI355X guide §5.7).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_at(srd_t r, unsigned voff, u32x4 v) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen\n\ts_nop 0" ::"v"(v), "v"(voff), "s"(r) : "memory");
}

// NWR = waves along M: 2 -> 4 waves (2x2), 4 -> 8 waves (4x2, 2 per SIMD at one workgroup per CU).  256-row
// tiles need one workgroup per CU (2 x 64 KB of stages at 256x256).  Two LDS stages: one K step in flight while the
// MFMAs run (three stages measured slower or neutral for every tile: profiles/r2/resnet_conv_ab.txt,
// profiles/r3/resnet_tile256_wgrad_ab.txt).
template <int BM, int BN, int EPI, int NWR>
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

// ------------------------------------------------------------------ tap-shared 256-row forward / data-grad
// Stride-1, pad-1, 3-tap convs over whole samples (Lin == Lout = L: every conv of a ResNet stage but its strided
// first one, forward AND data-grad).  The three taps of one 64-channel chunk read the SAME activation rows shifted
// by one: output row m, tap k reads input row m + k - 1 of its sample.  So per chunk the workgroup stages the
// activation rows [m0 - 1, m0 + 263) ONCE (the "A' image") and each tap's MFMAs read it at row offset k, while the
// weight tile of each (chunk, tap) step streams through a ring of its own.  Against the one-tap kernels (a 128 x 128
// tile restaging 16 KB of activations per tap) a 256 x BN tile moves 11 KB of activations + BN*128 B of weights per
// 64-deep step: 27 KB per 256x128x64 MACs instead of 64 KB for two 128x128 workgroups - and the one-tap loop is
// bound by its staged bytes (a CU keeps ~64 KB in flight against a ~1 us L2 round trip at B=1024: the isolated
// layer-4 forward ran at 690 TF/s at B=1024 vs 1000 TF/s with 256x256 tiles at B=4096, scripts/r4_conv_probe.py).
// Rows that cross a sample boundary are masked per lane: tap 0 at t == 0 and tap 2 at t == L-1 read a row of the
// neighbouring sample, so those A fragments are zeroed (zero padding).
// Layout: 8 waves as 4 (M) x 2 (N), each 64 x BN/2 (one workgroup per CU, two waves per SIMD).  LDS: two A' slots
// [264 rows][128 B] (16-B chunk cc of row r at cc ^ (r & 7): conflict-free ds_read_b128 at any row offset) and three
// weight slots [BN rows][128 B]; step s = 3c + k uses weight slot k, A' slot c & 1.  LDS-DMA from inline asm,
// counted vmcnt waits, raw s_barrier (a __syncthreads() would drain the DMA kept in flight).
constexpr int TAP_BM = 256;
constexpr int TAP_AROWS = TAP_BM + 8;       // image rows m0-1 .. m0+262 (258 used); 33 DMA pieces of 8 rows
constexpr int TAP_ASLOT = TAP_AROWS * 128;  // 33,792 B
constexpr int TAP_NA = 5;                   // DMA instructions per wave per A' image (4 full pieces + 1 row)

// Input pre-activation (FwdArgs::pa_*): each wave transforms its OWN DMA pieces of A'(c) in place right after the
// counted wait that makes them visible and before the step's barrier - the DMA writes lane-linear, so a lane's piece
// sits at a fixed LDS offset and always holds the same 8 channels of the chunk (source chunk (lane & 7) ^ (row & 7)
// with row & 7 == (lane >> 3) & 7).  Image rows outside the tensor stay zero (the conv's padding); nt == 0
// workgroups store their tile's rows (1 .. 256 of the image) for the weight gradient.  Per-channel scale / shift
// in an LDS table [2][Cin].
constexpr int PA_MAXC = 512;

template <int BN, bool PA = false>
struct TapCfg {
  static constexpr int BSLOT = BN * 128;
  static constexpr int BP = BN / 64;  // weight pieces per wave per step (8 waves x 8 rows)
  static constexpr int TOFF = 2 * TAP_ASLOT + 3 * BSLOT;  // pre-activation table (PA)
  static constexpr int STAGES = TOFF + (PA ? 2 * PA_MAXC * 4 : 0);
  static constexpr int SMEM = STAGES > FwdCfg<TAP_BM, BN, 4>::EP_BYTES ? STAGES : FwdCfg<TAP_BM, BN, 4>::EP_BYTES;
};

template <int BN, int EPI, bool PA>
// (launch bounds: one workgroup per CU is all the ~115 KB of LDS allows; 103-228 VGPRs per variant (two waves per
// SIMD allow 256), no scratch)
__global__ __launch_bounds__(512, 1) void conv1d_nlc_fwd_tap_kernel(FwdArgs a, int MT, int NT) {
  constexpr int BM = TAP_BM, NWR = 4, NW = 8;
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN;
  using TC = TapCfg<BN, PA>;
  constexpr int BP = TC::BP, BSLOT = TC::BSLOT;
  constexpr int ST = PA ? TAP_NA : 0;  // pre-activation stores per wave per chunk (issued at k = 0)
  static_assert(WM == 64 && FM == 4, "64-row wave tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int mt = wgid / NT, nt = wgid % NT;  // the NT column blocks of one M tile share an XCD (same A rows)
  const int m0 = mt * BM, n0 = nt * BN;
  const int L = a.Lout, M = a.B * L, Cin = a.Cin, CB = Cin / 64, K3 = 3 * Cin;
  const srd_t xr = make_rsrc(a.x, (long)M * Cin * 2);
  const srd_t wrs = make_rsrc(a.w, (long)a.Cout * K3 * 2);
  const unsigned lds0 = lds_addr(smem);
  const unsigned ldsA = lds0, ldsB = lds0 + 2 * TAP_ASLOT;
  // A' DMA: pieces p = wv + 8i (i < 4) cover image rows 8p .. 8p+7 (lane -> row 8p + lane/8, LDS chunk lane%8);
  // piece 32 (rows 256..263) is issued by every wave with lanes 8wv .. 8wv+7 only (row 256 + wv).
  unsigned aoff[TAP_NA];
#pragma unroll
  for (int i = 0; i < TAP_NA; ++i) {
    const int row = i < 4 ? 8 * (wv + NW * i) + (lane >> 3) : 256 + (lane >> 3);
    const int g = m0 - 1 + row;
    const int src = (lane & 7) ^ (row & 7);
    aoff[i] = (g >= 0 && g < M) ? (unsigned)(g * Cin * 2 + src * 16) : 0x7ffffff0u;
  }
  unsigned boff[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int n = 8 * (wv + NW * i) + (lane >> 3);
    boff[i] = (unsigned)((n0 + n) * K3 * 2 + (((lane & 7) ^ (n & 7)) * 16));
  }
  auto issue_a = [&](int c, int slot) {
    const unsigned base = ldsA + slot * TAP_ASLOT;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16_at(xr, aoff[i] + c * 128, base + (wv + NW * i) * 1024);
    if ((lane >> 3) == wv) dma16_at(xr, aoff[4] + c * 128, base + 32 * 1024);
  };
  auto issue_b = [&](int c, int k, int slot) {
    const unsigned base = ldsB + slot * BSLOT;
#pragma unroll
    for (int i = 0; i < BP; ++i) dma16_at(wrs, boff[i] + (k * Cin + c * 64) * 2, base + (wv + NW * i) * 1024);
  };
  // pre-activation: per-piece row validity, store offsets (image rows 1..256 = the tile's own rows, nt == 0 only;
  // the rest land out of range and are dropped) and the [2][Cin] scale / shift table
  srd_t pr{};
  unsigned soff[TAP_NA];
  unsigned pvalid = 0u;
  if constexpr (PA) {
    pr = make_rsrc(a.pa_out, a.pa_out ? (long)M * Cin * 2 : 0L);
#pragma unroll
    for (int i = 0; i < TAP_NA; ++i) {
      const int row = i < 4 ? 8 * (wv + NW * i) + (lane >> 3) : 256 + (lane >> 3);
      const int g = m0 - 1 + row;
      const bool in = g >= 0 && g < M && (i < 4 || (lane >> 3) == wv);
      pvalid |= (in ? 1u : 0u) << i;
      soff[i] = (in && nt == 0 && row >= 1 && row <= 256 && a.pa_out) ? aoff[i] : 0x7ffffff0u;
    }
    float* tab = reinterpret_cast<float*>(smem + TC::TOFF);
    for (int ch = tid; ch < Cin; ch += 512) {
      tab[ch] = a.pa_scale[ch];
      tab[Cin + ch] = a.pa_shift[ch];
    }
    __syncthreads();  // (no DMA in flight yet)
  }
  // the wave's own pieces of A'(c) (LDS slot) -> relu(x * scale + shift), stored to pa_out (ST stores, always issued)
  auto pre_act = [&](int c, int slot) {
    const float* tab = reinterpret_cast<const float*>(smem + TC::TOFF);
    const int ch = c * 64 + 8 * ((lane & 7) ^ ((lane >> 3) & 7));
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = tab[ch + e];
      sh[e] = tab[Cin + ch + e];
    }
#pragma unroll
    for (int i = 0; i < TAP_NA; ++i) {
      unsigned char* xp = smem + slot * TAP_ASLOT + (i < 4 ? wv + NW * i : 32) * 1024 + lane * 16;
      const u32x4 xv = *reinterpret_cast<const u32x4*>(xp);
      const bf16x8 x = __builtin_bit_cast(bf16x8, xv);
      bf16x8 y;
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = (__bf16)fmaxf(fmaf((float)x[e], sc[e], sh[e]), 0.f);
      const u32x4 v = ((pvalid >> i) & 1u) ? __builtin_bit_cast(u32x4, y) : xv;
      if (i < 4 || (lane >> 3) == wv) *reinterpret_cast<u32x4*>(xp) = v;  // (piece 32: 8 lanes of each wave)
      st16_at(pr, soff[i] + c * 128, v);
    }
  };
  // this lane's fragment rows: i_f = wr*64 + 16f + (lane & 15); tap 0 is invalid at t == 0, tap 2 at t == L-1
  unsigned ok0 = 0u, ok2 = 0u;
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int m = m0 + wr * WM + 16 * f + (lane & 15);
    const int t = m - (m / L) * L;
    ok0 |= (t != 0 ? 1u : 0u) << f;
    ok2 |= (t != L - 1 ? 1u : 0u) << f;
  }
  // read addresses (bytes from the slot base): row r chunk cc at r*128 + ((cc ^ (r & 7)) << 4).  A rows i_f + k have
  // r & 7 == (lane + k) & 7; B rows n = wc*WN + 16j + (lane & 15) have n & 7 == lane & 7.
  const int arow = (wr * WM + (lane & 15)) * 128, brow = (wc * WN + (lane & 15)) * 128;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = 3 * CB;
  issue_a(0, 0);
  issue_b(0, 0, 0);
  issue_b(0, 1, 1);
  for (int c = 0; c < CB; ++c) {
    const bool more = c + 1 < CB;  // block-uniform
    const unsigned char* As = smem + (c & 1) * TAP_ASLOT;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int s = 3 * c + k;
      // wait for weight step s (and, at k == 0, A'(c), issued before it): the younger vector-memory operations of
      // this wave are counted - per chunk, in issue order: [ST pre-activation stores] B(3c+2) A'(c+1) at k = 0,
      // B(3c+3) at k = 1, B(3c+4) at k = 2
      if (k == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP) : "memory");
        if constexpr (PA) pre_act(c, c & 1);
      } else if (k == 1) {
        if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST + BP + TAP_NA) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST + BP) : "memory");
      } else {
        if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP + TAP_NA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of step s-1 retired (WAR)
      __builtin_amdgcn_s_barrier();
      if (s + 2 < nk) issue_b((s + 2) / 3, (k + 2) % 3, (k + 2) % 3);  // into the slot step s-1 read
      if (k == 0 && more) issue_a(c + 1, (c + 1) & 1);                  // into the slot chunk c-1 read
      const unsigned char* Bs = smem + 2 * TAP_ASLOT + k * BSLOT;
      const unsigned okm = k == 0 ? ok0 : ok2;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cc = 4 * ks + (lane >> 4);
        const int asw = (cc ^ ((lane + k) & 7)) << 4, bsw = (cc ^ (lane & 7)) << 4;
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          af[f] = *reinterpret_cast<const bf16x8*>(As + arow + (16 * f + k) * 128 + asw);
          if (k != 1 && !((okm >> f) & 1u)) af[f] = bf16x8{};
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + brow + 16 * j * 128 + bsw);
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], bfr[j], acc[f][j], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the stage buffers
  EpiConst k;
  k.load<EPI == 1>(a, EpiLane<BN, NWR>::n(n0));
  fwd_epi_tile<BM, BN, EPI, NWR, EPI == 1>(a, acc, smem, k, m0, n0, L, M, 1, 0);
  if (a.stats) fwd_epi_stats<BM, BN, EPI, NWR>(a, smem, k, n0, mt, MT);  // block-uniform
  if (a.tail && a.stats)
    ecg::bn_tail<Cfg::NTHR>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, MT, a.Cout, mt, n0, BN, smem);
}

// ------------------------------------------------------------------ tap-shared strided data-grad
// The data-grad of a stride-2, pad-1, 3-tap conv (the first conv of a ResNet stage): dx[u] = sum_k W'[k] dz_dil[u + k
// - 1] over the zero-inserted dz.  Output u = 2i + ph: phase 0 takes tap 1 at dz row i, phase 1 takes tap 0 at row i
// and tap 2 at row i + 1 (inside the sample).  So both phases of the output rows 2i, 2i+1 for i in a 128-row range
// read the SAME dz rows [i0, i0 + 129): the workgroup stages that A' image once per 64-channel chunk and its three
// taps read it at row offsets 0 / 0 / 1 - the tap-shared kernel's structure, at half its MACs per tile (the
// phase-decomposed one-tap kernel restages the rows for every tap and phase).  256 output rows per tile (128 i-rows
// x 2 phases), 8 waves as 4 x 2: wave row wr computes phase wr >> 1, i-rows (wr & 1) * 64 .. + 64, so phase-0 waves
// run the MFMAs of tap 1 and phase-1 waves those of taps 0 and 2 (wave-uniform).  The epilogue maps the rows back
// to u = 2i + ph (fwd_epi_tile with ph < 0).  LDS: two A' slots [136 rows][128 B], three weight slots [BN][128 B].
constexpr int S2_IR = 128;                 // i-rows per tile
constexpr int S2_AROWS = S2_IR + 8;        // image rows i0 .. i0 + 135 (129 used): 17 DMA pieces of 8 rows
constexpr int S2_ASLOT = S2_AROWS * 128;   // 17,408 B
constexpr int S2_NA = 3;                   // DMA instructions per wave per A' image (2 full pieces + 1 row)

template <int BN>
struct TapS2Cfg {
  static constexpr int BSLOT = BN * 128;
  static constexpr int BP = BN / 64;
  static constexpr int STAGES = 2 * S2_ASLOT + 3 * BSLOT;
  static constexpr int SMEM = STAGES > FwdCfg<TAP_BM, BN, 4>::EP_BYTES ? STAGES : FwdCfg<TAP_BM, BN, 4>::EP_BYTES;
};

template <int BN, int EPI>
__global__ __launch_bounds__(512, 1) void conv1d_nlc_dgrad_s2_tap_kernel(FwdArgs a, int MT, int NT) {
  constexpr int NWR = 4, NW = 8;
  using Cfg = FwdCfg<TAP_BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN;
  constexpr int BP = TapS2Cfg<BN>::BP, BSLOT = TapS2Cfg<BN>::BSLOT;
  static_assert(WM == 64 && FM == 4, "64-row wave tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wv >> 1, wc = wv & 1, ph = wr >> 1, irow0 = (wr & 1) * WM;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int mt = wgid / NT, nt = wgid % NT;
  const int Lz = a.Lin, Mi = a.B * Lz;  // dz rows per sample / in total (the i-rows)
  const int i0 = mt * S2_IR, n0 = nt * BN;
  const int Cin = a.Cin, CB = Cin / 64, K3 = 3 * Cin;
  const srd_t xr = make_rsrc(a.x, (long)Mi * Cin * 2);
  const srd_t wrs = make_rsrc(a.w, (long)a.Cout * K3 * 2);
  const unsigned lds0 = lds_addr(smem);
  const unsigned ldsA = lds0, ldsB = lds0 + 2 * S2_ASLOT;
  // A' DMA: pieces p = wv + 8i (i < 2) cover image rows 8p .. 8p+7; piece 16 (rows 128..135) by every wave with lanes
  // 8wv .. 8wv+7 only (row 128 + wv).  Image row r <-> dz row i0 + r; rows past the tensor land as zeros.
  unsigned aoff[S2_NA];
#pragma unroll
  for (int i = 0; i < S2_NA; ++i) {
    const int row = i < 2 ? 8 * (wv + NW * i) + (lane >> 3) : S2_IR + (lane >> 3);
    const int g = i0 + row;
    const int src = (lane & 7) ^ (row & 7);
    aoff[i] = g < Mi ? (unsigned)(g * Cin * 2 + src * 16) : 0x7ffffff0u;
  }
  unsigned boff[BP];
#pragma unroll
  for (int i = 0; i < BP; ++i) {
    const int n = 8 * (wv + NW * i) + (lane >> 3);
    boff[i] = (unsigned)((n0 + n) * K3 * 2 + (((lane & 7) ^ (n & 7)) * 16));
  }
  auto issue_a = [&](int c, int slot) {
    const unsigned base = ldsA + slot * S2_ASLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16_at(xr, aoff[i] + c * 128, base + (wv + NW * i) * 1024);
    if ((lane >> 3) == wv) dma16_at(xr, aoff[2] + c * 128, base + 16 * 1024);
  };
  auto issue_b = [&](int c, int k, int slot) {
    const unsigned base = ldsB + slot * BSLOT;
#pragma unroll
    for (int i = 0; i < BP; ++i) dma16_at(wrs, boff[i] + (k * Cin + c * 64) * 2, base + (wv + NW * i) * 1024);
  };
  // phase 1, tap 2 reads dz row i + 1: invalid at the sample's last row
  unsigned ok2 = 0u;
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int m = i0 + irow0 + 16 * f + (lane & 15);
    const int t = m - (m / Lz) * Lz;
    ok2 |= (t != Lz - 1 ? 1u : 0u) << f;
  }
  const int arow = (irow0 + (lane & 15)) * 128, brow = (wc * WN + (lane & 15)) * 128;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = 3 * CB;
  issue_a(0, 0);
  issue_b(0, 0, 0);
  issue_b(0, 1, 1);
  for (int c = 0; c < CB; ++c) {
    const bool more = c + 1 < CB;  // block-uniform
    const unsigned char* As = smem + (c & 1) * S2_ASLOT;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int s = 3 * c + k;
      // the tap-shared kernel's counted waits (S2_NA A' instructions per chunk)
      if (k == 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP) : "memory");
      } else if (k == 1) {
        if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP + S2_NA) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP) : "memory");
      } else {
        if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(BP + S2_NA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (s + 2 < nk) issue_b((s + 2) / 3, (k + 2) % 3, (k + 2) % 3);
      if (k == 0 && more) issue_a(c + 1, (c + 1) & 1);
      if ((ph == 0) != (k == 1)) continue;  // wave-uniform: phase 0 takes tap 1, phase 1 taps 0 and 2
      const int off = k == 2 ? 1 : 0;
      const unsigned char* Bs = smem + 2 * S2_ASLOT + k * BSLOT;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cc = 4 * ks + (lane >> 4);
        const int asw = (cc ^ ((lane + off) & 7)) << 4, bsw = (cc ^ (lane & 7)) << 4;
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          af[f] = *reinterpret_cast<const bf16x8*>(As + arow + (16 * f + off) * 128 + asw);
          if (k == 2 && !((ok2 >> f) & 1u)) af[f] = bf16x8{};
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + brow + 16 * j * 128 + bsw);
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], bfr[j], acc[f][j], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the stage buffers
  EpiConst kc;
  kc.load<EPI == 1>(a, EpiLane<BN, NWR>::n(n0));
  fwd_epi_tile<TAP_BM, BN, EPI, NWR, EPI == 1>(a, acc, smem, kc, i0, n0, Lz, Mi, 2, -1);
  if (a.stats) fwd_epi_stats<TAP_BM, BN, EPI, NWR>(a, smem, kc, n0, mt, MT);  // block-uniform
  if (a.tail && a.stats)
    ecg::bn_tail<Cfg::NTHR>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, MT, a.Cout, mt, n0, BN, smem);
}

// ------------------------------------------------------------------ persistent tap-shared 64-channel kernel
// The 64-channel stage (C_in = C_out = 64, stride 1, pad 1, 3 taps: every conv of ResNet layer1, forward AND
// data-grad) is a thin GEMM - N = 64, K = 192 - over M = B*L = 128,000 rows at B=1024: 3.1 GFLOP against 33 MB of
// activations in and out, so it is bound by moving rows, not by the MFMA.  The one-tap multi-tile kernel re-stages
// the activation rows once per tap and the 64x64 weight tile every K step; here each workgroup
//   * keeps the whole 3 x 64 x 64 weight image resident in LDS for the launch (DMA'd once),
//   * walks M tiles gm, gm + GM, ... (persistent grid, two workgroups per CU), staging each tile's activation rows
//     ONCE as a 136-row A' image (rows m0-1 .. m0+128, read by the three taps at row offsets 0/1/2, as the
//     256-row tap-shared kernel does) in a two-slot ring: tile j+1's image lands while tile j's MFMAs and
//     epilogue run,
//   * stores each tile through its own LDS staging region (fwd_epi_tile_rowwise: bias / residual / masks / ReLU /
//     BatchNorm partials, the same epilogue as every other kernel here) and accumulates the BatchNorm partials of
//     all its tiles into ONE partial row (row gm of GM), finalized by the fused tail.
// 4 waves as 2 (M) x 2 (N), wave tile 64 x 32.  LDS: weights 24 KB | A' slots 2 x 17 KB | epilogue 19.5 KB = 77.5 KB.
constexpr int T64_BM = 128;
constexpr int T64_AROWS = 136;                 // 17 DMA pieces of 8 rows (130 used)
constexpr int T64_ASLOT = T64_AROWS * 128;     // 17,408 B
constexpr int T64_WBYTES = 3 * 64 * 128;       // 24,576 B
using T64Cfg = FwdCfg<T64_BM, 64, 2>;
constexpr int T64_SMEM = T64_WBYTES + 2 * T64_ASLOT + T64Cfg::EP_BYTES;
static_assert(2 * T64_SMEM <= 160 * 1024, "two workgroups per CU");

template <int EPI, bool PA = false>
__global__ __launch_bounds__(256, 2) void conv1d_nlc_tap64_kernel(FwdArgs a, int MT, int GM) {
  constexpr int BM = T64_BM, BN = 64, NWR = 2, NW = 4;
  constexpr int WM = T64Cfg::WM, WN = T64Cfg::WN, FM = T64Cfg::FM, FN = T64Cfg::FN;
  static_assert(WM == 64 && WN == 32 && FM == 4 && FN == 2, "64 x 32 wave tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* const Ws = smem;
  unsigned char* const As = smem + T64_WBYTES;
  unsigned char* const eps = As + 2 * T64_ASLOT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wv >> 1, wc = wv & 1;
  const int gm = blockIdx.x;
  const int L = a.Lout, M = a.B * L;
  const int ntiles = gm < MT ? (MT - gm + GM - 1) / GM : 0;
  const srd_t xr = make_rsrc(a.x, (long)M * 64 * 2);
  const srd_t wrs = make_rsrc(a.w, 64L * 192 * 2);
  const unsigned ldsW = lds_addr(Ws), ldsA = lds_addr(As);
  // weight image [tap k][row n][64 ch], 16-B chunk cc of row n at cc ^ (n & 7): 24 pieces (k, 8-row block), 6 per
  // wave; the XOR goes on the SOURCE chunk (the DMA writes lane-linear)
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int p = wv + NW * i, k = p >> 3, n = 8 * (p & 7) + (lane >> 3);
    dma16_at(wrs, (unsigned)(n * 384 + k * 128 + (((lane & 7) ^ (n & 7)) << 4)), ldsW + p * 1024);
  }
  // A' image of the tile at m0: image row r <-> global row m0 - 1 + r; pieces p = wv + 4i (i < 4) and, by every
  // wave with lanes 8wv .. 8wv+7 only, row 128 + wv (rows 128..131: 128 and 129 are used)
  auto issue_a = [&](int m0, int slot) {
    const unsigned base = ldsA + slot * T64_ASLOT;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int row = i < 4 ? 8 * (wv + NW * i) + (lane >> 3) : 128 + (lane >> 3);
      const int g = m0 - 1 + row;
      const unsigned off = (g >= 0 && g < M) ? (unsigned)(g * 128 + ((((lane & 7) ^ (row & 7))) << 4)) : 0x7ffffff0u;
      if (i < 4)
        dma16_at(xr, off, base + (wv + NW * i) * 1024);
      else if ((lane >> 3) == wv)
        dma16_at(xr, off, base + 16 * 1024);
    }
  };
  EpiConst k;
  k.load<EPI == 1>(a, EpiLane<BN, NWR>::n(0));
  const int arow = (wr * WM + (lane & 15)) * 128, brow = (wc * WN + (lane & 15)) * 128;
  // input pre-activation (FwdArgs::pa_*): a lane's DMA pieces always hold the same 8 channels (the single 64-channel
  // chunk, source chunk (lane & 7) ^ (row & 7) with row & 7 == (lane >> 3) & 7): their scale / shift in registers
  float psc[8], psh[8];
  if constexpr (PA) {
    const int ch = 8 * ((lane & 7) ^ ((lane >> 3) & 7));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      psc[e] = a.pa_scale[ch + e];
      psh[e] = a.pa_shift[ch + e];
    }
  }
  if (ntiles > 0) issue_a(gm * BM, 0);
  for (int j = 0; j < ntiles; ++j) {  // block-uniform
    const int m0 = (gm + j * GM) * BM;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of A'(j) (and, at j = 0, W) landed
    if constexpr (PA) {  // this wave's own pieces -> relu(x * scale + shift); image rows 1..128 (the tile) stored
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int row = i < 4 ? 8 * (wv + NW * i) + (lane >> 3) : 128 + (lane >> 3);
        const int g = m0 - 1 + row;
        if ((i < 4 || (lane >> 3) == wv) && g >= 0 && g < M) {
          bf16x8* xp = reinterpret_cast<bf16x8*>(As + (j & 1) * T64_ASLOT + (i < 4 ? wv + NW * i : 16) * 1024 + lane * 16);
          const bf16x8 x = *xp;
          bf16x8 y;
#pragma unroll
          for (int e = 0; e < 8; ++e) y[e] = (__bf16)fmaxf(fmaf((float)x[e], psc[e], psh[e]), 0.f);
          *xp = y;
          if (a.pa_out && row >= 1 && row <= BM)
            *reinterpret_cast<bf16x8*>(a.pa_out + (long)g * 64 + 8 * ((lane & 7) ^ (row & 7))) = y;
        }
      }
    }
    __syncthreads();                                  // ... every wave's; slot (j+1)&1 is no longer read
    if (j + 1 < ntiles) issue_a((gm + (j + 1) * GM) * BM, (j + 1) & 1);
    const unsigned char* Aj = As + (j & 1) * T64_ASLOT;
    unsigned ok0 = 0u, ok2 = 0u;  // tap 0 reads the previous sample at t == 0, tap 2 the next at t == L-1
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const int m = m0 + wr * WM + 16 * f + (lane & 15);
      const int t = m - (m / L) * L;
      ok0 |= (t != 0 ? 1u : 0u) << f;
      ok2 |= (t != L - 1 ? 1u : 0u) << f;
    }
    f32x4 acc[FM][FN];
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int q = 0; q < FN; ++q) acc[f][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
      const unsigned char* Bs = Ws + tap * 8192;
      const unsigned okm = tap == 0 ? ok0 : ok2;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cc = 4 * ks + (lane >> 4);
        const int asw = (cc ^ ((lane + tap) & 7)) << 4, bsw = (cc ^ (lane & 7)) << 4;
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          af[f] = *reinterpret_cast<const bf16x8*>(Aj + arow + (16 * f + tap) * 128 + asw);
          if (tap != 1 && !((okm >> f) & 1u)) af[f] = bf16x8{};
        }
#pragma unroll
        for (int q = 0; q < FN; ++q) bfr[q] = *reinterpret_cast<const bf16x8*>(Bs + brow + 16 * q * 128 + bsw);
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int q = 0; q < FN; ++q)
            acc[f][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], bfr[q], acc[f][q], 0, 0, 0);
      }
    }
    // tile j's output through the epilogue's own LDS region (A'(j+1) keeps landing in its slot meanwhile)
    fwd_epi_tile_rowwise<BM, BN, EPI, NWR>(a, acc, eps, k, m0, 0, L, M, 1, 0);
  }
  if (a.stats) {
    fwd_epi_stats<BM, BN, EPI, NWR>(a, eps, k, 0, gm, GM);
    if (a.tail) ecg::bn_tail<T64Cfg::NTHR>(a.tail, a.stats, EPI == 1 && a.szd ? 3 : 2, GM, a.Cout, gm, 0, BN, smem);
  }
}

// ECG_CONV_TAP64=0|1: the persistent 64-channel tap kernel (1, default) for C_in == C_out == 64 stride-1 3-tap
// convs over whole samples; 0: the one-tap multi-tile kernel.  Read once.
int g_conv_tap64 = -1;
inline bool conv_tap64() {
  if (g_conv_tap64 < 0) {
    const char* e = getenv("ECG_CONV_TAP64");
    g_conv_tap64 = e ? atoi(e) : 1;
  }
  return g_conv_tap64 != 0;
}
inline bool tap64_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad, int in_dil) {
  return conv_tap64() && Cin == 64 && Cout == 64 && Kw == 3 && stride == 1 && pad == 1 && in_dil == 1 && Lin == Lout &&
         Lout >= 2 && (long)B * Lout * 64 * 2 < 0x7fff0000L;
}
inline int tap64_groups(int B, int Lout) {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev))
      cus = 256;
  }
  const int MT = (int)(((long)B * Lout + T64_BM - 1) / T64_BM);
  return MT < 2 * cus ? MT : 2 * cus;
}

template <int EPI, bool PA = false>
int launch_tap64_t(const FwdArgs& a, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_tap64_kernel<EPI, PA>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, T64_SMEM));
    attr = true;
  }
  const int MT = (int)(((long)a.B * a.Lout + T64_BM - 1) / T64_BM), GM = tap64_groups(a.B, a.Lout);
  hipLaunchKernelGGL((conv1d_nlc_tap64_kernel<EPI, PA>), dim3((unsigned)GM), dim3(256), T64_SMEM, stream, a, MT, GM);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int launch_tap64(const FwdArgs& a, hipStream_t stream) {
  if (a.pa_scale) return a.stat_mode == 1 ? ecg::kBadArg : launch_tap64_t<0, true>(a, stream);  // (forward convs)
  return a.stat_mode == 1 ? launch_tap64_t<1>(a, stream) : launch_tap64_t<0>(a, stream);
}

// The tap-shared kernel applies to stride-1, pad-1, 3-tap convs over whole samples with BN | C_out (BN = 128 when
// C_out % 128 == 0, else 64) and 32-bit addressable operands.
inline bool tap_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad, int in_dil) {
  return Kw == 3 && stride == 1 && pad == 1 && in_dil == 1 && Lin == Lout && Lout >= 2 && Cin % 64 == 0 &&
         Cout % 64 == 0 && (long)B * Lout * Cin * 2 < 0x7fff0000L && (long)Cout * 3 * Cin * 2 < 0x7fff0000L;
}
inline int tap_mtiles(int B, int Lout) { return (int)(((long)B * Lout + TAP_BM - 1) / TAP_BM); }

template <int BN, int EPI, bool PA = false>
int launch_fwd_tap_t(const FwdArgs& a, hipStream_t stream) {
  constexpr int SMEM = TapCfg<BN, PA>::SMEM;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_tap_kernel<BN, EPI, PA>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int MT = tap_mtiles(a.B, a.Lout), NT = a.Cout / BN;
  hipLaunchKernelGGL((conv1d_nlc_fwd_tap_kernel<BN, EPI, PA>), dim3((unsigned)(MT * NT)), dim3(512), SMEM, stream, a,
                     MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int launch_fwd_tap(const FwdArgs& a, hipStream_t stream) {
  const bool b = a.stat_mode == 1;
  if (a.pa_scale) {  // input pre-activation (forward convs): 128-column tiles (ecg_conv1d_nlc_pa_ok)
    if (b || a.Cout % 128 || a.Cin > PA_MAXC) return ecg::kBadArg;
    return launch_fwd_tap_t<128, 0, true>(a, stream);
  }
  if (a.Cout % 128 == 0) return b ? launch_fwd_tap_t<128, 1>(a, stream) : launch_fwd_tap_t<128, 0>(a, stream);
  return b ? launch_fwd_tap_t<64, 1>(a, stream) : launch_fwd_tap_t<64, 0>(a, stream);
}

// ECG_CONV_TAP_S2=1|0: the tap-shared strided data-grad kernel (1, default) for the data-grads of stride-2 pad-1
// 3-tap convs, or the phase-decomposed one-tap kernels (0).  Read once.
int g_conv_tap_s2 = -1;
inline bool conv_tap_s2() {
  if (g_conv_tap_s2 < 0) {
    const char* e = getenv("ECG_CONV_TAP_S2");
    g_conv_tap_s2 = e ? atoi(e) : 1;
  }
  return g_conv_tap_s2 != 0;
}
// The call shape of such a data-grad: dz [B][Lin][Cin] read with input dilation 2, 3 flipped taps, pad 1, output
// length 2*Lin - 1 or 2*Lin (the forward's input length), 32-bit addressable operands.
inline bool tap_s2_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad, int in_dil) {
  return conv_tap_s2() && Kw == 3 && stride == 1 && pad == 1 && in_dil == 2 && (Lout + 1) / 2 == Lin && Lin >= 2 &&
         Cin % 64 == 0 && Cout % 64 == 0 && (long)B * Lin * Cin * 2 < 0x7fff0000L &&
         (long)Cout * 3 * Cin * 2 < 0x7fff0000L && (long)B * Lout * Cout < 0x7fffffffL;
}
inline int tap_s2_mtiles(int B, int Lin) { return (int)(((long)B * Lin + S2_IR - 1) / S2_IR); }

template <int BN, int EPI>
int launch_dgrad_s2_t(const FwdArgs& a, hipStream_t stream) {
  constexpr int SMEM = TapS2Cfg<BN>::SMEM;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_dgrad_s2_tap_kernel<BN, EPI>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int MT = tap_s2_mtiles(a.B, a.Lin), NT = a.Cout / BN;
  hipLaunchKernelGGL((conv1d_nlc_dgrad_s2_tap_kernel<BN, EPI>), dim3((unsigned)(MT * NT)), dim3(512), SMEM, stream, a,
                     MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int launch_dgrad_s2(const FwdArgs& a, hipStream_t stream) {
  const bool b = a.stat_mode == 1;
  if (a.Cout % 128 == 0) return b ? launch_dgrad_s2_t<128, 1>(a, stream) : launch_dgrad_s2_t<128, 0>(a, stream);
  return b ? launch_dgrad_s2_t<64, 1>(a, stream) : launch_dgrad_s2_t<64, 0>(a, stream);
}

// ECG_CONV_TAP=0|1|2: the tap-shared 256-row kernel for eligible convs with C_out % 128 == 0 (1, default), also
// for 64-channel outputs (2), or never (0).  Read once.
int g_conv_tap = -1;
inline int conv_tap_mode() {
  if (g_conv_tap < 0) {
    const char* e = getenv("ECG_CONV_TAP");
    g_conv_tap = e ? atoi(e) : 1;
  }
  return g_conv_tap;
}
inline bool conv_tap(int Cout) {
  const int v = conv_tap_mode();
  return v >= 2 || (v == 1 && Cout % 128 == 0);
}

inline int conv_big();
inline int conv_mt();

// Tile choice for the one-tap kernels (every conv the tap-shared kernel does not take: strided convs, 1x1 downsample
// convs, strided data-grads, 64-channel outputs): 256x256 (8 waves of 64x128) when that gives >= 2 tiles per CU (one
// workgroup per CU; half the L2->LDS bytes per MAC of 128x128: 1.04 vs 0.87 PF/s on the ResNet layer-4 shape at
// B=4096, profiles/r1_resnet/cmb_p3_big*.log), 256x128 only in the opt-in family 2 (measured neutral), else 128x128
// when that still gives >= 1 workgroup per CU, else 128x64, else 64x64.
inline void pick_fwd_tile(long M, int Cout, int in_dil, int* bm, int* bn) {
  const long mt128 = (M + 127) / 128, mt256 = (M + 255) / 256;
  const int big = in_dil == 1 ? conv_big() : 0;
  if (big >= 1 && Cout % 256 == 0 && mt256 * (Cout / 256) >= 512) {
    *bm = 256;
    *bn = 256;
  } else if (big >= 2 && Cout % 128 == 0 && mt256 * (Cout / 128) >= 512) {
    *bm = 256;
    *bn = 128;
  } else if (Cout == 128 && in_dil == 1 && conv_mt() >= 2 && mt128 * 2 > 512) {
    *bm = 128;  // multi-tile 128x64 (mode 2)
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

// Multi-tile forward workgroups (conv1d_nlc_fwd_dma_mt_kernel) for 128x64 tiles when the launch has more tiles than
// two resident workgroups per CU (1, default), also for the 128-channel shapes that would otherwise take 128x128 tiles
// (2), or never (0): ecg_conv1d_nlc_set_mt (tests).
int g_conv_mt = 1;
inline int conv_mt() { return g_conv_mt; }

// Workgroups along M of the multi-tile forward (0: the one-tile-per-workgroup kernels run).  A function of the
// shape and the tile alone, so the host can size the BatchNorm partial rows (ecg_conv1d_nlc_fwd_stat_tiles).
inline int fwd_mt_groups(long M, int Cout, int in_dil, int bm, int bn) {
  if (in_dil != 1 || conv_mt() == 0 || bm != 128 || bn != 64) return 0;
  const long MT = (M + bm - 1) / bm, NT = Cout / bn;
  const long slots = 2L * 256;  // two workgroups per CU
  if (MT * NT <= slots) return 0;
  const long tpw = (MT * NT + slots - 1) / slots;
  return (int)((MT + tpw - 1) / tpw);
}

// 256-row one-tap tiles: 0 = 128-row tiles only, 1 (default) = + 256x256 forward, 2 = + 256x128 forward and 256x256
// weight-gradient tiles (opt-in family; ecg_conv1d_nlc_set_big, tests).  Plans built before a change keep their tiling.
int g_conv_big = 1;
inline int conv_big() { return g_conv_big; }

template <int BM, int BN, int EPI, int NWR = (BM >= 256 ? 4 : 2)>  // 256-row tiles: 8 waves of 64 x BN/2
int launch_fwd_dma_st(const FwdArgs& a, hipStream_t stream) {
  using Cfg = FwdCfg<BM, BN, NWR>;
  constexpr int STAGE_BYTES = 2 * (BM + BN) * 128;
  constexpr int SMEM = STAGE_BYTES > Cfg::EP_BYTES ? STAGE_BYTES : Cfg::EP_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_dma_kernel<BM, BN, EPI, NWR>,
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
  hipLaunchKernelGGL((conv1d_nlc_fwd_dma_kernel<BM, BN, EPI, NWR>), dim3((unsigned)(MT * NT)), dim3(Cfg::NTHR), SMEM,
                     stream, b, MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
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
  return launch_fwd_dma_st<BM, BN, EPI>(a, stream);
}

// Register-staged loop: the fallback for operands beyond the LDS-DMA loop's 32-bit buffer offsets (and, with
// ecg_conv1d_nlc_set_dma_dil(0), the strided data-grads - a test cross-check).
template <int BM, int BN, int EPI>
int launch_fwd_cfg(const FwdArgs& a, hipStream_t stream) {
  using Cfg = FwdCfg<BM, BN>;
  constexpr int SMEM = Cfg::smem(1);
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_fwd_kernel<BM, BN, EPI>,
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
  hipLaunchKernelGGL((conv1d_nlc_fwd_kernel<BM, BN, EPI>), dim3((unsigned)(MT * NT)), dim3(THREADS), SMEM, stream, b,
                     MT, NT);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

// Strided (phase-decomposed) data-grads on the LDS-DMA loop (1, default) or the register-staged loop (0):
// ecg_conv1d_nlc_set_dma_dil (tests: the two are bitwise equal).
int g_conv_dma_dil = 1;
inline bool conv_dma_dil() { return g_conv_dma_dil == 1; }

template <int BM, int BN>
int launch_fwd(const FwdArgs& a, hipStream_t stream) {
  // the DMA loop addresses bytes with 32-bit buffer offsets from the tile's first sample
  const int Lrow = a.in_dil > 1 ? (a.Lout + a.in_dil - 1) / a.in_dil : a.Lout;
  const bool dma_ok = (a.in_dil == 1 || (conv_dma_dil() && a.stride == 1 && BM <= 128)) &&
                      (long)(BM / Lrow + 2) * a.Lin * a.Cin * 2 < 0x7fff0000L &&
                      (long)a.Cout * a.Kw * a.Cin * 2 < 0x7fff0000L;
  if (dma_ok && a.in_dil > 1)  // two stages, one tile per workgroup
    return a.stat_mode == 1 ? launch_fwd_dma_st<BM, BN, 1>(a, stream) : launch_fwd_dma_st<BM, BN, 0>(a, stream);
  if (dma_ok) return a.stat_mode == 1 ? launch_fwd_dma<BM, BN, 1>(a, stream) : launch_fwd_dma<BM, BN, 0>(a, stream);
  if (a.stats && fwd_mt_groups((long)a.B * a.Lout, a.Cout, a.in_dil, BM, BN) > 0)
    return ecg::kBadArg;  // the host sized the partial rows for the multi-tile kernel
  if constexpr (BM > 128) return ecg::kBadArg;  // 256-row tiles exist only as DMA kernels (the picker ensures it)
  else return a.stat_mode == 1 ? launch_fwd_cfg<BM, BN, 1>(a, stream) : launch_fwd_cfg<BM, BN, 0>(a, stream);
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

// Two-group LDS-DMA weight gradient (128x128 tiles, 8 waves): the workgroup's row-chunk range is split between two
// 4-wave groups that run the loop above side by side (each with its own two LDS stages, in lockstep on the one
// workgroup barrier); at the end group 1 hands its accumulators to group 0 through LDS and group 0 stores the sum.
// So one 8-wave workgroup per CU does the work of two 4-wave workgroups while writing ONE 64 KB partial tile: the
// split-K partial traffic (written here, re-read by the reduce) halves at equal occupancy, and the launch needs half
// the workgroups for the same depth of work per CU.
template <int NG>
__global__ __launch_bounds__(256 * NG, 1) void conv1d_nlc_wgrad_dma2_kernel(WgradArgs a, int TM, int TN,
                                                                                          int splits) {
  constexpr int BM = 128, BN = 128, NWR = 2;
  using Cfg = WgCfg<BM, BN, NWR>;
  constexpr int WM = Cfg::WM, WN = Cfg::WN, FM = Cfg::FM, FN = Cfg::FN, NW = Cfg::NW;  // per group: 4 waves
  constexpr int RA = BM * 2, RB = BN * 2;
  constexpr int A_BYTES = 64 * RA, STAGE = 64 * (RA + RB);  // 32 KB
  constexpr int AP = A_BYTES / 1024 / NW, BP = 64 * RB / 1024 / NW;
  constexpr int RPP = 1024 / RA, SH = 4, SLOT = RA / 16 - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wg = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave in the workgroup
  const int grp = wg >> 2, wv = wg & 3;                      // group, wave in the group
  const int wr = wv >> 1, wc = wv & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int tiles = TM * TN;
  const int split = wgid / tiles, tile = wgid % tiles;
  const int co0 = (tile / TN) * BM, n0 = (tile % TN) * BN;
  const int k = n0 / a.Cin, c0 = n0 % a.Cin;
  const int R = a.B * a.Lout;
  const int nchunks = (R + 63) / 64;
  const int w0 = split * a.chunks_per_split, w1 = min(nchunks, w0 + a.chunks_per_split);  // the workgroup's chunks
  const int half = (w1 - w0 + NG - 1) / NG;                                              // lockstep steps
  const int ch0 = min(w1, w0 + grp * half), ch1 = min(w1, ch0 + half);                   // this group's chunks
  unsigned char* const gs = smem + grp * 2 * STAGE;                                      // this group's stages
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (w0 < w1) {  // block-uniform
    const int r0 = w0 * 64, b0 = r0 / a.Lout;
    const long dyrem = (long)(R - r0) * a.Cout * 2, xrem = (long)(a.B - b0) * a.Lin * a.Cin * 2;
    const srd_t dyr = make_rsrc(a.dy + (long)r0 * a.Cout, dyrem < 0x7fff0000L ? dyrem : 0x7fff0000L);
    const srd_t xr = make_rsrc(a.x + (long)b0 * a.Lin * a.Cin, xrem < 0x7fff0000L ? xrem : 0x7fff0000L);
    const unsigned lds_g = lds_addr(gs);
    int arow[AP], brow[BP];
    unsigned asrc[AP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      arow[i] = RPP * (wv + NW * i) + (lane >> SH);
      asrc[i] = (unsigned)((co0 + ((lane & SLOT) ^ wg_swz(arow[i])) * 8) * 2);
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) brow[i] = RPP * (wv + NW * i) + (lane >> SH);
    auto issue = [&](int ch, int st) {
      const unsigned base = lds_g + st * STAGE;
      const int rel = (ch - w0) * 64;
#pragma unroll
      for (int i = 0; i < AP; ++i) {
        const int r = rel + arow[i];
        const unsigned voff = r0 + r < R ? (unsigned)(r * a.Cout * 2) + asrc[i] : 0x7ffffff0u;
        dma16_at(dyr, voff, base + (wv + NW * i) * 1024);
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
        dma16_at(xr, voff, base + A_BYTES + (wv + NW * i) * 1024);
      }
    };
    const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, h = lane >> 4;
    auto tr_at = [&](const unsigned char* img, int RB_, int rr, int col) -> s16x4 {
      return tr16(reinterpret_cast<const __bf16*>(img + rr * RB_ + ((((col >> 3) ^ wg_swz(rr))) << 4) +
                                                  ((col & 7) << 1)));
    };
    auto mma = [&](int st) {
      const unsigned char* As = gs + st * STAGE;
      const unsigned char* Bs = As + A_BYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
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
    const int n = ch1 - ch0;  // 0 <= n <= half (group 1 may have fewer chunks, or none)
    if (n > 0) issue(ch0, 0);
    for (int i = 0; i < half; ++i) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // step i's stage landed; step i-1's reads done
      __builtin_amdgcn_s_barrier();
      if (i + 1 < n) issue(ch0 + i + 1, (i + 1) & 1);  // into the stage step i-1 read
      if (i < n) mma(i & 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // every stage is dead
  if constexpr (NG == 2) {  // group 1 -> LDS (lane-linear per accumulator: no conflicts) -> group 0 adds
    f32x4* red = reinterpret_cast<f32x4*>(smem) + wv * (FM * FN * 64) + lane;
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) red[(i * FN + j) * 64] = acc[i][j];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] += red[(i * FN + j) * 64];
    }
  }
  // group 0's waves store the partial tile (LDS-staged float4 rows, as wgrad_epilogue); group 1 joins the barriers
  constexpr int EP_LD = Cfg::EP_LD, HR = WM / 2;
  float* ep = reinterpret_cast<float*>(smem) + (NG == 2 ? 64 * 1024 / 4 : 0) + wv * HR * EP_LD;  // past red[]
  constexpr int C4 = WN / 4, RSTEP = 64 / C4;
  const int c4 = lane % C4, rs = lane / C4;
  const long N = (long)a.Kw * a.Cin;
  float* out = a.part + (long)split * a.Cout * N;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < FM / 2; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
            ep[(i * 16 + 4 * (lane >> 4) + qq) * EP_LD + j * 16 + (lane & 15)] = acc[hh * (FM / 2) + i][j][qq];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll 4
      for (int r = rs; r < HR; r += RSTEP) {
        const float4 v = *reinterpret_cast<const float4*>(ep + r * EP_LD + c4 * 4);
        *reinterpret_cast<float4*>(out + (long)(co0 + wr * WM + hh * HR + r) * N + n0 + wc * WN + c4 * 4) = v;
      }
    }
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

// The tap-shared weight gradient applies to stride-1, pad-1, 3-tap convs with whole tensors addressable with 32-bit
// offsets and at most 64 channels (measured on MI355X, B=1024 ResNet1D-34 shapes, scripts/wgrad_micro.py,
// profiles/r3/wgrad_ts_ab.txt - 14.1 vs 21.6 us at 64 channels, where the one-tap path is the register-staged 64x64
// kernel; slower than the one-tap 128x128 LDS-DMA kernel at 128-512 channels).  It aims for 256 workgroups (one per
// CU; the split-K partials are workgroups x 48 KB) and runs a four-stage ring (two chunks in flight).
constexpr int WGRAD_TS_MAXC = 64, WGRAD_TS_WGS = 256, WGRAD_TS_NST = 4;
inline bool wgrad_ts_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad) {
  const long R = (long)B * Lout;
  return Cin <= WGRAD_TS_MAXC && Cout <= WGRAD_TS_MAXC && Kw == 3 && stride == 1 && pad == 1 && Lin == Lout &&
         Lout >= 8 && Cin % 64 == 0 && Cout % 64 == 0 && R * Cout * 2 < 0x7fff0000L && R * Cin * 2 < 0x7fff0000L;
}

int launch_wgrad_ts(const WgradArgs& a, int splits, hipStream_t stream) {
  constexpr int SMEM = WGRAD_TS_NST * TSW_STAGE;
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_wgrad_ts_kernel<WGRAD_TS_NST>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int TM = a.Cout / 64, TN = a.Cin / 64;
  hipLaunchKernelGGL(conv1d_nlc_wgrad_ts_kernel<WGRAD_TS_NST>, dim3((unsigned)(TM * TN * splits)), dim3(256), SMEM,
                     stream, a, TM, TN, splits);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
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

int launch_wgrad_dma2(const WgradArgs& a, int splits, hipStream_t stream) {
  constexpr int SMEM = 2 * 2 * 64 * (128 + 128) * 2;  // two groups x two stages x 32 KB
  static bool attr = false;
  if (!attr) {
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)conv1d_nlc_wgrad_dma2_kernel<2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int TM = a.Cout / 128, TN = a.Kw * a.Cin / 128;
  hipLaunchKernelGGL((conv1d_nlc_wgrad_dma2_kernel<2>), dim3((unsigned)(TM * TN * splits)), dim3(512), SMEM, stream, a,
                     TM, TN, splits);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
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
// ``relu``: bit 0 = ReLU on the output; bit 1 = bnb[0] is the mask as bits (FwdArgs::smask_bits).
// ``bnb`` (optional, stat_mode 1): {smask, sz, smean, srstd, szd, smean_d, srstd_d, mscale, mshift} of the
// BatchNorm whose backward statistics the data-grad epilogue produces ([2 or 3][M tiles][Cout] into ``stats``);
// mscale / mshift (both or neither) re-derive the ReLU mask from sz instead of reading smask.
// ``tail`` (optional, with ``stats``): a BatchNorm finalize fused into this launch (bn_tail.h).
// Whether ecg_conv1d_nlc_fwd_pa accepts an input pre-activation for this conv (it routes to the persistent
// 64-channel tap kernel or to the 128-column tap-shared kernel).
ECG_API int ecg_conv1d_nlc_pa_ok(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad,
                                 int in_dil) {
  if (tap64_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return 1;
  return conv_tap(Cout) && Cout % 128 == 0 && Cin <= PA_MAXC && tap_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)
             ? 1
             : 0;
}

ECG_API int ecg_conv1d_nlc_fwd_pa(const void* x, const void* w, const float* bias, void* y, float* stats,
                                  const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                  int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                  const void* tail, const void* const* pa, hipStream_t stream);

ECG_API int ecg_conv1d_nlc_fwd_ex(const void* x, const void* w, const float* bias, void* y, float* stats,
                                  const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                  int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                  const void* tail, hipStream_t stream) {
  return ecg_conv1d_nlc_fwd_pa(x, w, bias, y, stats, add, add_mask, B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil,
                               relu, bnb, tail, nullptr, stream);
}

// ecg_conv1d_nlc_fwd_ex with an input pre-activation ``pa`` = {scale, shift, out} (FwdArgs::pa_*; null = none):
// the conv's operand is bf16(relu(x * scale + shift)) per input channel, and the activated rows are also stored to
// ``out`` (null: not stored).  Forward convs (no ``bnb``) where ecg_conv1d_nlc_pa_ok holds.
ECG_API int ecg_conv1d_nlc_fwd_pa(const void* x, const void* w, const float* bias, void* y, float* stats,
                                  const void* add, const void* add_mask, int B, int Lin, int Cin, int Lout, int Cout,
                                  int Kw, int stride, int pad, int in_dil, int relu, const void* const* bnb,
                                  const void* tail, const void* const* pa, hipStream_t stream) {
  if (!x || !w || !y || B <= 0 || Lin <= 0 || Lout <= 0 || Kw <= 0 || stride <= 0 || in_dil <= 0 || pad < 0)
    return ecg::kBadArg;
  if (pa && (!pa[0] || !pa[1] || !ecg_conv1d_nlc_pa_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)))
    return ecg::kBadArg;
  if (Cin % BK != 0 || Cout % 64 != 0 || (add_mask && !add)) return ecg::kBadArg;
  if (bnb && (!stats || !bnb[1] || !bnb[2] || !bnb[3] || (bnb[4] && (!bnb[5] || !bnb[6])) || (!bnb[7] != !bnb[8])))
    return ecg::kBadArg;
  if (tail && !stats) return ecg::kBadArg;
  FwdArgs a{static_cast<const __bf16*>(x), static_cast<const __bf16*>(w), bias, static_cast<__bf16*>(y), stats,
            static_cast<const __bf16*>(add), static_cast<const __bf16*>(add_mask),
            B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil, relu & 1, bnb ? 1 : 0};
  if (bnb) {
    a.mscale = static_cast<const float*>(bnb[7]);
    a.mshift = static_cast<const float*>(bnb[8]);
    if (relu & 2)  // the mask operand is a bit mask (FwdArgs::smask_bits)
      a.smask_bits = static_cast<const uint8_t*>(bnb[0]);
    else
      a.smask = static_cast<const __bf16*>(bnb[0]);
    a.sz = static_cast<const __bf16*>(bnb[1]);
    a.smean = static_cast<const float*>(bnb[2]);
    a.srstd = static_cast<const float*>(bnb[3]);
    a.szd = static_cast<const __bf16*>(bnb[4]);
    a.smean_d = static_cast<const float*>(bnb[5]);
    a.srstd_d = static_cast<const float*>(bnb[6]);
  }
  a.tail = static_cast<const ecg::BnTail*>(tail);
  if (pa) {
    a.pa_scale = static_cast<const float*>(pa[0]);
    a.pa_shift = static_cast<const float*>(pa[1]);
    a.pa_out = static_cast<__bf16*>(const_cast<void*>(pa[2]));
    return tap64_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil) ? launch_tap64(a, stream)
                                                                      : launch_fwd_tap(a, stream);
  }
  if (tap64_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return launch_tap64(a, stream);
  if (conv_tap(Cout) && tap_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return launch_fwd_tap(a, stream);
  if (tap_s2_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return launch_dgrad_s2(a, stream);
  int bm, bn;
  pick_fwd_tile((long)B * Lout, Cout, in_dil, &bm, &bn);
  if (bm == 256 && bn == 256) return launch_fwd<256, 256>(a, stream);
  if (bm == 256) return launch_fwd<256, 128>(a, stream);
  if (bm == 128 && bn == 128) return launch_fwd<128, 128>(a, stream);
  if (bm == 128) return launch_fwd<128, 64>(a, stream);
  return launch_fwd<64, 64>(a, stream);
}

// Persistent 64-channel tap kernel on (1) / off (0); returns the previous setting (tests, A/B).  Step plans size
// their BatchNorm partial rows when built: set it first.
ECG_API int ecg_conv1d_nlc_set_tap64(int on) {
  const int prev = conv_tap64() ? 1 : 0;
  g_conv_tap64 = on ? 1 : 0;
  return prev;
}

// Tap-shared strided data-grad kernel on (1) / off (0); returns the previous setting (tests, A/B).  Step plans size
// their BatchNorm partial rows when built: set it first.
ECG_API int ecg_conv1d_nlc_set_tap_s2(int on) {
  const int prev = conv_tap_s2() ? 1 : 0;
  g_conv_tap_s2 = on ? 1 : 0;
  return prev;
}

// Strided data-grads on the LDS-DMA loop (1) or the register-staged loop (0); returns the previous setting (tests).
ECG_API int ecg_conv1d_nlc_set_dma_dil(int on) {
  const int prev = conv_dma_dil() ? 1 : 0;
  g_conv_dma_dil = on ? 1 : 0;
  return prev;
}

// Select the tap-shared kernel mode (see conv_tap); returns the previous setting.  Step plans size their BatchNorm
// partial rows when built: set it first.
ECG_API int ecg_conv1d_nlc_set_tap(int mode) {
  const int prev = conv_tap_mode();
  g_conv_tap = mode < 0 ? 0 : (mode > 2 ? 2 : mode);
  return prev;
}

// Select the one-tap tile family (see conv_big); returns the previous setting.
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

// Rows of BatchNorm partials for the kernel that runs this exact conv (any stride / taps / dilation): the
// tap-shared kernel's 256-row M tiles where it applies, else the tile-family rows below.
ECG_API int ecg_conv1d_nlc_fwd_stat_tiles_ex(int B, int Lout, int Cout, int in_dil);
ECG_API int ecg_conv1d_nlc_fwd_stat_rows(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad,
                                         int in_dil) {
  if (tap64_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return tap64_groups(B, Lout);
  if (conv_tap(Cout) && tap_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return tap_mtiles(B, Lout);
  if (tap_s2_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil)) return tap_s2_mtiles(B, Lin);
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

// LDS-DMA weight-gradient loops: 32-bit buffer offsets from the split's first row / sample (cps row chunks of 64).
inline bool wgrad_dma_ok(long cps, int Lin, int Cin, int Lout, int Cout) {
  const long rows = cps * 64;
  return rows * Cout * 2 < 0x7fff0000L && (rows / Lout + 2) * (long)Lin * Cin * 2 < 0x7fff0000L;
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
  const bool dma_ok = wgrad_dma_ok(cps, Lin, Cin, Lout, Cout);
  if (wgrad_big(Cout, Cin)) return dma_ok ? launch_wgrad_dma<256, 256>(a, splits, stream)
                                          : launch_wgrad<256, 256>(a, splits, stream);
  if (bm128 && bn128 && dma_ok) return launch_wgrad_dma2(a, splits, stream);
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

// Split count for the tap-shared weight-gradient kernel (64 x 64 x 3 output blocks, ~WGRAD_TS_WGS workgroups, >= 4
// row chunks each, at most 256 partial slices - the bound the reduce kernels and the engine's workspace assume), or
// 0 when this conv takes the one-tap kernels (the caller then sizes its own splits).
ECG_API int ecg_conv1d_nlc_wgrad_splits(int B, int Lin, int Cin, int Lout, int Cout, int Kw, int stride, int pad) {
  if (!wgrad_ts_ok(B, Lin, Cin, Lout, Cout, Kw, stride, pad)) return 0;
  const long chunks = ((long)B * Lout + 63) / 64;
  const int tiles = (Cout / 64) * (Cin / 64);
  long s = (WGRAD_TS_WGS + tiles - 1) / tiles;
  s = s < chunks / 4 ? s : chunks / 4;
  return (int)(s < 1 ? 1 : (s > 256 ? 256 : s));
}

// Workgroups the weight-gradient launch should aim for (tiles x splits): ~4 resident per CU for the 4-wave
// register-staged tiles, ~2 rounds of one per CU for the 8-wave 256x256 tile.  (B, Lin, Lout) decide whether the
// 128x128 shapes take the two-group LDS-DMA kernel at the split count that target implies; B = 0: assume it does.
ECG_API int ecg_conv1d_nlc_wgrad_target_wgs(int Cout, int Kw, int Cin, int B, int Lin, int Lout) {
  if (wgrad_big(Cout, Cin)) return 512;
  // 128x128 tiles: the two-group 8-wave kernel, a little under one workgroup per CU - 224 (ECG_WGRAD_TARGET, read
  // once): B=1024 ResNet1D-34 3.256-3.275 ms/step at 192-224 workgroups vs 3.30-3.35 at 256, 3.31 at 160-176 and
  // 3.43-3.45 at 128 / 384 on three boxes (profiles/r6/wgrad_target_ab.txt; round 4: 256 beat 512 and 768,
  // profiles/r4/wgrad_g2_ab.txt): the side lane's weight gradients leave CUs to the data-gradient chain - when its
  // 32-bit offsets hold; otherwise the 4-wave register-staged 128x128 kernel, which wants ~4 workgroups per CU
  if (Cout % 128 == 0 && Cin % 128 == 0) {
    if (B <= 0 || Lout <= 0) return 256;
    const int tiles = ecg_conv1d_nlc_wgrad_tiles(Cout, Kw, Cin);
    const long chunks = ((long)B * Lout + 63) / 64;
    long splits = (256 + tiles - 1) / tiles;
    splits = splits < 1 ? 1 : splits;
    const long cps = (chunks + splits - 1) / splits;
    static int tgt = -1;
    if (tgt < 0) {
      const char* e = getenv("ECG_WGRAD_TARGET");
      tgt = e ? atoi(e) : 224;
      if (tgt <= 0) tgt = 224;
    }
    return wgrad_dma_ok(cps, Lin, Cin, Lout, Cout) ? tgt : 1024;
  }
  return 1024;
}
