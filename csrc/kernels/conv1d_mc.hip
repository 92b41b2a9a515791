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
// Block tile 64x64, BK = 64, 4 waves (2x2, 32x32 each = 2x2 MFMA tiles), double-buffered LDS with the next
// tile's global loads issued before the current tile's MFMAs (register staging, write after the barrier).
#include "../include/ecg_common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 64;
constexpr int THREADS = 256;
constexpr int LDS_ROW = BK + 8;  // bf16 elements per LDS row (+16 B pad: conflict-free ds_read_b128)

typedef short s16x8 __attribute__((ext_vector_type(8)));

struct FwdArgs {
  const __bf16* x;    // [B][Lin][Cin]
  const __bf16* w;    // [Cout][Kw][Cin]
  const float* bias;  // [Cout] or nullptr
  __bf16* y;          // [B][Lout][Cout]
  int B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil, relu;
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

__global__ __launch_bounds__(THREADS) void conv1d_nlc_fwd_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][BM * LDS_ROW];  // [buf][A/B][row][k]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int K = a.Kw * a.Cin;
  const int nk = K / BK;
  const int e0 = tid, e1 = tid + THREADS;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  store_one(lds[0][0], e0, load_a_fwd(a, m0, 0, e0));
  store_one(lds[0][0], e1, load_a_fwd(a, m0, 0, e1));
  store_one(lds[0][1], e0, load_b_fwd(a, n0, 0, e0));
  store_one(lds[0][1], e1, load_b_fwd(a, n0, 0, e1));
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // issue the next tile's global loads before this tile's MFMAs (the last iteration re-reads its own tile,
    // keeping the loads unconditional so they stay in registers)
    const int kn = (kt + 1 < nk ? kt + 1 : kt) * BK;
    const uint4 ra0 = load_a_fwd(a, m0, kn, e0), ra1 = load_a_fwd(a, m0, kn, e1);
    const uint4 rb0 = load_b_fwd(a, n0, kn, e0), rb1 = load_b_fwd(a, n0, kn, e1);
    const __bf16* As = lds[cur][0];
    const __bf16* Bs = lds[cur][1];
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wr * 32 + i * 16 + (lane & 15)) * LDS_ROW + ks * 32 +
                                                 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wc * 32 + j * 16 + (lane & 15)) * LDS_ROW + ks * 32 +
                                                  8 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __bf16* An = lds[cur ^ 1][0];
    __bf16* Bn = lds[cur ^ 1][1];
    store_one(An, e0, ra0);
    store_one(An, e1, ra1);
    store_one(Bn, e0, rb0);
    store_one(Bn, e1, rb1);
    __syncthreads();
  }
  // epilogue: C layout row = 4*(lane>>4) + i, col = lane & 15
  const int M = a.B * a.Lout;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 32 + j * 16 + (lane & 15);
      const float bv = a.bias ? a.bias[n] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + wr * 32 + i * 16 + 4 * (lane >> 4) + q;
        if (m < M) {
          float v = acc[i][j][q] + bv;
          if (a.relu) v = fmaxf(v, 0.f);
          a.y[(long)m * a.Cout + n] = (__bf16)v;
        }
      }
    }
}

// ------------------------------------------------------------------------------------------- weight grad
struct WgradArgs {
  const __bf16* dy;  // [B][Lout][Cout]
  const __bf16* x;   // [B][Lin][Cin]
  float* part;       // [splits][Cout][Kw*Cin] fp32 partials
  int B, Lin, Cin, Lout, Cout, Kw, stride, pad, chunks_per_split;
};

constexpr int WG_ROW = 64 + 4;  // bf16 per LDS row for the [r][c] images (136 B: 8-B aligned tr reads)

__device__ __forceinline__ s16x4 tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__global__ __launch_bounds__(THREADS) void conv1d_nlc_wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][64 * WG_ROW];  // [dy tile | x tile], rows = r
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int co0 = blockIdx.x * 64;
  const int n0 = blockIdx.y * 64;  // n = k*Cin + ci, tile inside one tap (Cin % 64 == 0)
  const int k = n0 / a.Cin, c0 = n0 % a.Cin;
  const int R = a.B * a.Lout;
  const int nchunks = (R + 63) / 64;
  const int ch0 = blockIdx.z * a.chunks_per_split;
  const int ch1 = min(nchunks, ch0 + a.chunks_per_split);
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4, h = lane >> 4;
  for (int ch = ch0; ch < ch1; ++ch) {
    const int r0 = ch * 64;
    __syncthreads();  // previous chunk's reads done
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int e = tid + it * THREADS;  // 0..511: row = e >> 3, part = e & 7 (8 bf16 each)
      const int row = e >> 3, part = e & 7;
      const int r = r0 + row;
      uint4 vdy = make_uint4(0u, 0u, 0u, 0u), vx = make_uint4(0u, 0u, 0u, 0u);
      if (r < R) {
        vdy = *reinterpret_cast<const uint4*>(a.dy + (long)r * a.Cout + co0 + part * 8);
        const int b = r / a.Lout, t = r % a.Lout;
        const int u = t * a.stride + k - a.pad;
        if (u >= 0 && u < a.Lin) vx = *reinterpret_cast<const uint4*>(a.x + ((long)b * a.Lin + u) * a.Cin + c0 + part * 8);
      }
      *reinterpret_cast<uint2*>(lds[0] + row * WG_ROW + part * 8) = make_uint2(vdy.x, vdy.y);
      *reinterpret_cast<uint2*>(lds[0] + row * WG_ROW + part * 8 + 4) = make_uint2(vdy.z, vdy.w);
      *reinterpret_cast<uint2*>(lds[1] + row * WG_ROW + part * 8) = make_uint2(vx.x, vx.y);
      *reinterpret_cast<uint2*>(lds[1] + row * WG_ROW + part * 8 + 4) = make_uint2(vx.z, vx.w);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {  // two 32-deep k-steps over r
      bf16x8 af[2], bfr[2];
      // lane quarter h covers r = ks*32 + 8h .. +7 ; transposing reads give column (lane&15) of 4 rows
      const int rr = ks * 32 + 8 * h + q;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wr * 32 + i * 16 + p4;
        typedef short s16x8v __attribute__((ext_vector_type(8)));
        const s16x4 lo = tr16(lds[0] + rr * WG_ROW + col);
        const s16x4 hi = tr16(lds[0] + (rr + 4) * WG_ROW + col);
        s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wc * 32 + j * 16 + p4;
        typedef short s16x8v __attribute__((ext_vector_type(8)));
        const s16x4 lo = tr16(lds[1] + rr * WG_ROW + col);
        const s16x4 hi = tr16(lds[1] + (rr + 4) * WG_ROW + col);
        s16x8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  // partial[split][co][n]
  const int N = a.Kw * a.Cin;
  float* out = a.part + (long)blockIdx.z * a.Cout * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int co = co0 + wr * 32 + i * 16 + 4 * (lane >> 4) + qq;
        out[(long)co * N + n] = acc[i][j][qq];
      }
    }
}

}  // namespace

// y = conv(x) (+bias)(+ReLU); x [B][Lin][Cin] bf16, w [Cout][Kw][Cin] bf16, y [B][Lout][Cout] bf16.
// in_dil > 1 reads x as zero-inserted with that dilation (used for the data-gradient of strided convs).
ECG_API int ecg_conv1d_nlc_fwd(const void* x, const void* w, const float* bias, void* y, int B, int Lin, int Cin,
                               int Lout, int Cout, int Kw, int stride, int pad, int in_dil, int relu,
                               hipStream_t stream) {
  if (!x || !w || !y || B <= 0 || Lin <= 0 || Lout <= 0 || Kw <= 0 || stride <= 0 || in_dil <= 0 || pad < 0)
    return ecg::kBadArg;
  if (Cin % BK != 0 || Cout % BN != 0) return ecg::kBadArg;
  FwdArgs a{static_cast<const __bf16*>(x), static_cast<const __bf16*>(w), bias, static_cast<__bf16*>(y),
            B, Lin, Cin, Lout, Cout, Kw, stride, pad, in_dil, relu};
  const long M = (long)B * Lout;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)(Cout / BN));
  hipLaunchKernelGGL(conv1d_nlc_fwd_kernel, grid, dim3(THREADS), 0, stream, a);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
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
              stride, pad, cps};
  dim3 grid((unsigned)(Cout / 64), (unsigned)(Kw * Cin / 64), (unsigned)splits);
  hipLaunchKernelGGL(conv1d_nlc_wgrad_kernel, grid, dim3(THREADS), 0, stream, a);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}
