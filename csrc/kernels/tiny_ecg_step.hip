// Fused TinyECG training step for gfx950 (MI355X, CDNA4).
//
// One workgroup owns one ECG window and runs the WHOLE per-sample training computation out of LDS:
//   gather x[idx[b]]  ->  conv1(1->16,k7,p3)+bias+ReLU (VALU)  ->  conv2(16->16,k5,p2)+bias+ReLU
//   (MFMA bf16 16x16x32, implicit GEMM M=t, N=c_out, K=(tap,c_in)=80->96)  ->  mean-pool  ->
//   Linear(16->C)  ->  softmax-CE  ->  head grads  ->  dconv2 wgrad (MFMA, dh2 kept in the MFMA
//   accumulator layout and used directly as the A operand; h1 read as the B operand with the gfx950
//   transposing LDS read ds_read_b64_tr_b16)  ->  dconv2 dgrad (MFMA)  ->  ReLU mask  ->  dconv1 wgrad.
// It writes this sample's parameter-gradient contribution (1,458 floats for C=2) plus its loss into
// one row of a partial slab; ``slab_reduce_sgd`` then sums the rows and applies SGD+momentum to the
// flat fp32 master weights.  Two launches per step, graph-replayed for a whole FedAvg local round.
//
// Reference semantics being reproduced (per step): Module_3/TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:103-132
// (train_step_G0/G1: fwd, cross_entropy(mean), backward, SGD(lr=1e-2, momentum=0.9).step()) on the
// TinyECG of Module_3/tiny_ecg_model.py:8-29, with batches drawn as in Module_3/shard_dataset.py:118-136.
// Precision: bf16 MFMA operands, fp32 accumulation, fp32 master weights/optimizer state (native bf16 AMP).
#include "../include/ecg_common.h"

namespace {

constexpr int C = 16;   // hidden channels
constexpr int K1 = 7;   // conv1 taps (padding 3)
constexpr int K2 = 5;   // conv2 taps (padding 2)
constexpr int MAX_CLASSES = 16;
constexpr int MAX_PAIRS_PER_WAVE = 4;  // mask bits: 4 pairs x 2 tiles x 4 rows = 32 bits

struct Layout {
  int w1, b1, w2, b2, wh, bh, P;
};

__host__ __device__ inline Layout make_layout(int nc) {
  Layout l;
  l.w1 = 0;
  l.b1 = C * K1;             // 112
  l.w2 = l.b1 + C;           // 128
  l.b2 = l.w2 + C * C * K2;  // 1408
  l.wh = l.b2 + C;           // 1424
  l.bh = l.wh + nc * C;
  l.P = l.bh + nc;
  return l;
}

// LDS carve (bytes), all offsets multiples of 16.
struct Smem {
  int Lp;         // L rounded up to 32 (tile pairs)
  int xs_off, h1_off, dh2_off, red_off, bytes;
};

// red region (floats)
constexpr int RED_DW2 = 0;                  // [16][16][5] = 1280 (param layout co*80+ci*5+k)
constexpr int RED_DW1 = RED_DW2 + 1280;     // [16][8]: k<7 weight grad, k==7 bias grad
constexpr int RED_DB2 = RED_DW1 + 128;      // [16]
constexpr int RED_G = RED_DB2 + 16;         // [16] dL/dh2 scale per channel (dpooled / L)
constexpr int RED_POOL = RED_G + 16;        // [WAVES][16] pooled partials
constexpr int RED_FLOATS_FIXED = RED_POOL;

__host__ __device__ inline Smem make_smem(int L, int waves) {
  Smem s;
  s.Lp = (L + 31) / 32 * 32;
  s.xs_off = 0;
  int xs_bytes = ((s.Lp + 16) * 4 + 15) / 16 * 16;
  s.h1_off = s.xs_off + xs_bytes;
  int act_bytes = (s.Lp + 8) * C * 2;  // bf16 [Lp+8][16]
  s.dh2_off = s.h1_off + act_bytes;
  s.red_off = s.dh2_off + act_bytes;
  int red_bytes = ((RED_FLOATS_FIXED + waves * 16) * 4 + 15) / 16 * 16;
  s.bytes = s.red_off + red_bytes;
  return s;
}

__device__ __forceinline__ bf16x8 cat44(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ s16x4 lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// MODE 0: full training step (grads -> slab row).  MODE 1: forward only (logits -> out [B, nc]).
template <int WAVES, int MODE>
__global__ __launch_bounds__(WAVES * 64) void tiny_ecg_step_kernel(
    const float* __restrict__ X, int L, long ldx,        // dataset windows [N, ldx], window length L
    const int* __restrict__ idx,                         // [B] rows of X for this step (nullptr: b)
    const int* __restrict__ Y,                           // [N] int32 labels (unused in MODE 1)
    const float* __restrict__ params, int nc,            // flat fp32 params
    float* __restrict__ out, int out_stride,             // MODE0: slab [B][out_stride]; MODE1: logits
    float inv_B) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Smem sm = make_smem(L, WAVES);
  const Layout lay = make_layout(nc);
  const int Lp = sm.Lp;
  const int NP = Lp / 32;  // tile pairs (32 time steps each)

  float* xs = reinterpret_cast<float*>(smem + sm.xs_off);
  __bf16* h1s = reinterpret_cast<__bf16*>(smem + sm.h1_off);    // row (t+2), 16 channels
  __bf16* dh2s = reinterpret_cast<__bf16*>(smem + sm.dh2_off);  // row (t+4), 16 channels
  float* red = reinterpret_cast<float*>(smem + sm.red_off);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int h = lane >> 4;   // lane quarter
  const int c = lane & 15;   // channel owned by this lane in C-layout phases
  const int b = blockIdx.x;
  const long row = idx ? (long)idx[b] : (long)b;
  const float* xrow = X + row * ldx;

  // ---------------- phase 0: stage x, zero halos/accumulators, load weights -------------------
  for (int i = tid; i < Lp + 16; i += WAVES * 64) {
    int t = i - 3;
    xs[i] = (t >= 0 && t < L) ? xrow[t] : 0.f;
  }
  {
    // h1 halo rows: index 0,1 (t=-2,-1) and [Lp+2, Lp+8) ; dh2 halo rows: [0,4) and [Lp+4, Lp+8)
    uint32_t* h1w = reinterpret_cast<uint32_t*>(h1s);
    uint32_t* dhw = reinterpret_cast<uint32_t*>(dh2s);
    for (int i = tid; i < 8 * 8; i += WAVES * 64) {  // 8 rows x 8 dwords each
      int r = i >> 3, d = i & 7;
      int hr = r < 2 ? r : Lp + 2 + (r - 2);
      h1w[hr * 8 + d] = 0u;
      int dr = r < 4 ? r : Lp + 4 + (r - 4);
      dhw[dr * 8 + d] = 0u;
    }
    if (MODE == 0)
      for (int i = tid; i < RED_G; i += WAVES * 64) red[i] = 0.f;
  }
  float w1r[K1];
#pragma unroll
  for (int k = 0; k < K1; ++k) w1r[k] = params[lay.w1 + c * K1 + k];
  const float b1r = params[lay.b1 + c];
  const float b2r = params[lay.b2 + c];
  // conv2 forward B operand: B[r][co], r = 32s + 8h + j -> tap = r>>4, ci = r&15, co = c.
  bf16x8 Bf[3];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int r = 32 * s + 8 * h + j, tap = r >> 4, ci = r & 15;
      float v = tap < K2 ? params[lay.w2 + c * (C * K2) + ci * K2 + tap] : 0.f;
      Bf[s][j] = ecg::to_bf16(v);
    }
  __syncthreads();

  // ---------------- phase 1: conv1 + bias + ReLU (VALU) into h1s (bf16) ------------------------
  uint32_t mask1 = 0u, mask2 = 0u;
#pragma unroll
  for (int pi = 0; pi < MAX_PAIRS_PER_WAVE; ++pi) {
    const int pair = w + pi * WAVES;
    if (pair < NP) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int t0 = 32 * pair + 16 * half;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = t0 + 4 * h + i;
          float v = b1r;
#pragma unroll
          for (int k = 0; k < K1; ++k) v = fmaf(w1r[k], xs[t + k], v);
          v = (t < L) ? fmaxf(v, 0.f) : 0.f;
          __bf16 vb = ecg::to_bf16(v);
          h1s[(t + 2) * C + c] = vb;
          mask1 |= (ecg::from_bf16(vb) > 0.f ? 1u : 0u) << (pi * 8 + half * 4 + i);
        }
      }
    }
  }
  __syncthreads();

  // ---------------- phase 2: conv2 (MFMA) + bias + ReLU, mean-pool partials ---------------------
  float pool = 0.f;
#pragma unroll
  for (int pi = 0; pi < MAX_PAIRS_PER_WAVE; ++pi) {
    const int pair = w + pi * WAVES;
    if (pair < NP) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int t0 = 32 * pair + 16 * half;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tap = 2 * s + (h >> 1);
          const int r = t0 + (lane & 15) + tap - 2;  // h1 time index
          const bf16x8 A = *reinterpret_cast<const bf16x8*>(h1s + (r + 2) * C + 8 * (h & 1));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = t0 + 4 * h + i;
          float v = fmaxf(acc[i] + b2r, 0.f);
          if (t >= L) v = 0.f;
          pool += v;
          mask2 |= (v > 0.f ? 1u : 0u) << (pi * 8 + half * 4 + i);
        }
      }
    }
  }
  pool = ecg::quarter_sum(pool);
  if (lane < 16) red[RED_POOL + w * 16 + lane] = pool;
  __syncthreads();

  // ---------------- head: pooled -> logits -> CE -> dlogits, dWh, dbh, dpooled ----------------
  if (w == 0) {
    float pooled = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) pooled += red[RED_POOL + ww * 16 + c];
    pooled *= (1.0f / (float)L);
    // Broadcast the 16 pooled channels to every lane (all lanes active: no divergent shuffles).
    float pv[C];
#pragma unroll
    for (int co = 0; co < C; ++co) pv[co] = __shfl(pooled, co, 64);
    // lane n (< nc) of each 16-lane group computes logit n
    const int n = c;
    float logit = -INFINITY;
    if (n < nc) {
      logit = params[lay.bh + n];
#pragma unroll
      for (int co = 0; co < C; ++co) logit = fmaf(params[lay.wh + n * C + co], pv[co], logit);
    }
    if (MODE == 1) {
      if (lane < nc) out[(long)b * out_stride + n] = logit;
    } else {
      float m = logit;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
      float e = (n < nc) ? __expf(logit - m) : 0.f;
      float ssum = e;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) ssum += __shfl_xor(ssum, off, 64);
      const int y = Y[row];
      const float logit_y = __shfl(logit, (lane & 48) + y, 64);
      const float loss = m + __logf(ssum) - logit_y;
      const float dlogit = (n < nc) ? (e / ssum - (n == y ? 1.f : 0.f)) * inv_B : 0.f;
      float* srow = out + (long)b * out_stride;
      if (lane < nc) {
#pragma unroll
        for (int co = 0; co < C; ++co) srow[lay.wh + n * C + co] = dlogit * pv[co];
        srow[lay.bh + n] = dlogit;
      }
      if (lane == 0) srow[lay.P] = loss;
      // dpooled[co] = sum_n dlogit[n] * Wh[n][co]; lane co (< 16)
      float dp = 0.f;
      for (int nn = 0; nn < nc; ++nn) dp = fmaf(__shfl(dlogit, nn, 64), params[lay.wh + nn * C + c], dp);
      if (lane < 16) red[RED_G + c] = dp * (1.0f / (float)L);
    }
  }
  if (MODE == 1) return;
  __syncthreads();

  // ---------------- phase 3: dh2 (= g * relu'), db2, conv2 wgrad (MFMA) ------------------------
  const float g = red[RED_G + c];
  float db2 = 0.f;
  f32x4 accW[K2];
#pragma unroll
  for (int k = 0; k < K2; ++k) accW[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int pi = 0; pi < MAX_PAIRS_PER_WAVE; ++pi) {
    const int pair = w + pi * WAVES;
    if (pair < NP) {
      bf16x8 Adh;  // A[co][t] in the permuted k-order of the forward C layout
#pragma unroll
      for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = 32 * pair + 16 * half + 4 * h + i;
          const bool on = (mask2 >> (pi * 8 + half * 4 + i)) & 1u;
          const float d = on ? g : 0.f;
          const __bf16 db = ecg::to_bf16(d);
          dh2s[(t + 4) * C + c] = db;
          db2 += d;
          Adh[half * 4 + i] = db;
        }
      }
      const int t0 = 32 * pair;
      const int q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
#pragma unroll
      for (int k = 0; k < K2; ++k) {
        const int ra = t0 + 4 * h + k - 2 + q;  // h1 time index of row q of the first 4x16 block
        const s16x4 lo = lds_tr16(h1s + (ra + 2) * C + p4);
        const s16x4 hi = lds_tr16(h1s + (ra + 16 + 2) * C + p4);
        accW[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Adh, cat44(lo, hi), accW[k], 0, 0, 0);
      }
    }
  }
  // accW[k][i] = dW2[co = 4h+i][ci = c][k]
#pragma unroll
  for (int k = 0; k < K2; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&red[RED_DW2 + (4 * h + i) * (C * K2) + c * K2 + k], accW[k][i]);
  db2 = ecg::quarter_sum(db2);
  if (lane < 16) atomicAdd(&red[RED_DB2 + c], db2);
  // conv2 dgrad B operand: B[r][ci], r = 32s + 8h + j -> tap k = r>>4, co = r&15, ci = c.
  bf16x8 Bd[3];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int r = 32 * s + 8 * h + j, k = r >> 4, co = r & 15;
      float v = k < K2 ? params[lay.w2 + co * (C * K2) + c * K2 + k] : 0.f;
      Bd[s][j] = ecg::to_bf16(v);
    }
  __syncthreads();

  // ---------------- phase 4: conv2 dgrad (MFMA) * relu'(h1), conv1 wgrad (VALU) ---------------
  float dw1[K1 + 1];
#pragma unroll
  for (int k = 0; k <= K1; ++k) dw1[k] = 0.f;
#pragma unroll
  for (int pi = 0; pi < MAX_PAIRS_PER_WAVE; ++pi) {
    const int pair = w + pi * WAVES;
    if (pair < NP) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int t0 = 32 * pair + 16 * half;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int k = 2 * s + (h >> 1);
          const int r = t0 + (lane & 15) - k + 2;  // dh2 time index
          const bf16x8 A = *reinterpret_cast<const bf16x8*>(dh2s + (r + 4) * C + 8 * (h & 1));
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bd[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int t = t0 + 4 * h + i;
          const bool on = (mask1 >> (pi * 8 + half * 4 + i)) & 1u;
          const float d = on ? acc[i] : 0.f;
          dw1[K1] += d;
#pragma unroll
          for (int k = 0; k < K1; ++k) dw1[k] = fmaf(d, xs[t + k], dw1[k]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k <= K1; ++k) {
    float v = ecg::quarter_sum(dw1[k]);
    if (lane < 16) atomicAdd(&red[RED_DW1 + c * 8 + k], v);
  }
  __syncthreads();

  // ---------------- phase 5: write this sample's gradient row ---------------------------------
  float* srow = out + (long)b * out_stride;
  for (int i = tid; i < lay.wh; i += WAVES * 64) {
    float v;
    if (i < lay.b1) {
      v = red[RED_DW1 + (i / K1) * 8 + (i % K1)];
    } else if (i < lay.w2) {
      v = red[RED_DW1 + (i - lay.b1) * 8 + K1];
    } else if (i < lay.b2) {
      v = red[RED_DW2 + (i - lay.w2)];
    } else {
      v = red[RED_DB2 + (i - lay.b2)];
    }
    srow[i] = v;
  }
}

// Sum the per-sample gradient rows and apply SGD (+momentum, weight decay, nesterov) in place.
// grid = ceil((P+1)/64) blocks of 256 threads; column P of the slab carries the per-sample loss.
__global__ __launch_bounds__(256) void slab_reduce_sgd_kernel(
    const float* __restrict__ slab, int G, int stride, int P,
    float* __restrict__ params, float* __restrict__ mom, float* __restrict__ grad_out,
    float* __restrict__ loss_acc, float lr, float momentum, float wd, int nesterov, int apply) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col <= P) {
    int r = w;
    for (; r + 12 < G; r += 16) {
      float a0 = slab[(long)r * stride + col];
      float a1 = slab[(long)(r + 4) * stride + col];
      float a2 = slab[(long)(r + 8) * stride + col];
      float a3 = slab[(long)(r + 12) * stride + col];
      s += (a0 + a1) + (a2 + a3);
    }
    for (; r < G; r += 4) s += slab[(long)r * stride + col];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && col <= P) {
    float gsum = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (col == P) {
      if (loss_acc) loss_acc[0] += gsum;
    } else {
      if (grad_out) grad_out[col] = gsum;
      if (apply) {
        float p = params[col];
        float d = gsum + wd * p;
        if (momentum != 0.f) {
          float bm = momentum * mom[col] + d;
          mom[col] = bm;
          d = nesterov ? d + momentum * bm : bm;
        }
        params[col] = p - lr * d;
      }
    }
  }
}

template <int WAVES, int MODE>
int launch_step(const float* X, int L, long ldx, const int* idx, const int* Y, const float* params, int nc,
                float* out, int out_stride, int B, float inv_B, hipStream_t stream) {
  const Smem sm = make_smem(L, WAVES);
  auto kern = tiny_ecg_step_kernel<WAVES, MODE>;
  if (sm.bytes > 64 * 1024)
    ECG_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, sm.bytes));
  hipLaunchKernelGGL(kern, dim3(B), dim3(WAVES * 64), sm.bytes, stream, X, L, ldx, idx, Y, params, nc, out,
                     out_stride, inv_B);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

int pick_waves(int L) {
  const int Lp = (L + 31) / 32 * 32;
  return Lp <= 32 * 4 * 8 ? 8 : 16;  // 4 tile pairs per wave max
}

int check_step_args(int L, int nc, int B, int out_stride, int mode) {
  if (L < 8 || B <= 0 || nc < 1 || nc > MAX_CLASSES) return ecg::kBadArg;
  const int Lp = (L + 31) / 32 * 32;
  if (Lp > 32 * 4 * 16) return ecg::kTooLarge;  // > 2048 samples per window: use the op-by-op path
  if (make_smem(L, 16).bytes > 160 * 1024) return ecg::kTooLarge;
  const Layout lay = make_layout(nc);
  if (mode == 0 && out_stride < lay.P + 1) return ecg::kBadArg;
  if (mode == 1 && out_stride < nc) return ecg::kBadArg;
  return ecg::kOk;
}

int step_dispatch(int mode, const float* X, int L, long ldx, const int* idx, const int* Y, const float* params,
                  int nc, float* out, int out_stride, int B, float inv_B, hipStream_t stream) {
  int st = check_step_args(L, nc, B, out_stride, mode);
  if (st) return st;
  const int waves = pick_waves(L);
  if (mode == 0)
    return waves == 8 ? launch_step<8, 0>(X, L, ldx, idx, Y, params, nc, out, out_stride, B, inv_B, stream)
                      : launch_step<16, 0>(X, L, ldx, idx, Y, params, nc, out, out_stride, B, inv_B, stream);
  return waves == 8 ? launch_step<8, 1>(X, L, ldx, idx, Y, params, nc, out, out_stride, B, inv_B, stream)
                    : launch_step<16, 1>(X, L, ldx, idx, Y, params, nc, out, out_stride, B, inv_B, stream);
}

int reduce_dispatch(const float* slab, int G, int stride, int P, float* params, float* mom, float* grad_out,
                    float* loss_acc, float lr, float momentum, float wd, int nesterov, int apply,
                    hipStream_t stream) {
  if (G <= 0 || P <= 0 || stride < P + 1) return ecg::kBadArg;
  if (apply && (!params || (momentum != 0.f && !mom))) return ecg::kBadArg;
  const int blocks = (P + 1 + 63) / 64;
  hipLaunchKernelGGL(slab_reduce_sgd_kernel, dim3(blocks), dim3(256), 0, stream, slab, G, stride, P, params, mom,
                     grad_out, loss_acc, lr, momentum, wd, nesterov, apply);
  ECG_HIP_CHECK(hipGetLastError());
  return ecg::kOk;
}

struct RoundGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int steps = 0;
};

}  // namespace

// ---------------------------------------------------------------------------- C ABI
ECG_API int ecg_tiny_param_count(int nc) { return make_layout(nc).P; }

ECG_API int ecg_tiny_smem_bytes(int L) { return make_smem(L, pick_waves(L)).bytes; }

// One fused training step's gradient pass: writes slab[B][slab_stride] (grads + loss at column P).
ECG_API int ecg_tiny_step_grads(const float* X, int L, long ldx, const int* idx, const int* Y,
                                const float* params, int nc, float* slab, int slab_stride, int B, float inv_B,
                                hipStream_t stream) {
  return step_dispatch(0, X, L, ldx, idx, Y, params, nc, slab, slab_stride, B, inv_B, stream);
}

// Inference: logits[B][nc] for windows X[idx[b]].
ECG_API int ecg_tiny_forward(const float* X, int L, long ldx, const int* idx, const float* params, int nc,
                             float* logits, int B, hipStream_t stream) {
  return step_dispatch(1, X, L, ldx, idx, nullptr, params, nc, logits, nc, B, 0.f, stream);
}

ECG_API int ecg_slab_reduce_sgd(const float* slab, int G, int stride, int P, float* params, float* mom,
                                float* grad_out, float* loss_acc, float lr, float momentum, float wd, int nesterov,
                                int apply, hipStream_t stream) {
  return reduce_dispatch(slab, G, stride, P, params, mom, grad_out, loss_acc, lr, momentum, wd, nesterov, apply,
                         stream);
}

// Full step = grads + reduce/SGD (two launches on ``stream``).
ECG_API int ecg_tiny_train_step(const float* X, int L, long ldx, const int* idx, const int* Y, float* params,
                                float* mom, int nc, float* slab, int slab_stride, int B, float* loss_acc, float lr,
                                float momentum, float wd, int nesterov, hipStream_t stream) {
  int st = step_dispatch(0, X, L, ldx, idx, Y, params, nc, slab, slab_stride, B, 1.0f / (float)B, stream);
  if (st) return st;
  return reduce_dispatch(slab, B, slab_stride, make_layout(nc).P, params, mom, nullptr, loss_acc, lr, momentum, wd,
                         nesterov, 1, stream);
}

// Capture ``steps`` consecutive fused steps (batch s reads idx_table + s*B) into one hipGraph.
// All pointers are baked into the graph: callers keep the buffers alive and refill idx_table in place.
ECG_API int ecg_round_graph_create(void** handle, const float* X, int L, long ldx, const int* idx_table,
                                   const int* Y, float* params, float* mom, int nc, float* slab, int slab_stride,
                                   int B, int steps, float* loss_acc, float lr, float momentum, float wd,
                                   int nesterov) {
  if (!handle || steps <= 0) return ecg::kBadArg;
  int st = check_step_args(L, nc, B, slab_stride, 0);
  if (st) return st;
  hipStream_t cap;
  ECG_HIP_CHECK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  RoundGraph* rg = new RoundGraph();
  rg->steps = steps;
  hipError_t e = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    delete rg;
    (void)hipStreamDestroy(cap);
    return ecg::kHipError;
  }
  for (int s = 0; s < steps && st == 0; ++s)
    st = ecg_tiny_train_step(X, L, ldx, idx_table + (long)s * B, Y, params, mom, nc, slab, slab_stride, B, loss_acc,
                             lr, momentum, wd, nesterov, cap);
  e = hipStreamEndCapture(cap, &rg->graph);
  (void)hipStreamDestroy(cap);
  if (st != 0 || e != hipSuccess) {
    if (rg->graph) (void)hipGraphDestroy(rg->graph);
    delete rg;
    return st ? st : ecg::kHipError;
  }
  e = hipGraphInstantiate(&rg->exec, rg->graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(rg->graph);
    delete rg;
    return ecg::kHipError;
  }
  *handle = rg;
  return ecg::kOk;
}

ECG_API int ecg_round_graph_launch(void* handle, hipStream_t stream) {
  if (!handle) return ecg::kBadArg;
  RoundGraph* rg = static_cast<RoundGraph*>(handle);
  ECG_HIP_CHECK(hipGraphLaunch(rg->exec, stream));
  return ecg::kOk;
}

ECG_API int ecg_round_graph_destroy(void* handle) {
  if (!handle) return ecg::kOk;
  RoundGraph* rg = static_cast<RoundGraph*>(handle);
  if (rg->exec) (void)hipGraphExecDestroy(rg->exec);
  if (rg->graph) (void)hipGraphDestroy(rg->graph);
  delete rg;
  return ecg::kOk;
}
