// SpeechEmbedder LSTM stack on gfx950: fp32 MFMA GEMMs + per-timestep recurrent
// kernels with the gate nonlinearities and cell update fused into the epilogue.
//
// Replaces the reference's nn.LSTM forward (speech_embedder_net.py:19,28) and its
// autograd backward (train_speech_embedder.py:62), SURVEY §8 rows a-B and a-H.
//
// HBM layout (time-major, so every timestep slice is one contiguous [B, *] block):
//   x_tm   [T, B, F]      layer input
//   gates  [T, B, 4H]     in: x W_ih^T + b_ih + b_hh (K1); out: activated i,f,g,o (K2)
//   c_tm   [T, B, H]      cell state c_t
//   h_tm   [T+1, B, H]    h_tm[0] = h_{-1} = 0, h_tm[t+1] = h_t
//   dgates [T, B, 4H]     dL/d(pre-activation gates)
#include <stdlib.h>
#include <algorithm>
#include <atomic>
#include <type_traits>
#include "sv_common.h"
#include "sv_gemm.h"
#include "sv_gemm_f32_256.h"
#include "../../include/sv_ge2e.h"


#define SV_BKM 32

// ============================================================================
// generic fp32 GEMM  C[M,N] = op(A) op(B) (+ bias) (+ beta C), or split-K slabs
// ============================================================================
enum { EPI_STORE = 0, EPI_SLAB = 1 };

template <int BM, int BN, bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, long lda,
                                                       const float* __restrict__ B, long ldb, float* __restrict__ C,
                                                       long ldc, long slab, int M, int N, int K, int kchunk,
                                                       const float* __restrict__ bias0,
                                                       const float* __restrict__ bias1, float beta) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int TM = BM / 64, TN = BN / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // column tile fastest: the blocks an XCD runs together share one A row-panel (the large
  // operand, read from HBM once) and sweep the small B operand, which stays cache-resident
  const int tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_n * ((M + BM - 1) / BM);
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int kbeg = blockIdx.y * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int wm0 = (w >> 1) * (BM / 2), wn0 = (w & 1) * (BN / 2);
  f32x16 acc[TM][TN];
  zero_acc(acc);
  gemm_mainloop<BM, BN, 256, AK, BKC, TM, TN>(A, lda, RowMapLinear{tm * BM, M}, B, ldb, RowMapLinear{tn * BN, N},
                                              kbeg, kend, lds, tid, wm0, wn0, acc);
  float* Cz = C + (EPI == EPI_SLAB ? (long)blockIdx.y * slab : 0);
  // bias sums of the lane's columns, loaded before any store (a load between stores waits for
  // every store issued before it)
  float bsum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = tn * BN + wn0 + 32 * j + (lane & 31);
    float badd = 0.f;
    if (EPI == EPI_STORE && col < N) {
      if (bias0) badd += bias0[col];
      if (bias1) badd += bias1[col];
    }
    bsum[j] = badd;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = tn * BN + wn0 + 32 * j + (lane & 31);
      if (col >= N) continue;
      const float badd = bsum[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tm * BM + wm0 + 32 * i + acc_row(r, lane);
        if (row >= M) continue;
        float v = acc[i][j][r];
        float* dst = Cz + (long)row * ldc + col;
        if (EPI == EPI_STORE) {
          v += badd;
          if (beta != 0.f) v += beta * *dst;
        }
        *dst = v;
      }
    }
}

// out[M,N] (ld ldc) = sum_z slab[z][M,N] (+ beta*out), fixed summation order
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int nz, long zstride, float* __restrict__ out,
                                   long ldc, int M, int N, float beta, const float* __restrict__ bias0,
                                   const float* __restrict__ bias1) {
  const long total = (long)M * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = (int)(e / N), col = (int)(e % N);
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += slab[z * zstride + e];
    if (bias0) s += bias0[col];
    if (bias1) s += bias1[col];
    float* dst = out + (long)row * ldc + col;
    *dst = (beta != 0.f ? beta * *dst : 0.f) + s;
  }
}

// column sums of X[R, C] (row-major): partial[chunk][C] over row chunks
__global__ void colsum_partial_kernel(const float* __restrict__ X, int R, int C, int rows_per_chunk,
                                      float* __restrict__ partial) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = blockIdx.y;
  if (col >= C) return;
  const int r0 = chunk * rows_per_chunk, r1 = min(R, r0 + rows_per_chunk);
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += X[(long)r * C + col];
  partial[(long)chunk * C + col] = s;
}
__global__ void colsum_final_kernel(const float* __restrict__ partial, int nchunk, int C, float* __restrict__ out0,
                                    float* __restrict__ out1) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= C) return;
  float s = 0.f;
  for (int k = 0; k < nchunk; ++k) s += partial[(long)k * C + col];
  out0[col] = s;
  if (out1) out1[col] = s;
}

// [B, T, F] (batch_first) -> [T, B, F]
__global__ void to_time_major_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int T, int F4) {
  const long total = (long)B * T * F4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int f = (int)(e % F4);
    const long bt = e / F4;
    const int t = (int)(bt % T), b = (int)(bt / T);
    reinterpret_cast<f32x4*>(y)[((long)t * B + b) * F4 + f] = reinterpret_cast<const f32x4*>(x)[e];
  }
}

// k-major ("NT") GEMM: both operands k-contiguous; the fast path for every large GEMM.
// X6 / X3: the bf16x6 / bf16x3 product forms of the `products` argument (sv_lstm_stack_fwd).
template <int BM, int BN, int EPI, int D = 1, bool X6 = false, bool X3 = false>
__global__ __launch_bounds__(256) void gemm_km_kernel(const float* __restrict__ A, long lda, const float* __restrict__ B,
                                                      long ldb, float* __restrict__ C, long ldc, long slab, int M,
                                                      int N, int K, int kchunk, const float* __restrict__ bias0,
                                                      const float* __restrict__ bias1, float beta) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int BLK = 32;                                // MFMA output block edge
  constexpr int TM = BM / 2 / BLK, TN = BN / 2 / BLK;    // blocks per wave (2x2 waves)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // column tile fastest: the blocks an XCD runs together share one A row-panel (the large
  // operand, read from HBM once) and sweep the small B operand, which stays cache-resident
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int kbeg = blockIdx.y * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int wm0 = (w >> 1) * (BM / 2), wn0 = (w & 1) * (BN / 2);
  f32x16 acc[TM][TN];
  zero_acc(acc);
  if constexpr (X3)
    gemm_mainloop_x3<BM, BN, 256, 16, 2, TM, TN>(A, lda, RowMapLinear{tm * BM, M}, B, ldb, RowMapLinear{tn * BN, N},
                                                 kbeg, kend, lds, tid, wm0, wn0, acc);
  else
    gemm_mainloop_km_d<BM, BN, 256, SV_BKM, D, TM, TN, false, X6>(A, lda, RowMapLinear{tm * BM, M}, B, ldb,
                                                                RowMapLinear{tn * BN, N}, kbeg, kend, lds, tid, wm0,
                                                                wn0, acc);
  float* Cz = C + (EPI == EPI_SLAB ? (long)blockIdx.y * slab : 0);
  // bias sums of the lane's columns, loaded before any store (a load between stores waits for
  // every store issued before it)
  float bsum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = tn * BN + wn0 + BLK * j + (lane & (BLK - 1));
    float badd = 0.f;
    if (EPI == EPI_STORE && col < N) {
      if (bias0) badd += bias0[col];
      if (bias1) badd += bias1[col];
    }
    bsum[j] = badd;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = tn * BN + wn0 + BLK * j + (lane & (BLK - 1));
      if (col >= N) continue;
      const float badd = bsum[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tm * BM + wm0 + BLK * i + acc_row(r, lane);
        if (row >= M) continue;
        float v = acc[i][j][r];
        float* dst = Cz + (long)row * ldc + col;
        if (EPI == EPI_STORE) {
          v += badd;
          if (beta != 0.f) v += beta * *dst;
        }
        *dst = v;
      }
    }
}

// row sums out[r] = sum_c X[r*ld + c], one block of RS_T threads per row, fixed order.
// 512-thread blocks: 4 per CU resident, so the 4H = 3072 rows of c2 run as 3 full rounds of
// 1024 blocks (256-thread blocks left a half-empty second round: 3072 / 2048)
#define RS_T 512
__global__ __launch_bounds__(RS_T) void rowsum_kernel(const float* __restrict__ X, long ld, int C,
                                                      float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float red[RS_T / 64];
  const float* x = X + (long)blockIdx.x * ld;
  // four independent 16-B loads in flight per thread per trip (a row is 400 KB at c2), summed
  // in a fixed order
  const int C4 = C / 4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int c = threadIdx.x;
  for (; c + 3 * RS_T < C4; c += 4 * RS_T) {
    const f32x4 v0 = x4[c], v1 = x4[c + RS_T], v2 = x4[c + 2 * RS_T], v3 = x4[c + 3 * RS_T];
    s0 += (v0.x + v0.y) + (v0.z + v0.w);
    s1 += (v1.x + v1.y) + (v1.z + v1.w);
    s2 += (v2.x + v2.y) + (v2.z + v2.w);
    s3 += (v3.x + v3.y) + (v3.z + v3.w);
  }
  for (; c < C4; c += RS_T) {
    const f32x4 v = x4[c];
    s0 += (v.x + v.y) + (v.z + v.w);
  }
  float s = (s0 + s1) + (s2 + s3);
  for (int c1 = C4 * 4 + threadIdx.x; c1 < C; c1 += RS_T) s += x[c1];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < RS_T / 64; ++i) t += red[i];
    out0[blockIdx.x] = t;
    if (out1) out1[blockIdx.x] = t;
  }
}

// dst[c*ldd + r] = src[r*lds + c]  (R x C), 32x32 tiles through LDS
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ src, long lds_, int R, int C,
                                                        float* __restrict__ dst, long ldd) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? src[(long)r * lds_ + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) dst[(long)c * ldd + r] = tile[tx][i];
  }
}

// ============================================================================
// K2: forward recurrent step.  Block = 64 batch rows x 32 hidden units (= 128 gate
// columns: i,f,g,o of those units), 4 waves in 2x2; K = H, k-major LDS tiles.
// Epilogue: + x-projection, sigmoid/tanh, c_t = f c_{t-1} + i g, h_t = o tanh(c_t);
// stores the activated gates (for BPTT), c_t, h_t and h_t^T (column block t+1 of
// hT[H, (T+1) B], the k-contiguous operand of the weight-gradient GEMMs).
// ============================================================================
#define FWD_BM 64
#define FWD_U 32

// ============================================================================
// K3: backward recurrent step at time t.  Block = 64 batch rows x 32 hidden units;
// wave w computes dG_{t+1}[:, gate w] . W_hh[gate w rows, units] (K = H each, an
// in-block split of K = 4H by gate) from W_hh^T [H, 4H] (k-contiguous), partials summed
// in LDS in fixed order.  Epilogue: dh = that + dh_up; dc = dc_{t+1} f_{t+1} + dh o
// (1 - tanh^2 c); dG_t = [dc g i(1-i), dc c_{t-1} f(1-f), dc i (1-g^2), dh tanh(c) o(1-o)],
// stored as dG[t] [B, 4H] and as column block t of dG^T [4H, T B].
// ============================================================================
#define BWD_BM 64
#define BWD_U 32
#define X3_GBUF_BYTES (12 * (BWD_BM + BWD_U) * (16 + 8))  // one gate group's X3 double buffer

// ============================================================================
// 8-wave variants of K2/K3 (512 threads, 2 waves per SIMD so one wave's MFMAs cover the
// other's LDS/global waits).
//   K2v2: the 64 x 128 gate tile is split 2 (rows) x 4 (gate) over 8 waves, one 32x32
//         accumulator each, all sharing the same staged A/B tiles.
//   K3v2: 4 groups of 2 waves, group = gate (its K range of W_hh^T), waves split the rows.
// ============================================================================
template <int BKX, int D = 1, bool X6 = false, bool X3 = false>
__global__ __launch_bounds__(512) void lstm_step_fwd_v2_kernel(const float* __restrict__ hprev,
                                                               const float* __restrict__ whh,
                                                               float* __restrict__ gates,
                                                               const float* __restrict__ cprev,
                                                               float* __restrict__ cout, float* __restrict__ hout,
                                                               float* __restrict__ hT, long ldhT, int t, int Bp, int B,
                                                               int H) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int BN = 4 * FWD_U, LDP = BN + 4, LDH = FWD_BM + 1;
  constexpr int PER = FWD_BM * FWD_U / 512;  // epilogue elements per thread
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * FWD_U, b0 = blockIdx.y * FWD_BM;
  const int wm0 = (w >> 2) * 32, wn0 = (w & 3) * 32;
  const long G = 4L * H;
  // the epilogue's inputs do not depend on the GEMM: issue their loads first
  float xg[PER][4], cpv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / FWD_U, u = e % FWD_U;
    const int gb = b0 + b, gj = j0 + u;
    const bool ok = gb < B && gj < H;
    const float* gp = gates + (long)gb * G + gj;
#pragma unroll
    for (int q = 0; q < 4; ++q) xg[k][q] = ok ? gp[q * H] : 0.f;
    cpv[k] = (ok && cprev) ? cprev[(long)gb * H + gj] : 0.f;
  }
  f32x16 acc[1][1];
  zero_acc(acc);
  if (hprev) {
    if constexpr (X3)
      gemm_mainloop_x3<FWD_BM, BN, 512, 32, 2, 1, 1>(hprev + (long)b0 * H, H, RowMapLinear{0, B - b0}, whh, H,
                                                     RowMapGates<FWD_U>{j0, H}, 0, H, lds, tid, wm0, wn0, acc);
    else
      gemm_mainloop_km_d<FWD_BM, BN, 512, BKX, D, 1, 1, false, X6>(hprev + (long)b0 * H, H, RowMapLinear{0, B - b0},
                                                                  whh, H, RowMapGates<FWD_U>{j0, H}, 0, H, lds, tid,
                                                                  wm0, wn0, acc);
  }
  float* pre = lds;
  float* hs = lds + FWD_BM * LDP;
#pragma unroll
  for (int r = 0; r < 16; ++r) pre[(wm0 + acc_row(r, lane)) * LDP + wn0 + (lane & 31)] = acc[0][0][r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / FWD_U, u = e % FWD_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    float* gp = gates + (long)gb * G + gj;
    const float* pr = pre + b * LDP + u;
    const float i = sv_sigmoid(pr[0] + xg[k][0]);
    const float f = sv_sigmoid(pr[FWD_U] + xg[k][1]);
    const float g = sv_tanh(pr[2 * FWD_U] + xg[k][2]);
    const float o = sv_sigmoid(pr[3 * FWD_U] + xg[k][3]);
    const float c = f * cpv[k] + i * g;
    const float h = o * sv_tanh(c);
    gp[0] = i;
    gp[H] = f;
    gp[2 * H] = g;
    gp[3 * H] = o;
    cout[(long)gb * H + gj] = c;
    hout[(long)gb * H + gj] = h;
    hs[u * LDH + b] = h;
  }
  if (!hT) return;
  __syncthreads();
  for (int e = tid; e < FWD_BM * FWD_U; e += 512) {
    const int u = e / FWD_BM, b = e % FWD_BM;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    float* row = hT + (long)gj * ldhT;
    row[(long)(t + 1) * Bp + gb] = hs[u * LDH + b];
    if (t == 0) row[gb] = 0.f;
  }
}

template <int BKX, int D = 1, bool X6 = false, bool X3 = false>
__global__ __launch_bounds__(512) void lstm_step_bwd_v2_kernel(
    const float* __restrict__ dgnext, const float* __restrict__ whhT, const float* __restrict__ dhup,
    const float* __restrict__ dcf_next, const float* __restrict__ acts, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, float* __restrict__ dg, float* __restrict__ dcf, float* __restrict__ dgT,
    long lddgT, int t, int Bp, int B, int H, unsigned long long* __restrict__ ts = nullptr) {
  // ts (timing sample, bench only): [start, end] of this launch on the 100 MHz real-time clock,
  // first workgroup start (min) and last workgroup end (max), vector atomics
  if (ts && threadIdx.x == 0) atomicMin(ts, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int GBUF = 2 * (BWD_BM + BWD_U) * (BKX + 4);
  constexpr int LDR = BWD_U + 1;
  constexpr int LDT = BWD_BM + 1;
  constexpr int PER = BWD_BM * BWD_U / 512;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int gate = w >> 1, gt = tid & 127;
  const int j0 = blockIdx.x * BWD_U, b0 = blockIdx.y * BWD_BM;
  const long G = 4L * H;
  // prefetch the epilogue's element-wise inputs (independent of the GEMM)
  float av[PER][4], cv[PER], cpv[PER], dcfv[PER], upv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BWD_U, u = e % BWD_U;
    const int gb = b0 + b, gj = j0 + u;
    const bool ok = gb < B && gj < H;
    const long hi = (long)gb * H + gj;
    const float* ap = acts + (long)gb * G + gj;
#pragma unroll
    for (int q = 0; q < 4; ++q) av[k][q] = ok ? ap[q * H] : 0.f;
    cv[k] = ok ? c_t[hi] : 0.f;
    cpv[k] = (ok && c_prev) ? c_prev[hi] : 0.f;
    dcfv[k] = (ok && dcf_next) ? dcf_next[hi] : 0.f;
    upv[k] = (ok && dhup) ? dhup[hi] : 0.f;
  }
  f32x16 acc[1][1];
  zero_acc(acc);
  if (dgnext) {
    if constexpr (X3)
      gemm_mainloop_x3<BWD_BM, BWD_U, 128, 16, 2, 1, 1>(dgnext + (long)b0 * G, G, RowMapLinear{0, B - b0}, whhT, G,
                                                        RowMapLinear{j0, H}, gate * H, (gate + 1) * H,
                                                        reinterpret_cast<char*>(lds) + gate * X3_GBUF_BYTES, gt,
                                                        (w & 1) * 32, 0, acc);
    else
      gemm_mainloop_km_d<BWD_BM, BWD_U, 128, BKX, D, 1, 1, false, X6>(
          dgnext + (long)b0 * G, G, RowMapLinear{0, B - b0}, whhT, G, RowMapLinear{j0, H}, gate * H, (gate + 1) * H,
          lds + gate * GBUF, gt, (w & 1) * 32, 0, acc);
  }
  __syncthreads();
  float* red = lds;                    // [4][64][LDR]
  float* gT = lds + 4 * BWD_BM * LDR;  // [4*32][LDT]
#pragma unroll
  for (int r = 0; r < 16; ++r)
    red[(gate * BWD_BM + (w & 1) * 32 + acc_row(r, lane)) * LDR + (lane & 31)] = acc[0][0][r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BWD_U, u = e % BWD_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    const long hi = (long)gb * H + gj;
    float dh = red[(0 * BWD_BM + b) * LDR + u];
    dh += red[(1 * BWD_BM + b) * LDR + u];
    dh += red[(2 * BWD_BM + b) * LDR + u];
    dh += red[(3 * BWD_BM + b) * LDR + u];
    dh += upv[k];
    const float i = av[k][0], f = av[k][1], g = av[k][2], o = av[k][3];
    const float tc = sv_tanh(cv[k]);
    const float dc = dh * o * (1.f - tc * tc) + dcfv[k];
    const float d0 = dc * g * i * (1.f - i), d1 = dc * cpv[k] * f * (1.f - f);
    const float d2 = dc * i * (1.f - g * g), d3 = dh * tc * o * (1.f - o);
    float* dp = dg + (long)gb * G + gj;
    dp[0] = d0;
    dp[H] = d1;
    dp[2 * H] = d2;
    dp[3 * H] = d3;
    dcf[hi] = dc * f;
    gT[(0 * BWD_U + u) * LDT + b] = d0;
    gT[(1 * BWD_U + u) * LDT + b] = d1;
    gT[(2 * BWD_U + u) * LDT + b] = d2;
    gT[(3 * BWD_U + u) * LDT + b] = d3;
  }
  if (dgT) {
    __syncthreads();
    for (int e = tid; e < 4 * BWD_U * BWD_BM; e += 512) {
      const int gu = e / BWD_BM, b = e % BWD_BM;
      const int gte = gu / BWD_U, u = gu % BWD_U;
      const int gb = b0 + b, gj = j0 + u;
      if (gb >= B || gj >= H) continue;
      dgT[((long)gte * H + gj) * lddgT + (long)t * Bp + gb] = gT[gu * LDT + b];
    }
  }
  if (ts) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(ts + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

// ============================================================================
// host side
// ============================================================================
namespace {

// fp32 product mode of the calling thread's current entry point (the `products` argument of
// sv_gemm_f32 / sv_lstm_stack_fwd / sv_lstm_stack_bwd, set for the duration of that call by
// F32ProductScope; every other entry point runs exact):
//   0  exact fp32 MFMA (v_mfma_f32_32x32x2_f32) everywhere -- the default
//   1  bf16x6 split where it measured faster: NT GEMMs split in registers (x6), K2 split at the
//      LDS store (x3), K3 exact
//   2  x3 everywhere, 3  x6 everywhere (diagnostics)
thread_local int t_f32_mode = 0;
int gemm_x() {  // 0 exact, 1 x6, 2 x3
  const int m = t_f32_mode;
  return m == 1 || m == 3 ? 1 : m == 2 ? 2 : 0;
}
int k2_x() {
  const int m = t_f32_mode;
  return m == 1 || m == 2 ? 2 : m == 3 ? 1 : 0;
}
int k3_x() {
  const int m = t_f32_mode;
  return m == 2 ? 2 : m == 3 ? 1 : 0;
}

template <int BM, int BN, bool AK, bool BKC, int EPI>
int launch_gemm_t(const float* A, long lda, const float* B, long ldb, float* C, long ldc, long slab, int M, int N,
                  int K, int splitk, int kchunk, const float* b0, const float* b1, float beta, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (AK && BKC) {
    // KTileStage's buffer loads address a tile's rows with 32-bit byte offsets
    if ((long)BM * lda * 4 >= (1L << 31) || (long)BN * ldb * 4 >= (1L << 31)) return SV_ESHAPE;
    constexpr int LDS_KM = 2 * (BM + BN) * (SV_BKM + 4);
    if (gemm_x() == 2)
      hipLaunchKernelGGL((gemm_km_kernel<BM, BN, EPI, 1, false, true>), dim3(tiles, splitk), dim3(256),
                         12 * (BM + BN) * (16 + 8), s, A, lda, B, ldb, C, ldc, slab, M, N, K, kchunk, b0, b1, beta);
    else if (gemm_x() == 1)
      hipLaunchKernelGGL((gemm_km_kernel<BM, BN, EPI, 1, true>), dim3(tiles, splitk), dim3(256), LDS_KM * sizeof(float),
                         s, A, lda, B, ldb, C, ldc, slab, M, N, K, kchunk, b0, b1, beta);
    else
      hipLaunchKernelGGL((gemm_km_kernel<BM, BN, EPI>), dim3(tiles, splitk), dim3(256), LDS_KM * sizeof(float), s, A,
                         lda, B, ldb, C, ldc, slab, M, N, K, kchunk, b0, b1, beta);
  } else {
    constexpr int LDS_FLOATS = 2 * SV_BK * (TileLd<AK, BM>::value + TileLd<BKC, BN>::value);
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AK, BKC, EPI>), dim3(tiles, splitk), dim3(256),
                       LDS_FLOATS * sizeof(float), s, A, lda, B, ldb, C, ldc, slab, M, N, K, kchunk, b0, b1, beta);
  }
  SV_LAUNCH_CHECK();
  return SV_OK;
}

template <int BM, int BN, int EPI>
int dispatch_layout(bool ak, bool bk, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                    long slab, int M, int N, int K, int splitk, int kchunk, const float* b0, const float* b1,
                    float beta, hipStream_t s) {
  if (ak && bk) return launch_gemm_t<BM, BN, true, true, EPI>(A, lda, B, ldb, C, ldc, slab, M, N, K, splitk, kchunk, b0, b1, beta, s);
  if (ak && !bk) return launch_gemm_t<BM, BN, true, false, EPI>(A, lda, B, ldb, C, ldc, slab, M, N, K, splitk, kchunk, b0, b1, beta, s);
  if (!ak && bk) return launch_gemm_t<BM, BN, false, true, EPI>(A, lda, B, ldb, C, ldc, slab, M, N, K, splitk, kchunk, b0, b1, beta, s);
  return launch_gemm_t<BM, BN, false, false, EPI>(A, lda, B, ldb, C, ldc, slab, M, N, K, splitk, kchunk, b0, b1, beta, s);
}

struct GemmPlan {
  int bm, bn, splitk, kchunk;
};

// Tile 128x128 when there are enough tiles to fill the chip, else 64x64.  When the tiles leave
// resident slots (2 blocks/CU x 256 CUs, 4 for 64x64) idle, split K: the split count minimises
// a wave-quantised time model, rounds(tiles*sk / slots) x (time of one K/sk chunk) + the slab
// traffic of the split (sk x M x N x 4 B written and read back), over sk <= 32 with K chunks of
// at least 512.  At the dW shape (144 tiles, K = 102400) this picks 32 splits = 9 full rounds of
// 512 blocks (the old 512/144 = 3 left 80 CUs with one block and the rest with two).
GemmPlan plan_gemm(int M, int N, int K, bool fine = false) {
  GemmPlan p;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  const bool small = t128 < 128;
  p.bm = small ? 64 : 128;
  p.bn = small ? 64 : 128;
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const long slots = small ? 1024 : 512;
  int sk = 1;
  if (tiles < slots) {
    // per-block rate at ~120 TF/s shared by all resident blocks; HBM ~5 TB/s for the slabs
    const double rate = 120e12 / (double)slots, hbm = 5e12;
    // K chunks of at least 512, or with `fine` 128 when the tiles alone would leave most of the
    // chip idle (the projection GEMMs: 8-48 tiles of 64 x 64 over K = 256-768 ran 12-24 us on 8-48
    // CUs)
    const int kmax = std::max(1, std::min(32, K / (fine && tiles * 8 < slots ? 128 : 512)));
    double best = 1e30;
    for (int c = 1; c <= kmax; ++c) {
      const long rounds = (tiles * c + slots - 1) / slots;
      const double kc = (double)K / c;
      const double t = rounds * (2.0 * p.bm * p.bn * kc / rate) + (c > 1 ? 2.0 * c * M * N * 4.0 / hbm + 5e-6 : 0.0);
      if (t < best * 0.999) {
        best = t;
        sk = c;
      }
    }
  }
  const int q = SV_BKM;
  p.kchunk = ((K + sk - 1) / sk + q - 1) / q * q;
  p.splitk = (K + p.kchunk - 1) / p.kchunk;
  return p;
}

// ---- narrow NT GEMM (N <= 48): layer 0's dW_ih = dG^T x (M = 4H, N = F = 40, K = T B) ----
// The 64 x 64 tiles (4 waves of v_mfma_f32_32x32x2_f32) padded N = 40 to 64 and ran this shape at
// 75 TF/s (334 us at c2); it streams dG^T (1.26 GB at c2) once.  Here a workgroup is 128 rows x 48
// columns (3 blocks of 16) over a K chunk: v_mfma_f32_16x16x4_f32, exact fp32 products, each wave
// 32 rows (2 x 3 accumulators).  A lane reads 4 consecutive k of its row (one 16-B LDS read) and
// spends them over 4 MFMAs (MFMA j takes k = 4 q + j of lane group q, for A and B alike, so the 4
// MFMAs cover 16 k); LDS images are [rows][32 k] with 16-B chunk c of row r at c ^ (r & 7), filled
// by LDS-DMA (two stages of 32 k).  Split-K slabs, reduced by slab_reduce_kernel.
constexpr int GN_BM = 128, GN_BN = 48, GN_BK = 32;
__global__ __launch_bounds__(256) void gemm_f32_narrow_kernel(const float* __restrict__ A, long lda,
                                                              const float* __restrict__ B, long ldb,
                                                              float* __restrict__ slab, long slab_stride, int M, int N,
                                                              int K, int kchunk) {
  __shared__ __attribute__((aligned(16))) float lds[2][(GN_BM + GN_BN) * GN_BK];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int m0 = blockIdx.x * GN_BM, s = blockIdx.y;
  const int kbeg = s * kchunk, nk = (min(K, kbeg + kchunk) - kbeg) / GN_BK;
  // DMA map: chunk q (16 B) of the stage: A rows 0..127 (q < 1024), then B rows 0..47
  auto fill = [&](int kt, int st) {
    const int k0 = kbeg + kt * GN_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, pc = q & 7, c = pc ^ (row & 7);
      __builtin_amdgcn_global_load_lds((gf_glb_ptr_t)(A + (long)(m0 + row) * lda + k0 + 4 * c),
                                       (gf_lds_ptr_t)(&lds[st][0] + 4 * (w * 64 + 256 * i)), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && w >= 2) break;  // 384 chunks of B: waves 0-1 issue a second one (wave-uniform)
      const int q = tid + 256 * i, row = q >> 3, pc = q & 7, c = pc ^ (row & 7);
      const int n = min(row, N - 1);  // padding columns read row N - 1 (their sums are not stored)
      __builtin_amdgcn_global_load_lds((gf_glb_ptr_t)(B + (long)n * ldb + k0 + 4 * c),
                                       (gf_lds_ptr_t)(&lds[st][GN_BM * GN_BK] + 4 * (w * 64 + 256 * i)), 16, 0, 0);
    }
  };
  f32x4 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) fill(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st landed for every wave; stage st ^ 1 free
    if (kt + 1 < nk) fill(kt + 1, st ^ 1);
    const float* As = &lds[st][0];
    const float* Bs = &lds[st][GN_BM * GN_BK];
#pragma unroll
    for (int ks = 0; ks < GN_BK / 16; ++ks) {
      const int c = 4 * ks + lq;
      f32x4 a[2], b[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 32 * w + 16 * i + lr;
        a[i] = *reinterpret_cast<const f32x4*>(As + row * GN_BK + 4 * (c ^ (row & 7)));
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int row = 16 * j + lr;
        b[j] = *reinterpret_cast<const f32x4*>(Bs + row * GN_BK + 4 * (c ^ (row & 7)));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
    }
  }
  // lane holds C[4 lq + v][lr] of each 16 x 16 block
  float* Cz = slab + (long)s * slab_stride;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = 16 * j + lr;
      if (col >= N) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) Cz[(long)(m0 + 32 * w + 16 * i + 4 * lq + v) * N + col] = acc[i][j][v];
    }
}
// the narrow kernel's plan: exact products, NT, N <= 48, whole 128-row tiles and 32-k steps; K
// chunks of at least 1024 over up to 32 slabs (c2: 24 row tiles x 32 slabs = 768 workgroups)
bool narrow_ok(int M, int N, int K, long lda, long ldb, int mode) {
  return mode == 0 && N <= GN_BN && M % GN_BM == 0 && K % GN_BK == 0 && K >= 4096 && lda % 4 == 0 &&
         ldb % 4 == 0;
}
int narrow_splitk(int K, int& kchunk) {
  const int sk = std::max(1, std::min(32, K / 1024));
  kchunk = ((K + sk - 1) / sk + GN_BK - 1) / GN_BK * GN_BK;
  return (K + kchunk - 1) / kchunk;
}

// ---- 256 x BN LDS-DMA tile (sv_gemm_f32_256.h) for the exact-fp32 NT GEMMs that tile exactly ----
int gf256_bn(int N) { return N % 256 == 0 ? 256 : 128; }
bool gf256_ok(int M, int N, int K, const float* C, long ldc, const float* b0, const float* b1) {
  return M % GF_BM == 0 && N % 128 == 0 && K % GF_BK == 0 && ldc % 4 == 0 &&
         !(((uintptr_t)C | (uintptr_t)b0 | (uintptr_t)b1) & 15);
}
// one workgroup per CU: split K only to fill the CUs (dW: 36 tiles x 7 slabs at c2)
GemmPlan plan_gf256(int M, int N, int K) {
  GemmPlan p;
  p.bm = GF_BM;
  p.bn = gf256_bn(N);
  const long tiles = (long)(M / GF_BM) * (N / p.bn);
  int sk = 1;
  if (tiles < 256) sk = (int)std::max(1L, std::min(256L / tiles, (long)K / 1024));
  p.kchunk = ((K + sk - 1) / sk + GF_BK - 1) / GF_BK * GF_BK;
  p.splitk = (K + p.kchunk - 1) / p.kchunk;
  return p;
}
template <int BN, int EPI>
void launch_gf256(dim3 grid, hipStream_t s, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                  long slab, int M, int N, int K, int kchunk, const float* b0, const float* b1, float beta) {
  constexpr size_t lds = 2 * (size_t)(GF_BM + BN) * GF_BK * 4;
  hipLaunchKernelGGL((gemm_f32_256_kernel<BN, 32, EPI>), grid, dim3(512), lds, s, A, lda, B, ldb, C, ldc, slab,
                     M, N, K, kchunk, b0, b1, beta);
}
int gemm_f32_256(const float* A, long lda, const float* B, long ldb, float* C, long ldc, int M, int N, int K,
                 const float* bias0, const float* bias1, float beta, float* workspace, hipStream_t stream) {
  const GemmPlan p = plan_gf256(M, N, K);
  const int tiles = (M / GF_BM) * (N / p.bn);
  if (p.splitk == 1) {
    const int cus = sv_stream_cus(stream);
    if (p.bn == 256 && beta == 0.f && cus > 0 && tiles > cus && K / GF_BK <= 32 &&
        K / GF_BK >= 2) {
      // more tiles than CUs, short K (K1; dx's 96 k-tiles measured slower persistent, 3.80 vs
      // 3.73 ms): the persistent form (each tile's k-tile 0 fetched during the previous tile)
      hipLaunchKernelGGL((gemm_f32_256p_kernel<256, 32>), dim3(cus), dim3(512),
                         2 * (size_t)(GF_BM + 256) * GF_BK * 4, stream, A, lda, B, ldb, C, ldc, M, N, K, bias0, bias1);
    } else if (p.bn == 256)
      launch_gf256<256, GF_STORE>(dim3(tiles, 1), stream, A, lda, B, ldb, C, ldc, 0L, M, N, K, p.kchunk, bias0, bias1,
                                  beta);
    else
      launch_gf256<128, GF_STORE>(dim3(tiles, 1), stream, A, lda, B, ldb, C, ldc, 0L, M, N, K, p.kchunk, bias0, bias1,
                                  beta);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (!workspace) return SV_EARG;
  const long slab = (long)M * N;
  if (p.bn == 256)
    launch_gf256<256, GF_SLAB>(dim3(tiles, p.splitk), stream, A, lda, B, ldb, workspace, (long)N, slab, M, N, K,
                               p.kchunk, nullptr, nullptr, 0.f);
  else
    launch_gf256<128, GF_SLAB>(dim3(tiles, p.splitk), stream, A, lda, B, ldb, workspace, (long)N, slab, M, N, K,
                               p.kchunk, nullptr, nullptr, 0.f);
  SV_LAUNCH_CHECK();
  const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C, ldc, M, N, beta,
                     bias0, bias1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// dx = dG W_ih of the fp32 persistent backward with A read from its fragment-order hand-off
// (gemm_f32_256_kernel AF, GfAFrag): the recurrence then writes no row-major dG.  Exact products,
// whole 256-row tiles, whole 32-row groups per slot, one k-split; else -1 (use the row-major dG).
int dx_afrag_bn(int T, int B, int H, int Fl) {
  if (gemm_x() != 0 || B % 32 || H % 32 || ((long)T * B) % GF_BM) return -1;
  if ((unsigned long long)T * B * B >= (1ull << 32) || 4ull * H * H >= (1ull << 32)) return -1;  // gf_afrag's magic
  const int bn = gf256_bn(Fl);
  if (Fl % bn || plan_gf256(T * B, Fl, 4 * H).splitk != 1) return -1;
  return bn;
}
// stream-K scratch of the dx GEMM (gemm_f32_256sk_kernel): two partial slots of 512 threads x 128
// fp32 per workgroup (grid capped at GF_SK_GRID) + the stream-K tiles' arrival counters
constexpr int GF_SK_GRID = 256;
constexpr size_t GF_SK_SLOT = (size_t)512 * 128 * sizeof(float);
size_t gf_sk_bytes() { return 2 * GF_SK_GRID * GF_SK_SLOT + GF_SK_GRID * sizeof(unsigned) * 4; }
int gemm_f32_dx_afrag(int bn, const float* dgf, int T, int B, int H, const float* wihT, long ldw, int Fl, float* dx,
                      hipStream_t s, void* skws = nullptr) {
  const long nrb = (B + 63) / 64, fs = nrb * 8 * (H / 8) * 256;
  const GfAFrag af = gf_afrag(dgf, fs, B, H);
  const int M = T * B, K = 4 * H, tiles = (M / GF_BM) * (Fl / bn);
  const size_t lds = 2 * (size_t)(GF_BM + bn) * GF_BK * 4;
  const int G = std::min(sv_stream_cus(s), GF_SK_GRID), nk = K / GF_BK;
  if (skws && bn == 256 && G > 0 && tiles > G && tiles % G) {
    // c2 dx: 1200 tiles on 256 CUs = 4 whole rounds + 176 tiles as 66 k-tiles per workgroup
    GfSK sk;
    sk.R = tiles / G;
    sk.rem = tiles % G;
    sk.L = (int)(((long)sk.rem * nk + G - 1) / G);
    if (sk.L * 3 >= nk) {  // <= GF_SK_MAXSEG pieces per tile
      sk.part = static_cast<float*>(skws);
      sk.cnt = reinterpret_cast<unsigned*>(static_cast<char*>(skws) + 2 * GF_SK_GRID * GF_SK_SLOT);
      hipError_t e = (hipError_t)sv_zero_counters(sk.cnt, 1, 0, sk.rem, s);
      if (e != hipSuccess) return (int)e;
      hipLaunchKernelGGL((gemm_f32_256sk_kernel<256, 1>), dim3(G), dim3(512), lds, s, nullptr, 0L, wihT, ldw, dx,
                         (long)Fl, M, Fl, K, sk, af);
      SV_LAUNCH_CHECK();
      return SV_OK;
    }
  }
  if (bn == 256)
    hipLaunchKernelGGL((gemm_f32_256_kernel<256, 32, GF_STORE, 1>), dim3(tiles, 1), dim3(512), lds, s, nullptr,
                       0L, wihT, ldw, dx, (long)Fl, 0L, M, Fl, K, K, nullptr, nullptr, 0.f, af);
  else
    hipLaunchKernelGGL((gemm_f32_256_kernel<128, 32, GF_STORE, 1>), dim3(tiles, 1), dim3(512), lds, s, nullptr,
                       0L, wihT, ldw, dx, (long)Fl, 0L, M, Fl, K, K, nullptr, nullptr, 0.f, af);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

}  // namespace

F32ProductScope::F32ProductScope(int mode) : prev(t_f32_mode) { t_f32_mode = mode; }
F32ProductScope::~F32ProductScope() { t_f32_mode = prev; }

extern "C" size_t sv_gemm_f32_workspace(int M, int N, int K) {
  // the larger of the two kernels' split-K slabs (which one runs depends on pointers and mode)
  const GemmPlan p = plan_gemm(M, N, K), pf = plan_gemm(M, N, K, true);  // both plans (gemm_f32's `fine`)
  size_t ws = p.splitk > 1 ? (size_t)p.splitk * M * N * sizeof(float) : 0;
  if (pf.splitk > 1) ws = std::max(ws, (size_t)pf.splitk * M * N * sizeof(float));
  if (M % GF_BM == 0 && N % 128 == 0 && K % GF_BK == 0) {
    const GemmPlan q = plan_gf256(M, N, K);
    if (q.splitk > 1) ws = std::max(ws, (size_t)q.splitk * M * N * sizeof(float));
  }
  if (narrow_ok(M, N, K, K, K, 0)) {  // (the narrow kernel's slabs)
    int kchunk;
    ws = std::max(ws, (size_t)narrow_splitk(K, kchunk) * M * N * sizeof(float));
  }
  return ws;
}

extern "C" int sv_gemm_f32(int a_kcontig, int b_kcontig, int M, int N, int K, const float* A, long lda, const float* B,
                           long ldb, float* C, long ldc, const float* bias0, const float* bias1, float beta,
                           float* workspace, int products, hipStream_t stream) {
  if (products < 0 || products > 3) return SV_EARG;
  F32ProductScope scope(products);
  return gemm_f32(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C, ldc, bias0, bias1, beta, workspace, stream);
}

int gemm_f32(int a_kcontig, int b_kcontig, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
             float* C, long ldc, const float* bias0, const float* bias1, float beta, float* workspace,
             hipStream_t stream, bool fine) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C) return SV_EARG;
  if (a_kcontig ? (K % 4 || lda % 4) : (M % 4 || lda % 4)) return SV_EALIGN;
  if (b_kcontig ? (K % 4 || ldb % 4) : (N % 4 || ldb % 4)) return SV_EALIGN;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return SV_EALIGN;
  if (a_kcontig && b_kcontig && gemm_x() == 0 && gf256_ok(M, N, K, C, ldc, bias0, bias1))
    return gemm_f32_256(A, lda, B, ldb, C, ldc, M, N, K, bias0, bias1, beta, workspace, stream);
  if (a_kcontig && b_kcontig && workspace && narrow_ok(M, N, K, lda, ldb, gemm_x())) {
    int kchunk;
    const int sk = narrow_splitk(K, kchunk);
    const long slab = (long)M * N;
    hipLaunchKernelGGL(gemm_f32_narrow_kernel, dim3(M / GN_BM, sk), dim3(256), 0, stream, A, lda, B, ldb, workspace,
                       slab, M, N, K, kchunk);
    SV_LAUNCH_CHECK();
    const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid), dim3(256), 0, stream, workspace, sk, slab, C, ldc, M, N, beta, bias0,
                       bias1);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  const GemmPlan p = plan_gemm(M, N, K, fine && workspace != nullptr);
  const bool ak = a_kcontig != 0, bk = b_kcontig != 0;
  if (p.splitk == 1) {
    if (p.bm == 64)
      return dispatch_layout<64, 64, EPI_STORE>(ak, bk, A, lda, B, ldb, C, ldc, 0, M, N, K, 1, p.kchunk, bias0, bias1, beta, stream);
    return dispatch_layout<128, 128, EPI_STORE>(ak, bk, A, lda, B, ldb, C, ldc, 0, M, N, K, 1, p.kchunk, bias0, bias1, beta, stream);
  }
  if (!workspace) return SV_EARG;
  const long slab = (long)M * N;
  int rc;
  if (p.bm == 64)
    rc = dispatch_layout<64, 64, EPI_SLAB>(ak, bk, A, lda, B, ldb, workspace, N, slab, M, N, K, p.splitk, p.kchunk, nullptr, nullptr, 0.f, stream);
  else
    rc = dispatch_layout<128, 128, EPI_SLAB>(ak, bk, A, lda, B, ldb, workspace, N, slab, M, N, K, p.splitk, p.kchunk, nullptr, nullptr, 0.f, stream);
  if (rc) return rc;
  const long total = slab;
  const int grid = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C, ldc, M, N, beta,
                     bias0, bias1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// the projection's split-K slabs summed and the rows normalised in one launch (one wave per row,
// P <= 256): y = sum_z slab[z] + bias in slab_reduce_kernel's order, emb = y / |y| and |y| in
// rownorm_fwd_kernel's (sv_misc.hip) -- the two launches' results bit for bit, one launch fewer
#define SR_NZ 8
__global__ __launch_bounds__(256) void slab_rownorm_kernel(const float* __restrict__ slab, int nz, long zstride, int B,
                                                           int P, const float* __restrict__ bias, float* __restrict__ y,
                                                           float* __restrict__ emb, float* __restrict__ ynorm) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= B) return;
  // every slab value of the lane's 4 columns loaded at once (nz <= SR_NZ: one round trip, where a
  // loop over z waited for each load in turn), then summed in z order
  float x[SR_NZ][4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = lane + 64 * j;
    bv[j] = (bias && p < P) ? bias[p] : 0.f;
#pragma unroll
    for (int z = 0; z < SR_NZ; ++z) x[z][j] = (z < nz && p < P) ? slab[z * zstride + (long)r * P + p] : 0.f;
  }
  float v[4];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = lane + 64 * j;
    if (p < P) {
      float s = 0.f;
#pragma unroll
      for (int z = 0; z < SR_NZ; ++z)
        if (z < nz) s += x[z][j];
      if (bias) s += bv[j];
      v[j] = 0.f + s;  // (slab_reduce_kernel's store with beta = 0)
      y[(long)r * P + p] = v[j];
      ss += v[j] * v[j];
    }
  }
  const float n = sqrtf(wave_sum(ss));
  const float inv = 1.0f / n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = lane + 64 * j;
    if (p < P) emb[(long)r * P + p] = v[j] * inv;
  }
  if (lane == 0) ynorm[r] = n;
}

// y = h W^T + b (h [B,K], W [P,K], both k-contiguous) with the row norm fused into the split-K
// reduce where gemm_f32 would take that form (P <= 256, P % 4 == 0); returns 1 if it ran, 0 if
// the caller should take gemm_f32 + its own norm
int proj_norm_fused(const float* h, int B, int K, int P, const float* W, const float* bias, float* y, float* emb,
                    float* ynorm, float* workspace, hipStream_t stream, int* rc) {
  *rc = SV_OK;
  if (!workspace || P > 256 || P % 4 || K % 4 || (((uintptr_t)h | (uintptr_t)W) & 15) || gemm_x() != 0) return 0;
  if (gf256_ok(B, P, K, y, P, bias, nullptr) || narrow_ok(B, P, K, K, K, 0)) return 0;
  const GemmPlan p = plan_gemm(B, P, K, true);
  if (p.splitk <= 1 || p.splitk > SR_NZ) return 0;
  const long slab = (long)B * P;
  if (p.bm == 64)
    *rc = dispatch_layout<64, 64, EPI_SLAB>(true, true, h, K, W, K, workspace, P, slab, B, P, K, p.splitk, p.kchunk,
                                            nullptr, nullptr, 0.f, stream);
  else
    *rc = dispatch_layout<128, 128, EPI_SLAB>(true, true, h, K, W, K, workspace, P, slab, B, P, K, p.splitk, p.kchunk,
                                              nullptr, nullptr, 0.f, stream);
  if (*rc) return 1;
  hipLaunchKernelGGL(slab_rownorm_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, workspace, p.splitk, slab, B, P, bias,
                     y, emb, ynorm);
  *rc = (int)hipGetLastError();
  return 1;
}

extern "C" int sv_frames_to_time_major(const float* x, float* x_tm, int B, int T, int F, hipStream_t stream) {
  if (!x || !x_tm || B <= 0 || T <= 0 || F <= 0) return SV_EARG;
  if (F % 4 || (((uintptr_t)x | (uintptr_t)x_tm) & 15)) return SV_EALIGN;
  const long total = (long)B * T * (F / 4);
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(to_time_major_kernel, dim3(grid), dim3(256), 0, stream, x, x_tm, B, T, F / 4);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_transpose(const float* src, long ld_src, int R, int C, float* dst, long ld_dst, hipStream_t stream) {
  if (!src || !dst || R <= 0 || C <= 0) return SV_EARG;
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, stream, src, ld_src, R, C, dst,
                     ld_dst);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// rows per partial-sum chunk: about 1024 workgroups in all, chunks of 32..1024 rows, so a small R
// (the projection's B rows) still spreads over many workgroups instead of one thread walking
// every row, and a large R keeps the final pass short
static int colsum_rows(int R, int C) {
  const int target = std::max(1, 1024 / ((C + 255) / 256));
  int rpc = (R + target - 1) / target;
  rpc = (rpc + 31) / 32 * 32;
  return std::min(1024, std::max(32, rpc));
}
static int colsum(const float* X, int R, int C, float* out0, float* out1, float* partial, hipStream_t s) {
  const int rows_per_chunk = colsum_rows(R, C);
  const int nchunk = (R + rows_per_chunk - 1) / rows_per_chunk;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((C + 255) / 256, nchunk), dim3(256), 0, s, X, R, C, rows_per_chunk,
                     partial);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, partial, nchunk, C, out0, out1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" size_t sv_colsum_workspace(int R, int C) {
  const int rpc = colsum_rows(R, C);
  return (size_t)((R + rpc - 1) / rpc) * C * sizeof(float);
}

extern "C" int sv_colsum(const float* X, int R, int C, float* out, float* workspace, hipStream_t stream) {
  if (!X || !out || !workspace || R <= 0 || C <= 0) return SV_EARG;
  return colsum(X, R, C, out, nullptr, workspace, stream);
}

static bool lstm_dims_ok(int T, int B, int F, int H) {
  return T > 0 && B > 0 && F > 0 && H > 0 && F % 4 == 0 && H % 4 == 0;
}

namespace {
constexpr int FWD_LDS_MAIN = 2 * (FWD_BM + 4 * FWD_U) * (SV_BKM + 4);
constexpr int FWD_LDS_EPI = FWD_BM * (4 * FWD_U + 4) + FWD_U * (FWD_BM + 1);
constexpr int FWD_LDS = (FWD_LDS_MAIN > FWD_LDS_EPI ? FWD_LDS_MAIN : FWD_LDS_EPI) * (int)sizeof(float);
constexpr int BWD_LDS_MAIN = 4 * 2 * (BWD_BM + BWD_U) * (SV_BKM + 4);
constexpr int BWD_LDS_EPI = 4 * BWD_BM * (BWD_U + 1) + 4 * BWD_U * (BWD_BM + 1);
constexpr int BWD_LDS = (BWD_LDS_MAIN > BWD_LDS_EPI ? BWD_LDS_MAIN : BWD_LDS_EPI) * (int)sizeof(float);
// step-kernel main loops: pipelined local read (gemm_mainloop_km_plr; one barrier per k-tile, LDS
// writes issued behind the first k-group's MFMAs) with 1 register stage for K2 and 2 for K3.
// Measured at c2 against the rolling register prefetch of depth 2 (us): K2 35.1-35.6 vs 41.7,
// K3 37.2-38.0 vs 41.5; c2 step 69.3 -> 66.4-67.0 ms.  The x6 / x3 forms are the bf16x6 product
// mode's (`products`, F32ProductScope): K2 split at the LDS store (x3), K3 exact.
constexpr int FWD_X3_MAIN = 12 * (FWD_BM + 4 * FWD_U) * (32 + 8);
constexpr int FWD_X3_LDS = FWD_X3_MAIN > FWD_LDS ? FWD_X3_MAIN : FWD_LDS;
constexpr int BWD_X3_MAIN = 4 * X3_GBUF_BYTES;
constexpr int BWD_X3_LDS = BWD_X3_MAIN > BWD_LDS ? BWD_X3_MAIN : BWD_LDS;
dim3 fwd_step_grid(int B, int H) { return dim3((H + FWD_U - 1) / FWD_U, (B + FWD_BM - 1) / FWD_BM); }
void launch_fwd_step(dim3 grid, hipStream_t s, const float* hp, const float* whh, float* g, const float* cp, float* c,
                     float* h, float* hT, long ldhT, int t, int Bp, int B, int H) {
  if (k2_x() == 2)
    hipLaunchKernelGGL((lstm_step_fwd_v2_kernel<SV_BKM, 2, false, true>), grid, dim3(512), FWD_X3_LDS, s, hp, whh, g,
                       cp, c, h, hT, ldhT, t, Bp, B, H);
  else if (k2_x() == 1)
    hipLaunchKernelGGL((lstm_step_fwd_v2_kernel<SV_BKM, 2, true>), grid, dim3(512), FWD_LDS, s, hp, whh, g, cp, c, h,
                       hT, ldhT, t, Bp, B, H);
  else
    hipLaunchKernelGGL((lstm_step_fwd_v2_kernel<SV_BKM, SV_PLR + 1>), grid, dim3(512), FWD_LDS, s, hp, whh, g, cp, c, h,
                       hT, ldhT, t, Bp, B, H);
}
void launch_bwd_step(dim3 grid, hipStream_t s, const float* dgn, const float* whhT, const float* up, const float* dcfi,
                     const float* acts, const float* ct, const float* cp, float* dg, float* dcfo, float* dgT,
                     long lddgT, int t, int Bp, int B, int H, unsigned long long* ts = nullptr) {
  if (k3_x() == 2)
    hipLaunchKernelGGL((lstm_step_bwd_v2_kernel<SV_BKM, 2, false, true>), grid, dim3(512), BWD_X3_LDS, s, dgn, whhT, up,
                       dcfi, acts, ct, cp, dg, dcfo, dgT, lddgT, t, Bp, B, H, ts);
  else if (k3_x() == 1)
    hipLaunchKernelGGL((lstm_step_bwd_v2_kernel<SV_BKM, 2, true>), grid, dim3(512), BWD_LDS, s, dgn, whhT, up, dcfi,
                       acts, ct, cp, dg, dcfo, dgT, lddgT, t, Bp, B, H, ts);
  else
    hipLaunchKernelGGL((lstm_step_bwd_v2_kernel<SV_BKM, SV_PLR + 2>), grid, dim3(512), BWD_LDS, s, dgn, whhT, up, dcfi,
                       acts, ct, cp, dg, dcfo, dgT, lddgT, t, Bp, B, H, ts);
}
}  // namespace

extern "C" int sv_lstm_step_fwd(const float* h_prev, const float* w_hh, float* gates_t, const float* c_prev,
                                float* c_t, float* h_t, int B, int H, hipStream_t stream) {
  if (!w_hh || !gates_t || !c_t || !h_t || B <= 0 || H <= 0 || H % 4) return SV_EARG;
  const dim3 grid = fwd_step_grid(B, H);
  launch_fwd_step(grid, stream, h_prev, w_hh, gates_t, c_prev, c_t, h_t, nullptr, 0L, 0, B, B, H);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// one backward recurrent step (K3) on its own (timing / tests): dg_next may be NULL (t = T-1)
extern "C" int sv_lstm_step_bwd(const float* dg_next, const float* w_hhT, const float* dh_up, const float* dcf_next,
                                const float* acts_t, const float* c_t, const float* c_prev, float* dg_t, float* dcf_t,
                                int B, int H, hipStream_t stream) {
  if (!w_hhT || !acts_t || !c_t || !dg_t || !dcf_t || B <= 0 || H <= 0 || H % 4) return SV_EARG;
  const dim3 grid((H + BWD_U - 1) / BWD_U, (B + BWD_BM - 1) / BWD_BM);
  launch_bwd_step(grid, stream, dg_next, w_hhT, dh_up, dcf_next, acts_t, c_t, c_prev, dg_t, dcf_t, nullptr, 0L, 0, B, B,
                  H);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_lstm_layer_fwd(const float* x_tm, int T, int B, int F, int H, const float* w_ih, const float* w_hh,
                                 const float* b_ih, const float* b_hh, float* gates, float* c_tm, float* h_tm,
                                 float* hT, hipStream_t stream) {
  if (!x_tm || !w_ih || !w_hh || !gates || !c_tm || !h_tm) return SV_EARG;
  if (!lstm_dims_ok(T, B, F, H)) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  // K1: all-timestep input projection  gates = x W_ih^T + b_ih + b_hh
  int rc = gemm_f32(1, 1, T * B, 4 * H, F, x_tm, F, w_ih, F, gates, 4L * H, b_ih, b_hh, 0.f, nullptr, stream);
  if (rc) return rc;
  hipError_t e = sv_memset0(h_tm, BH * sizeof(float), stream);
  if (e != hipSuccess) return (int)e;
  const dim3 grid = fwd_step_grid(B, H);
  const int Bp = (B + 3) & ~3;
  const long ldhT = (long)(T + 1) * Bp;
  if (hT && Bp != B) {  // zero the padding columns of the transposed layout
    e = sv_memset0(hT, (size_t)H * ldhT * sizeof(float), stream);
    if (e != hipSuccess) return (int)e;
  }
  for (int t = 0; t < T; ++t) {
    launch_fwd_step(grid, stream, t ? h_tm + t * BH : nullptr, w_hh, gates + t * BG, t ? c_tm + (t - 1) * BH : nullptr,
                    c_tm + t * BH, h_tm + (t + 1) * BH, hT, ldhT, t, Bp, B, H);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

// Row stride (floats) of the library's own W_ih^T copies (fp32 [F][4H]), the dx GEMMs' B operand:
// 4H + 64.  A 12-KB row stride put the 256 rows of a k-tile fill on one L2 channel;
// 64 more floats spread them (the c2 dx GEMM 3707 -> 3654 us isolated, scripts/gemm_ld_ab.py).
static inline long f32_wiht_ld(int H) { return 4L * H + 64; }

namespace {
struct BwdWs {
  float *dcf0, *dcf1, *whhT, *wihT, *gws;
  size_t total;
};
size_t al4(size_t n) { return (n + 63) & ~size_t(63); }
BwdWs carve_bwd(float* base, int T, int B, int F, int H) {
  BwdWs w;
  size_t off = 0;
  auto take = [&](size_t n) {
    float* p = base ? base + off : nullptr;
    off += al4(n);
    return p;
  };
  w.dcf0 = take((size_t)B * H);
  w.dcf1 = take((size_t)B * H);
  w.whhT = take((size_t)4 * H * H);
  w.wihT = take((size_t)f32_wiht_ld(H) * F);
  const int TBp = T * ((B + 3) & ~3);
  size_t g = sv_gemm_f32_workspace(4 * H, H, TBp);
  g = std::max(g, sv_gemm_f32_workspace(4 * H, F, TBp));
  g = std::max(g, sv_gemm_f32_workspace(T * B, F, 4 * H));
  w.gws = take((g + 3) / 4);
  w.total = off * sizeof(float);
  return w;
}
}  // namespace

extern "C" size_t sv_lstm_layer_bwd_workspace(int T, int B, int F, int H) { return carve_bwd(nullptr, T, B, F, H).total; }

extern "C" int sv_lstm_layer_bwd(int T, int B, int F, int H, const float* xT, long ld_xT, const float* w_ih,
                                 const float* w_hh, const float* gates, const float* c_tm, const float* hT,
                                 const float* dh_up, int dh_up_full, float* dgates, float* dgT, float* dx_tm,
                                 float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, float* workspace,
                                 hipStream_t stream) {
  if (!xT || !w_ih || !w_hh || !gates || !c_tm || !hT || !dgates || !dgT || !dw_ih || !dw_hh || !db_ih || !workspace)
    return SV_EARG;
  if (!lstm_dims_ok(T, B, F, H) || ld_xT % 4) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 3) & ~3;
  const int TB = T * B, TBp = T * Bp;
  const BwdWs ws = carve_bwd(workspace, T, B, F, H);
  int rc = sv_transpose(w_hh, H, 4 * H, H, ws.whhT, 4L * H, stream);  // W_hh^T [H, 4H]
  if (rc) return rc;
  const dim3 grid((H + BWD_U - 1) / BWD_U, (B + BWD_BM - 1) / BWD_BM);
  if (Bp != B) {
    hipError_t e = sv_memset0(dgT, (size_t)4 * H * TBp * sizeof(float), stream);
    if (e != hipSuccess) return (int)e;
  }
  for (int t = T - 1; t >= 0; --t) {
    const float* up = nullptr;
    if (dh_up) up = dh_up_full ? dh_up + t * BH : (t == T - 1 ? dh_up : nullptr);
    float* dcf_out = (t & 1) ? ws.dcf1 : ws.dcf0;
    const float* dcf_in = (t == T - 1) ? nullptr : ((t & 1) ? ws.dcf0 : ws.dcf1);
    launch_bwd_step(grid, stream, t == T - 1 ? nullptr : dgates + (t + 1) * BG, ws.whhT, up, dcf_in, gates + t * BG,
                    c_tm + t * BH, t ? c_tm + (t - 1) * BH : nullptr, dgates + t * BG, dcf_out, dgT, (long)TBp, t, Bp,
                    B, H);
    SV_LAUNCH_CHECK();
  }
  const long ldhT = (long)(T + 1) * Bp;
  // dW_hh = sum_t dG_t^T h_{t-1}: A = dG^T [4H, T Bp], B = hT[:, 0:T Bp] (column block t = h_{t-1})
  rc = gemm_f32(1, 1, 4 * H, H, TBp, dgT, TBp, hT, ldhT, dw_hh, H, nullptr, nullptr, 0.f, ws.gws, stream);
  if (rc) return rc;
  // dW_ih = sum_t dG_t^T x_t: B = x^T [F, T Bp]
  rc = gemm_f32(1, 1, 4 * H, F, TBp, dgT, TBp, xT, ld_xT, dw_ih, F, nullptr, nullptr, 0.f, ws.gws, stream);
  if (rc) return rc;
  // db_ih = db_hh = row sums of dG^T
  hipLaunchKernelGGL(rowsum_kernel, dim3(4 * H), dim3(RS_T), 0, stream, dgT, (long)TBp, TBp, db_ih, db_hh);
  SV_LAUNCH_CHECK();
  // dx = dG W_ih: A = dG [TB, 4H], B = W_ih^T [F, 4H]
  if (dx_tm) {
    rc = sv_transpose(w_ih, F, 4 * H, F, ws.wihT, f32_wiht_ld(H), stream);
    if (rc) return rc;
    rc = gemm_f32(1, 1, TB, F, 4 * H, dgates, 4L * H, ws.wihT, f32_wiht_ld(H), dx_tm, F, nullptr, nullptr, 0.f, ws.gws,
                     stream);
    if (rc) return rc;
  }
  return SV_OK;
}

// ============================================================================
// Layer-pipelined stack forward.  Layer l runs on side[l]; its timesteps are processed in
// chunks of `chunk`: [chunk input-projection GEMM (K1) -> chunk step kernels (K2)].  Layer l
// waits only for layer l-1 to finish the same chunk, so up to L layers' kernels run at once
// and one layer's latency-bound step kernels overlap another's GEMM / steps (each K2 block
// leaves room for a second resident block per CU).  Joins back into `main` before returning.
// Host arrays (length L) carry the per-layer device pointers; ev needs L*ceil(T/chunk) + 1
// caller-created events.
// ============================================================================
// the fp32 W-stationary persistent recurrences (sv_persist_f32.hip) instead of the per-step
// kernels: never under SV_SCHED_PER_STEP; where they fit co-resident, under SV_SCHED_PERSIST
// always, under SV_SCHED_AUTO when the grid fills at least 3/4 of the device (c2: 240 of 256 CUs;
// a half-empty grid leaves the chip to per-step kernels that share it with the GEMMs)
static bool f32_persist(int schedule, int B, int H, hipStream_t s) {
  if (schedule & SV_SCHED_PER_STEP) return false;
  const int cus = sv_stream_cus(s);
  if (!sv_persist_f32_fits(B, H, cus)) return false;
  return (schedule & SV_SCHED_PERSIST) || 4L * (H / 32) * ((B + 63) / 64) >= 3L * cus;
}

extern "C" int sv_lstm_f32_persist_ok(int B, int H, int schedule) { return f32_persist(schedule, B, H, nullptr); }

extern "C" int sv_lstm_stack_fwd(int L, int T, int B, int F, int H, const float* x_tm, const float* const* w_ih,
                                 const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                                 float* const* gates, float* const* c_tm, float* const* h_tm, float* const* hT,
                                 int chunk, hipStream_t main, const hipStream_t* side, hipEvent_t* ev,
                                 int products, int schedule, unsigned* sync, hipEvent_t* probe) {
  if (L <= 0 || !x_tm || !w_ih || !w_hh || !gates || !c_tm || !h_tm || !side || !ev || chunk <= 0) return SV_EARG;
  if (products < 0 || products > 3 || schedule < 0 || schedule > SV_SCHED_MASK) return SV_EARG;
  F32ProductScope scope(products);
  if (!lstm_dims_ok(T, B, F, H)) return SV_ESHAPE;
  const int nch = (T + chunk - 1) / chunk;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 3) & ~3;
  const long ldhT = (long)(T + 1) * Bp;
  hipError_t e;
  if (f32_persist(schedule, B, H, main)) {
    // one layer after another on `main`: the whole-T input projection (K1), then ONE persistent
    // launch for the layer's recurrence (the persistent grid needs the whole chip)
    if (!sync) return SV_EARG;
    for (int l = 0; l < L; ++l) {
      const int Fl = l == 0 ? F : H;
      const float* in = l == 0 ? x_tm : h_tm[l - 1] + BH;
      if ((e = sv_memset0(h_tm[l], BH * sizeof(float), main)) != hipSuccess) return (int)e;
      if (hT[l] && Bp != B && (e = sv_memset0(hT[l], (size_t)H * ldhT * sizeof(float), main)) != hipSuccess)
        return (int)e;
      // layer 0 at F = 40: the input projection inside the recurrence (c2 layer 0:
      // the K=40 GEMM wrote 1.26 GB that the recurrence read back)
      // (exact fp32 products only: the bf16x6 mode keeps the GEMM, whose products it splits; and 16-B
      // aligned x_tm / W_ih only: the kernel reads them by LDS-DMA / f32x4 -- else the GEMM path
      // rejects the misaligned pointer with SV_EALIGN)
      const bool fuse = l == 0 && F == 40 && products == 0 &&
                        !(((uintptr_t)x_tm | (uintptr_t)w_ih[0]) & 15);
      int rc = 0;
      if (!fuse) {
        rc = gemm_f32(1, 1, T * B, 4 * H, Fl, in, Fl, w_ih[l], Fl, gates[l], 4L * H, b_ih[l], b_hh[l], 0.f, nullptr,
                      main);
        if (rc) return rc;
      }
      rc = sv_persist_fwd_f32(T, B, H, w_hh[l], gates[l], c_tm[l], h_tm[l], hT[l], main, sync, 0,
                              probe ? probe[2 * l] : nullptr, probe ? probe[2 * l + 1] : nullptr,
                              fuse ? x_tm : nullptr, F, w_ih[l], b_ih[l], b_hh[l]);
      if (rc) return rc;
    }
    return SV_OK;
  }
  hipEvent_t ev_start = ev[L * nch];
  e = hipEventRecord(ev_start, main);
  if (e != hipSuccess) return (int)e;
  for (int l = 0; l < L; ++l) {
    hipStream_t s = side[l];
    if ((e = hipStreamWaitEvent(s, ev_start, 0)) != hipSuccess) return (int)e;
    if ((e = sv_memset0(h_tm[l], BH * sizeof(float), s)) != hipSuccess) return (int)e;
    if (hT[l] && Bp != B && (e = sv_memset0(hT[l], (size_t)H * ldhT * sizeof(float), s)) != hipSuccess)
      return (int)e;
  }
  const dim3 grid = fwd_step_grid(B, H);
  // wavefront issue order: chunk c of layer l after chunk c of layer l-1 on the host too
  for (int c = 0; c < nch + L - 1; ++c) {
    for (int l = 0; l < L; ++l) {
      const int cc = c - l;
      if (cc < 0 || cc >= nch) continue;
      hipStream_t s = side[l];
      const int t0 = cc * chunk, t1 = std::min(T, t0 + chunk);
      const int Fl = l == 0 ? F : H;
      const float* in = l == 0 ? x_tm + (long)t0 * B * F : h_tm[l - 1] + (long)(t0 + 1) * BH;
      if (l > 0 && (e = hipStreamWaitEvent(s, ev[(l - 1) * nch + cc], 0)) != hipSuccess) return (int)e;
      int rc = gemm_f32(1, 1, (t1 - t0) * B, 4 * H, Fl, in, Fl, w_ih[l], Fl, gates[l] + t0 * BG, 4L * H, b_ih[l],
                           b_hh[l], 0.f, nullptr, s);
      if (rc) return rc;
      for (int t = t0; t < t1; ++t) {
        launch_fwd_step(grid, s, t ? h_tm[l] + t * BH : nullptr, w_hh[l], gates[l] + t * BG,
                        t ? c_tm[l] + (t - 1) * BH : nullptr, c_tm[l] + t * BH, h_tm[l] + (t + 1) * BH, hT[l], ldhT,
                        t, Bp, B, H);
        SV_LAUNCH_CHECK();
      }
      if ((e = hipEventRecord(ev[l * nch + cc], s)) != hipSuccess) return (int)e;
    }
  }
  for (int l = 0; l < L; ++l)
    if ((e = hipStreamWaitEvent(main, ev[l * nch + nch - 1], 0)) != hipSuccess) return (int)e;
  return SV_OK;
}

// ============================================================================
// Layer-pipelined stack backward.  Layer l runs on side[l], top layer first in issue order:
// its timesteps in reverse chunks of `chunk` (K3 steps, then -- for l > 0 -- the chunk's
// dx = dG W_ih GEMM, which is the next-lower layer's dh_up for those timesteps), then its
// whole-T weight-gradient GEMMs and bias row sums behind the recurrence on the same stream.
// Layer l-1 waits only for layer l's dx of the same chunk, so one layer's (latency-bound)
// recurrence overlaps the upper layers' GEMMs.
//   xT[l], ld_xT[l]: layer input transposed (layer 0: the frames; l > 0: hT[l-1] + Bp cols)
//   dx[l] [T,B,H] for l > 0 (dh_up of layer l-1); dx[0] may be NULL
//   workspace: sv_lstm_stack_bwd_workspace bytes; side: L streams
//   ev: L*ceil(T/chunk) + L + 1 caller-created events.  Joins back into `main`.
// ============================================================================
extern "C" size_t sv_lstm_stack_bwd_workspace(int L, int T, int B, int F, int H) {
  // + the persistent backward's fragment-order hand-off (shared by the layers, one after another)
  // + the dx GEMM's stream-K scratch behind it
  const size_t dgf = H == 768 ? ((sv_persist_f32_bwd_scratch(T, B, H) + 255) & ~size_t(255)) + gf_sk_bytes() : 0;
  return (size_t)L * ((carve_bwd(nullptr, T, B, std::max(F, H), H).total + 255) & ~size_t(255)) + dgf;
}

extern "C" int sv_lstm_stack_bwd(int L, int T, int B, int F, int H, const float* const* xT, const long* ld_xT,
                                 const float* const* w_ih, const float* const* w_hh, const float* const* gates,
                                 const float* const* c_tm, const float* const* hT, const float* dh_last,
                                 float* const* dgates, float* const* dgT, float* const* dx, float* const* dw_ih,
                                 float* const* dw_hh, float* const* db_ih, float* const* db_hh, float* workspace,
                                 int chunk, hipStream_t main, const hipStream_t* side, hipEvent_t* ev,
                                 int products, hipEvent_t* probe, unsigned long long* kstamp, int schedule,
                                 unsigned* sync) {
  if (L <= 0 || !xT || !ld_xT || !w_ih || !w_hh || !gates || !c_tm || !hT || !dh_last || !dgates || !dgT || !dx ||
      !dw_ih || !dw_hh || !db_ih || !workspace || !side || !ev || chunk <= 0)
    return SV_EARG;
  if (products < 0 || products > 3 || schedule < 0 || schedule > SV_SCHED_MASK) return SV_EARG;
  F32ProductScope scope(products);
  if (!lstm_dims_ok(T, B, F, H)) return SV_ESHAPE;
  const int nch = (T + chunk - 1) / chunk;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 3) & ~3;
  const int TBp = T * Bp;
  const long ldhT = (long)(T + 1) * Bp;
  const size_t per = (carve_bwd(nullptr, T, B, std::max(F, H), H).total + 255) & ~size_t(255);
  hipError_t e;
  if (f32_persist(schedule, B, H, main)) {
    // per layer, top first, all on `main`: ONE persistent launch for the recurrence, then the
    // whole-T dx = dG W_ih GEMM (the next layer's dh_up), the dW GEMMs and the bias row sums
    if (!sync) return SV_EARG;
    float* dgf = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + per * L);
    void* skws = reinterpret_cast<char*>(dgf) + ((sv_persist_f32_bwd_scratch(T, B, H) + 255) & ~size_t(255));
    for (int l = L - 1; l >= 0; --l) {
      const int Fl = l == 0 ? F : H;
      const BwdWs ws = carve_bwd((float*)((char*)workspace + per * l), T, B, std::max(F, H), H);
      int rc = sv_transpose(w_hh[l], H, 4 * H, H, ws.whhT, 4L * H, main);
      if (rc) return rc;
      if (l > 0 && (rc = sv_transpose(w_ih[l], Fl, 4 * H, Fl, ws.wihT, f32_wiht_ld(H), main))) return rc;
      const float* up = l == L - 1 ? dh_last : dx[l + 1];
      // the row-major dG only where a dx GEMM needs it and cannot read the fragment-order hand-off
      // (layer 0 computes no dx here)
      const int abn = l > 0 ? dx_afrag_bn(T, B, H, Fl) : 0;
      rc = sv_persist_bwd_f32(T, B, H, ws.whhT, gates[l], c_tm[l], up, l < L - 1, abn < 0 ? dgates[l] : nullptr,
                              dgT[l], dgf, main, sync, probe ? probe[2 * l] : nullptr,
                              probe ? probe[2 * l + 1] : nullptr, db_ih[l], db_hh ? db_hh[l] : nullptr);
      if (rc) return rc;
      // the completion events of layers >= 1 (grad_ready: a caller's bucketed all-reduce) fire once
      // the last recurrence is done, so a collective never shares the device with a persistent
      // launch (a concurrent RCCL kernel would hold CUs its grid waits for) but overlaps layer 0's
      // weight-gradient GEMMs
      for (int k = 1; l == 0 && k < L && !(schedule & SV_SCHED_NO_EVENTS); ++k)
        if ((e = hipEventRecord(ev[L * nch + k], main)) != hipSuccess) return (int)e;
      if (l > 0 && abn > 0 && (rc = gemm_f32_dx_afrag(abn, dgf, T, B, H, ws.wihT, f32_wiht_ld(H), Fl, dx[l], main, skws))) return rc;
      if (l > 0 && abn < 0 &&
          (rc = gemm_f32(1, 1, T * B, Fl, 4 * H, dgates[l], 4L * H, ws.wihT, f32_wiht_ld(H), dx[l], Fl, nullptr, nullptr, 0.f,
                         ws.gws, main)))
        return rc;
      if ((rc = gemm_f32(1, 1, 4 * H, H, TBp, dgT[l], TBp, hT[l], ldhT, dw_hh[l], H, nullptr, nullptr, 0.f, ws.gws,
                         main)))
        return rc;
      if ((rc = gemm_f32(1, 1, 4 * H, Fl, TBp, dgT[l], TBp, xT[l], ld_xT[l], dw_ih[l], Fl, nullptr, nullptr, 0.f,
                         ws.gws, main)))
        return rc;
      // (bias gradients: summed inside the persistent recurrence, finalized after it)
    }
    if (!(schedule & SV_SCHED_NO_EVENTS) && (e = hipEventRecord(ev[L * nch], main)) != hipSuccess) return (int)e;
    return SV_OK;
  }
  hipEvent_t ev_start = ev[L * nch + L];
  e = hipEventRecord(ev_start, main);
  if (e != hipSuccess) return (int)e;
  const dim3 grid((H + BWD_U - 1) / BWD_U, (B + BWD_BM - 1) / BWD_BM);
  for (int l = L - 1; l >= 0; --l) {
    hipStream_t s = side[l];
    const int Fl = l == 0 ? F : H;
    const BwdWs ws = carve_bwd((float*)((char*)workspace + per * l), T, B, std::max(F, H), H);
    if ((e = hipStreamWaitEvent(s, ev_start, 0)) != hipSuccess) return (int)e;
    int rc = sv_transpose(w_hh[l], H, 4 * H, H, ws.whhT, 4L * H, s);
    if (rc) return rc;
    if (l > 0 && (rc = sv_transpose(w_ih[l], Fl, 4 * H, Fl, ws.wihT, f32_wiht_ld(H), s))) return rc;
    if (Bp != B && (e = sv_memset0(dgT[l], (size_t)4 * H * TBp * sizeof(float), s)) != hipSuccess) return (int)e;
    for (int c = nch - 1; c >= 0; --c) {
      const int t0 = c * chunk, t1 = std::min(T, t0 + chunk);
      if (l < L - 1 && (e = hipStreamWaitEvent(s, ev[(l + 1) * nch + c], 0)) != hipSuccess) return (int)e;
      // timing probe: one K3 launch per chunk (the chunk's second, behind a running K3 on its
      // stream; the first if the chunk has one) bracketed by the caller's event pair
      const int tp = t1 - t0 > 1 ? t1 - 2 : t0;
      for (int t = t1 - 1; t >= t0; --t) {
        const float* up = (l == L - 1) ? (t == T - 1 ? dh_last : nullptr) : dx[l + 1] + t * BH;
        float* dcf_out = (t & 1) ? ws.dcf1 : ws.dcf0;
        const float* dcf_in = (t == T - 1) ? nullptr : ((t & 1) ? ws.dcf0 : ws.dcf1);
        if (probe && t == tp && (e = hipEventRecord(probe[2 * (l * nch + c)], s)) != hipSuccess) return (int)e;
        launch_bwd_step(grid, s, t == T - 1 ? nullptr : dgates[l] + (t + 1) * BG, ws.whhT, up, dcf_in,
                        gates[l] + t * BG, c_tm[l] + t * BH, t ? c_tm[l] + (t - 1) * BH : nullptr, dgates[l] + t * BG,
                        dcf_out, dgT[l], (long)TBp, t, Bp, B, H,
                        kstamp ? kstamp + 2 * ((long)l * T + t) : nullptr);
        SV_LAUNCH_CHECK();
        if (probe && t == tp && (e = hipEventRecord(probe[2 * (l * nch + c) + 1], s)) != hipSuccess) return (int)e;
      }
      if (l > 0) {  // dh_up of layer l-1 for this chunk: dx = dG W_ih
        rc = gemm_f32(1, 1, (t1 - t0) * B, Fl, 4 * H, dgates[l] + t0 * BG, 4L * H, ws.wihT, f32_wiht_ld(H),
                      dx[l] + (long)t0 * B * Fl, Fl, nullptr, nullptr, 0.f, ws.gws, s);
        if (rc) return rc;
      }
      if ((e = hipEventRecord(ev[l * nch + c], s)) != hipSuccess) return (int)e;
    }
    // whole-T weight gradients behind the recurrence, on its stream
    rc = gemm_f32(1, 1, 4 * H, H, TBp, dgT[l], TBp, hT[l], ldhT, dw_hh[l], H, nullptr, nullptr, 0.f, ws.gws, s);
    if (rc) return rc;
    rc = gemm_f32(1, 1, 4 * H, Fl, TBp, dgT[l], TBp, xT[l], ld_xT[l], dw_ih[l], Fl, nullptr, nullptr, 0.f, ws.gws, s);
    if (rc) return rc;
    hipLaunchKernelGGL(rowsum_kernel, dim3(4 * H), dim3(RS_T), 0, s, dgT[l], (long)TBp, TBp, db_ih[l],
                       db_hh ? db_hh[l] : nullptr);
    SV_LAUNCH_CHECK();
    if ((e = hipEventRecord(ev[L * nch + l], s)) != hipSuccess) return (int)e;
  }
  for (int l = 0; l < L; ++l)
    if ((e = hipStreamWaitEvent(main, ev[L * nch + l], 0)) != hipSuccess) return (int)e;
  return SV_OK;
}
