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
#include "sv_common.h"
#include "sv_gemm.h"
#include "../../include/sv_ge2e.h"

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
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * ((N + BN - 1) / BN);
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tm = id % tiles_m, tn = id / tiles_m;
  const int kbeg = blockIdx.y * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int wm0 = (w >> 1) * (BM / 2), wn0 = (w & 1) * (BN / 2);
  f32x16 acc[TM][TN];
  zero_acc(acc);
  gemm_mainloop<BM, BN, 256, AK, BKC, TM, TN>(A, lda, RowMapLinear{tm * BM, M}, B, ldb, RowMapLinear{tn * BN, N},
                                              kbeg, kend, lds, tid, wm0, wn0, acc);
  float* Cz = C + (EPI == EPI_SLAB ? (long)blockIdx.y * slab : 0);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = tn * BN + wn0 + 32 * j + (lane & 31);
      if (col >= N) continue;
      float badd = 0.f;
      if (EPI == EPI_STORE) {
        if (bias0) badd += bias0[col];
        if (bias1) badd += bias1[col];
      }
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

// ============================================================================
// K2: forward recurrent step.  Block = 64 batch rows x 32 hidden units (= 128 gate
// columns: i,f,g,o of those units), 4 waves in 2x2; K = H.  Epilogue: + x-projection,
// sigmoid/tanh, c_t = f c_{t-1} + i g, h_t = o tanh(c_t).
// ============================================================================
#define FWD_BM 64
#define FWD_U 32

__global__ __launch_bounds__(256) void lstm_step_fwd_kernel(const float* __restrict__ hprev,
                                                            const float* __restrict__ whh, float* __restrict__ gates,
                                                            const float* __restrict__ cprev, float* __restrict__ cout,
                                                            float* __restrict__ hout, int B, int H) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int BN = 4 * FWD_U, LDP = BN + 4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * FWD_U, b0 = blockIdx.y * FWD_BM;
  const int wm0 = (w >> 1) * 32, wn0 = (w & 1) * 64;
  f32x16 acc[1][2];
  zero_acc(acc);
  if (hprev)
    gemm_mainloop<FWD_BM, BN, 256, true, true, 1, 2>(hprev + (long)b0 * H, H, RowMapLinear{0, B - b0}, whh, H,
                                                     RowMapGates<FWD_U>{j0, H}, 0, H, lds, tid, wm0, wn0, acc);
  // pre-activations (recurrent part) -> LDS [64][LDP]
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[(wm0 + acc_row(r, lane)) * LDP + wn0 + 32 * j + (lane & 31)] = acc[0][j][r];
  __syncthreads();
  const long G = 4L * H;
  for (int e = tid; e < FWD_BM * FWD_U; e += 256) {
    const int b = e / FWD_U, u = e % FWD_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    float* gp = gates + (long)gb * G + gj;
    const float* pr = lds + b * LDP + u;
    const float pi = pr[0] + gp[0];
    const float pf = pr[FWD_U] + gp[H];
    const float pg = pr[2 * FWD_U] + gp[2 * H];
    const float po = pr[3 * FWD_U] + gp[3 * H];
    const float i = sv_sigmoid(pi), f = sv_sigmoid(pf), g = tanhf(pg), o = sv_sigmoid(po);
    const float cp = cprev ? cprev[(long)gb * H + gj] : 0.f;
    const float c = f * cp + i * g;
    const float h = o * tanhf(c);
    gp[0] = i;
    gp[H] = f;
    gp[2 * H] = g;
    gp[3 * H] = o;
    cout[(long)gb * H + gj] = c;
    hout[(long)gb * H + gj] = h;
  }
}

// ============================================================================
// K3: backward recurrent step at time t.  Block = 64 batch rows x 32 hidden units;
// wave w computes dG_{t+1}[:, gate w] . W_hh[gate w rows, units] (K = H each, an
// in-block split of K = 4H by gate), partials summed in LDS in fixed order.
// Epilogue: dh = that + dh_up; dc = dc_{t+1} f_{t+1} + dh o (1 - tanh^2 c);
// dG_t = [dc g i(1-i), dc c_{t-1} f(1-f), dc i (1-g^2), dh tanh(c) o(1-o)].
// ============================================================================
#define BWD_BM 64
#define BWD_U 32

__global__ __launch_bounds__(256) void lstm_step_bwd_kernel(
    const float* __restrict__ dgnext, const float* __restrict__ whh, const float* __restrict__ dhup,
    const float* __restrict__ dcf_next, const float* __restrict__ acts, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, float* __restrict__ dg, float* __restrict__ dcf, int B, int H) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int LDA = TileLd<true, BWD_BM>::value, LDB = TileLd<false, BWD_U>::value;
  constexpr int WBUF = 2 * SV_BK * (LDA + LDB);
  constexpr int LDR = BWD_U + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * BWD_U, b0 = blockIdx.y * BWD_BM;
  const long G = 4L * H;
  f32x16 acc[2][1];
  zero_acc(acc);
  if (dgnext)
    gemm_mainloop<BWD_BM, BWD_U, 64, true, false, 2, 1>(dgnext + (long)b0 * G, G, RowMapLinear{0, B - b0}, whh, H,
                                                        RowMapLinear{j0, H}, w * H, (w + 1) * H, lds + w * WBUF,
                                                        lane, 0, 0, acc);
  __syncthreads();
  float* red = lds;  // [4][64][LDR]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(w * BWD_BM + 32 * i + acc_row(r, lane)) * LDR + (lane & 31)] = acc[i][0][r];
  __syncthreads();
  for (int e = tid; e < BWD_BM * BWD_U; e += 256) {
    const int b = e / BWD_U, u = e % BWD_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    const long hi = (long)gb * H + gj;
    float dh = red[(0 * BWD_BM + b) * LDR + u];
    dh += red[(1 * BWD_BM + b) * LDR + u];
    dh += red[(2 * BWD_BM + b) * LDR + u];
    dh += red[(3 * BWD_BM + b) * LDR + u];
    if (dhup) dh += dhup[hi];
    const float* ap = acts + (long)gb * G + gj;
    const float i = ap[0], f = ap[H], g = ap[2 * H], o = ap[3 * H];
    const float c = c_t[hi];
    const float tc = tanhf(c);
    float dc = dh * o * (1.f - tc * tc);
    if (dcf_next) dc += dcf_next[hi];
    const float cp = c_prev ? c_prev[hi] : 0.f;
    float* dp = dg + (long)gb * G + gj;
    dp[0] = dc * g * i * (1.f - i);
    dp[H] = dc * cp * f * (1.f - f);
    dp[2 * H] = dc * i * (1.f - g * g);
    dp[3 * H] = dh * tc * o * (1.f - o);
    dcf[hi] = dc * f;
  }
}

// ============================================================================
// host side
// ============================================================================
namespace {

template <int BM, int BN, bool AK, bool BKC, int EPI>
int launch_gemm_t(const float* A, long lda, const float* B, long ldb, float* C, long ldc, long slab, int M, int N,
                  int K, int splitk, int kchunk, const float* b0, const float* b1, float beta, hipStream_t s) {
  constexpr int LDS_FLOATS = 2 * SV_BK * (TileLd<AK, BM>::value + TileLd<BKC, BN>::value);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AK, BKC, EPI>), dim3(tiles, splitk), dim3(256),
                     LDS_FLOATS * sizeof(float), s, A, lda, B, ldb, C, ldc, slab, M, N, K, kchunk, b0, b1, beta);
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

GemmPlan plan_gemm(int M, int N, int K) {
  GemmPlan p;
  const bool small = (long)((M + 127) / 128) * ((N + 127) / 128) < 128;
  p.bm = small ? 64 : 128;
  p.bn = small ? 64 : 128;
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  int sk = 1;
  while (tiles * sk < 512 && K / (sk * 2) >= 256 && sk < 32) sk *= 2;
  p.splitk = sk;
  p.kchunk = ((K + sk - 1) / sk + SV_BK - 1) / SV_BK * SV_BK;
  p.splitk = (K + p.kchunk - 1) / p.kchunk;
  return p;
}

}  // namespace

extern "C" size_t sv_gemm_f32_workspace(int M, int N, int K) {
  const GemmPlan p = plan_gemm(M, N, K);
  return p.splitk > 1 ? (size_t)p.splitk * M * N * sizeof(float) : 0;
}

extern "C" int sv_gemm_f32(int a_kcontig, int b_kcontig, int M, int N, int K, const float* A, long lda, const float* B,
                           long ldb, float* C, long ldc, const float* bias0, const float* bias1, float beta,
                           float* workspace, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C) return SV_EARG;
  if (a_kcontig ? (K % 4 || lda % 4) : (M % 4 || lda % 4)) return SV_EALIGN;
  if (b_kcontig ? (K % 4 || ldb % 4) : (N % 4 || ldb % 4)) return SV_EALIGN;
  if (((uintptr_t)A | (uintptr_t)B) & 15) return SV_EALIGN;
  const GemmPlan p = plan_gemm(M, N, K);
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

extern "C" int sv_frames_to_time_major(const float* x, float* x_tm, int B, int T, int F, hipStream_t stream) {
  if (!x || !x_tm || B <= 0 || T <= 0 || F <= 0) return SV_EARG;
  if (F % 4 || (((uintptr_t)x | (uintptr_t)x_tm) & 15)) return SV_EALIGN;
  const long total = (long)B * T * (F / 4);
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(to_time_major_kernel, dim3(grid), dim3(256), 0, stream, x, x_tm, B, T, F / 4);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

static int colsum(const float* X, int R, int C, float* out0, float* out1, float* partial, hipStream_t s) {
  const int rows_per_chunk = 1024;
  const int nchunk = (R + rows_per_chunk - 1) / rows_per_chunk;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((C + 255) / 256, nchunk), dim3(256), 0, s, X, R, C, rows_per_chunk,
                     partial);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, partial, nchunk, C, out0, out1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" size_t sv_colsum_workspace(int R, int C) { return (size_t)((R + 1023) / 1024) * C * sizeof(float); }

extern "C" int sv_colsum(const float* X, int R, int C, float* out, float* workspace, hipStream_t stream) {
  if (!X || !out || !workspace || R <= 0 || C <= 0) return SV_EARG;
  return colsum(X, R, C, out, nullptr, workspace, stream);
}

static bool lstm_dims_ok(int T, int B, int F, int H) {
  return T > 0 && B > 0 && F > 0 && H > 0 && F % 4 == 0 && H % 4 == 0;
}

extern "C" int sv_lstm_layer_fwd(const float* x_tm, int T, int B, int F, int H, const float* w_ih, const float* w_hh,
                                 const float* b_ih, const float* b_hh, float* gates, float* c_tm, float* h_tm,
                                 hipStream_t stream) {
  if (!x_tm || !w_ih || !w_hh || !gates || !c_tm || !h_tm) return SV_EARG;
  if (!lstm_dims_ok(T, B, F, H)) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  // K1: all-timestep input projection  gates = x W_ih^T + b_ih + b_hh
  int rc = sv_gemm_f32(1, 1, T * B, 4 * H, F, x_tm, F, w_ih, F, gates, 4L * H, b_ih, b_hh, 0.f, nullptr, stream);
  if (rc) return rc;
  hipError_t e = hipMemsetAsync(h_tm, 0, BH * sizeof(float), stream);
  if (e != hipSuccess) return (int)e;
  constexpr int LDS_MAIN = 2 * SV_BK * (TileLd<true, FWD_BM>::value + TileLd<true, 4 * FWD_U>::value);
  constexpr int LDS_EPI = FWD_BM * (4 * FWD_U + 4);
  constexpr int LDS = (LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI) * sizeof(float);
  const dim3 grid((H + FWD_U - 1) / FWD_U, (B + FWD_BM - 1) / FWD_BM);
  for (int t = 0; t < T; ++t) {
    hipLaunchKernelGGL(lstm_step_fwd_kernel, grid, dim3(256), LDS, stream, t ? h_tm + t * BH : nullptr, w_hh,
                       gates + t * BG, t ? c_tm + (t - 1) * BH : nullptr, c_tm + t * BH, h_tm + (t + 1) * BH, B, H);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

// one forward recurrent step (K2) on its own: gates_t holds x_t W_ih^T + b on entry
extern "C" int sv_lstm_step_fwd(const float* h_prev, const float* w_hh, float* gates_t, const float* c_prev,
                                float* c_t, float* h_t, int B, int H, hipStream_t stream) {
  if (!w_hh || !gates_t || !c_t || !h_t || B <= 0 || H <= 0 || H % 4) return SV_EARG;
  constexpr int LDS_MAIN = 2 * SV_BK * (TileLd<true, FWD_BM>::value + TileLd<true, 4 * FWD_U>::value);
  constexpr int LDS_EPI = FWD_BM * (4 * FWD_U + 4);
  constexpr int LDS = (LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI) * sizeof(float);
  const dim3 grid((H + FWD_U - 1) / FWD_U, (B + FWD_BM - 1) / FWD_BM);
  hipLaunchKernelGGL(lstm_step_fwd_kernel, grid, dim3(256), LDS, stream, h_prev, w_hh, gates_t, c_prev, c_t, h_t, B, H);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" size_t sv_lstm_layer_bwd_workspace(int T, int B, int F, int H) {
  size_t dcf = 2ull * B * H * sizeof(float);
  size_t g1 = sv_gemm_f32_workspace(4 * H, H, T * B);
  size_t g2 = sv_gemm_f32_workspace(4 * H, F, T * B);
  size_t g3 = sv_gemm_f32_workspace(T * B, F, 4 * H);
  size_t cs = sv_colsum_workspace(T * B, 4 * H);
  size_t m = g1;
  if (g2 > m) m = g2;
  if (g3 > m) m = g3;
  if (cs > m) m = cs;
  return dcf + ((m + 255) & ~size_t(255));
}

extern "C" int sv_lstm_layer_bwd(int T, int B, int F, int H, const float* x_tm, const float* w_ih, const float* w_hh,
                                 const float* gates, const float* c_tm, const float* h_tm, const float* dh_up,
                                 int dh_up_full, float* dgates, float* dx_tm, float* dw_ih, float* dw_hh,
                                 float* db_ih, float* db_hh, float* workspace, hipStream_t stream) {
  if (!x_tm || !w_ih || !w_hh || !gates || !c_tm || !h_tm || !dgates || !dw_ih || !dw_hh || !db_ih || !workspace)
    return SV_EARG;
  if (!lstm_dims_ok(T, B, F, H)) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  float* dcf0 = workspace;
  float* dcf1 = workspace + BH;
  float* gws = workspace + 2 * BH;
  gws = (float*)(((uintptr_t)gws + 255) & ~uintptr_t(255));
  constexpr int LDS_MAIN = 4 * 2 * SV_BK * (TileLd<true, BWD_BM>::value + TileLd<false, BWD_U>::value);
  constexpr int LDS_RED = 4 * BWD_BM * (BWD_U + 1);
  constexpr int LDS = (LDS_MAIN > LDS_RED ? LDS_MAIN : LDS_RED) * sizeof(float);
  const dim3 grid((H + BWD_U - 1) / BWD_U, (B + BWD_BM - 1) / BWD_BM);
  for (int t = T - 1; t >= 0; --t) {
    const float* up = nullptr;
    if (dh_up) up = dh_up_full ? dh_up + t * BH : (t == T - 1 ? dh_up : nullptr);
    float* dcf_out = (t & 1) ? dcf1 : dcf0;
    const float* dcf_in = (t == T - 1) ? nullptr : ((t & 1) ? dcf0 : dcf1);
    hipLaunchKernelGGL(lstm_step_bwd_kernel, grid, dim3(256), LDS, stream, t == T - 1 ? nullptr : dgates + (t + 1) * BG,
                       w_hh, up, dcf_in, gates + t * BG, c_tm + t * BH, t ? c_tm + (t - 1) * BH : nullptr,
                       dgates + t * BG, dcf_out, B, H);
    SV_LAUNCH_CHECK();
  }
  const int TB = T * B;
  // dW_hh = sum_t dG_t^T h_{t-1}   (A = dG as [K=TB][M=4H], B = h_tm[0..T-1] as [K=TB][N=H])
  int rc = sv_gemm_f32(0, 0, 4 * H, H, TB, dgates, 4L * H, h_tm, H, dw_hh, H, nullptr, nullptr, 0.f, gws, stream);
  if (rc) return rc;
  // dW_ih = sum_t dG_t^T x_t
  rc = sv_gemm_f32(0, 0, 4 * H, F, TB, dgates, 4L * H, x_tm, F, dw_ih, F, nullptr, nullptr, 0.f, gws, stream);
  if (rc) return rc;
  // db_ih = db_hh = sum_{t,b} dG
  rc = colsum(dgates, TB, 4 * H, db_ih, db_hh, gws, stream);
  if (rc) return rc;
  // dx = dG W_ih  (A = dG [TB, 4H] k-contig, B = W_ih as [K=4H][N=F] n-contig)
  if (dx_tm) {
    rc = sv_gemm_f32(1, 0, TB, F, 4 * H, dgates, 4L * H, w_ih, F, dx_tm, F, nullptr, nullptr, 0.f, gws, stream);
    if (rc) return rc;
  }
  return SV_OK;
}
