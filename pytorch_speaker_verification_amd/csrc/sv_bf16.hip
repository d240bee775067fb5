// bf16-operand variant of the LSTM stack (BASELINE config c3: "gate GEMMs on MFMA", mixed
// precision).  GEMM operands (weights, h, dgates) are bf16 and feed v_mfma_f32_32x32x16_bf16
// with fp32 accumulation; cell state, activations, biases, gradients, the projection, the
// GE2E loss and the optimizer stay fp32.  Same algorithm, layouts and epilogues
// as sv_lstm.hip; transposed layouts use column blocks of Bp = B rounded up to 8 so every
// bf16 row stays 16-byte aligned.
#include <vector>
#include <algorithm>
#include "sv_common.h"
#include "sv_gemm.h"
#include "../../include/sv_ge2e.h"
#include "sv_bf16.h"
#include "sv_gemm256.h"
#include "sv_persist_dev.h"


// ============================================================================
// GEMM: C[M,N] fp32 = A[M,K] . B[N,K]^T (bf16, both k-contiguous) (+bias) / split-K slabs
// ============================================================================
enum { BEPI_STORE = 0, BEPI_SLAB = 1, BEPI_STORE_BF16 = 2 };

template <int BM, int BN, int EPI>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16_t* __restrict__ A, long lda,
                                                        const bf16_t* __restrict__ B, long ldb, void* __restrict__ Cv,
                                                        long ldc, long slab, int M, int N, int K, int kchunk,
                                                        const float* __restrict__ bias0,
                                                        const float* __restrict__ bias1, float beta) {
  extern __shared__ __attribute__((aligned(16))) bf16_t ldsb[];
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
  gemm_mainloop_bf<BM, BN, 256, BBK, TM, TN>(A, lda, RowMapLinear{tm * BM, M}, B, ldb, RowMapLinear{tn * BN, N}, kbeg,
                                             kend, ldsb, tid, wm0, wn0, acc);
  float* Cz = reinterpret_cast<float*>(Cv) + (EPI == BEPI_SLAB ? (long)blockIdx.y * slab : 0);
  // bias sums of the lane's columns, loaded before any store (a load between stores waits for
  // every store issued before it)
  float bsum[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = tn * BN + wn0 + 32 * j + (lane & 31);
    float badd = 0.f;
    if (EPI != BEPI_SLAB && col < N) {
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
        if (EPI == BEPI_STORE_BF16) {
          reinterpret_cast<bf16_t*>(Cv)[(long)row * ldc + col] = to_bf(v + badd);
          continue;
        }
        float* dst = Cz + (long)row * ldc + col;
        if (EPI == BEPI_STORE) {
          v += badd;
          if (beta != 0.f) v += beta * *dst;
        }
        *dst = v;
      }
    }
}

__global__ void slab_reduce_bf_kernel(const float* __restrict__ slab, int nz, long zstride, float* __restrict__ out,
                                      long ldc, int M, int N, float beta, const float* __restrict__ bias0,
                                      const float* __restrict__ bias1, bf16_t* __restrict__ outb = nullptr,
                                      float* __restrict__ out2 = nullptr, long ldc2 = 0, int n1 = 0) {
  const long total = (long)M * N;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = (int)(e / N), col = (int)(e % N);
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += slab[z * zstride + e];
    if (out2 && col >= n1) {  // fused pair: columns past n1 belong to the second product
      out2[(long)row * ldc2 + col - n1] = s;
      continue;
    }
    if (bias0) s += bias0[col];
    if (bias1) s += bias1[col];
    if (outb) {  // bf16 output (beta unused)
      outb[(long)row * ldc + col] = to_bf(s);
      continue;
    }
    float* dst = out + (long)row * ldc + col;
    *dst = (beta != 0.f ? beta * *dst : 0.f) + s;
  }
}

// up to 8 casts / transpose-casts in ONE launch (the per-step weight copies of the bf16 path: at
// the c4 rank shape each of the 13 separate launches took ~5 us for ~1 us of traffic); the
// single-matrix entry points (sv_cast_bf16, sv_transpose_cast_bf16) are batches of one
struct CastBatch {
  const float* x[8];
  bf16_t* y[8];
  long start[9];  // element prefix sums
  int n;
};
// VEC: start[] counts groups of 4 elements (every count % 4 == 0, every pointer 16-B aligned):
// one float4 load and one 8-B store per thread-iteration
template <bool VEC>
__global__ void cast_bf16_batch_kernel(const CastBatch cb) {
  const long total = cb.start[cb.n];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int b = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) b += (k < cb.n && i >= cb.start[k]) ? 1 : 0;
    const long j = i - cb.start[b];
    if constexpr (VEC) {
      const float4 v = reinterpret_cast<const float4*>(cb.x[b])[j];
      reinterpret_cast<uint2*>(cb.y[b])[j] = pack_bf4(v.x, v.y, v.z, v.w);
    } else {
      cb.y[b][j] = to_bf(cb.x[b][j]);
    }
  }
}
struct TCastBatch {
  const float* src[8];
  bf16_t* dst[8];   // transposed copy (null: none)
  bf16_t* dstr[8];  // row-major copy, row stride C (null: none; ABI v10, sv_lstm_weights_bf16)
  long lds[8], ldd[8];
  int R[8], C[8], tx[8];  // column tiles per matrix
  int tile0[9];           // 64 x 64 tile prefix sums
  int n;
  unsigned vec;           // bit b: matrix b takes the 16-B paths (lds % 4, ldd % 8, aligned bases)
};
// the frames' part of the bf16 stack's input preparation (sv_frames_to_bf16 / sv_lstm_prep_bf16):
// frames x [B,T,F] fp32 -> x_bf [T,B,F] and, when xT is given, xT [F][T Bp] with column t Bp + b =
// x[b,t,:] (padding columns b in [B, Bp) zero) -- layer 0's dW_ih operand.  Workgroup (t, 64 rows
// b): the tile goes through LDS so both stores coalesce.
struct FramesArgs {
  const float* x;
  bf16_t *x_bf, *xT;
  int B, T, F, Bp, nbx;  // nbx: 64-row blocks per timestep
};
__device__ __forceinline__ void frames_tile(const FramesArgs& fa, int bx, int t, float (*tile)[65]) {
  const int b0 = bx * 64, tid = threadIdx.x, B = fa.B, T = fa.T, F = fa.F, Bp = fa.Bp;
  // 16 predicated loads per thread, all in flight before the first LDS write (a rolled loop
  // waited for each load on its own); thread -> (row tid / 64 + 4 i, column tid % 64)
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int b = (tid >> 6) + 4 * i, f = tid & 63;
    v[i] = (f < F && b0 + b < B) ? fa.x[((long)(b0 + b) * T + t) * F + f] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) tile[(tid >> 6) + 4 * i][tid & 63] = v[i];
  __syncthreads();
  for (int i = tid; i < 64 * F; i += 256) {
    const int b = i / F, f = i % F;
    if (b0 + b < B) fa.x_bf[((long)t * B + b0 + b) * F + f] = to_bf(tile[b][f]);
  }
  if (fa.xT)
    for (int i = tid; i < 64 * F; i += 256) {
      const int f = i / 64, b = i % 64;
      if (b0 + b < Bp) fa.xT[(long)f * T * Bp + (long)t * Bp + b0 + b] = to_bf(tile[b][f]);
    }
}

// 64 x 64 tiles: float4 loads along a source row (16 threads per row, 16 rows per pass) and 16-B
// bf16 stores along a destination row (8 threads per row, 32 rows per pass) where the matrix's
// leading dimensions and base pointers allow (tb.vec bit b), element-wise at the edges.
// The first nfr workgroups (fa.x given): the frames' part, beside the tiles in the same launch --
// dispatched first, so that these latency-bound workgroups overlap the tiles instead of forming
// the launch's tail (placed after the tiles, the launch took the two kernels' sum, 27 us at c4)
__global__ __launch_bounds__(256) void transpose_cast_batch_kernel(const TCastBatch tb, const FramesArgs fa, int nfr) {
  __shared__ float tile[64][65];
  if ((int)blockIdx.x < nfr) {
    frames_tile(fa, blockIdx.x % fa.nbx, blockIdx.x / fa.nbx, tile);
    return;
  }
  const int blk = blockIdx.x - nfr;
  int b = 0;
#pragma unroll
  for (int k = 1; k < 8; ++k) b += (k < tb.n && blk >= tb.tile0[k]) ? 1 : 0;
  const int t = blk - tb.tile0[b];
  const int R = tb.R[b], C = tb.C[b];
  const int c0 = (t % tb.tx[b]) * 64, r0 = (t / tb.tx[b]) * 64;
  const bool vec = (tb.vec >> b) & 1;
  const float* src = tb.src[b];
  {
    const int lc = (threadIdx.x & 15) * 4, lr = threadIdx.x >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + lr + 16 * i, c = c0 + lc;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        if (vec && c + 3 < C) {
          const float4 q = *reinterpret_cast<const float4*>(src + (long)r * tb.lds[b] + c);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < C) v[e] = src[(long)r * tb.lds[b] + c + e];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[lr + 16 * i][lc + e] = v[e];
      if (tb.dstr[b] && r < R) {  // the row-major copy straight from the registers
        bf16_t* d = tb.dstr[b] + (long)r * C + c;
        if (vec && c + 3 < C) {
          *reinterpret_cast<uint2*>(d) = pack_bf4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < C) d[e] = to_bf(v[e]);
        }
      }
    }
  }
  bf16_t* dst = tb.dst[b];
  if (!dst) return;  // uniform per workgroup: no barrier skipped by part of it
  __syncthreads();
  const int lr8 = (threadIdx.x & 7) * 8, lcr = threadIdx.x >> 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int cc = lcr + 32 * i, c = c0 + cc, r = r0 + lr8;
    if (c >= C) continue;
    bf16_t* d = dst + (long)c * tb.ldd[b] + r;
    if (vec && r + 7 < R) {
      const uint2 lo = pack_bf4(tile[lr8][cc], tile[lr8 + 1][cc], tile[lr8 + 2][cc], tile[lr8 + 3][cc]);
      const uint2 hi = pack_bf4(tile[lr8 + 4][cc], tile[lr8 + 5][cc], tile[lr8 + 6][cc], tile[lr8 + 7][cc]);
      *reinterpret_cast<uint4*>(d) = uint4{lo.x, lo.y, hi.x, hi.y};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (r + e < R) d[e] = to_bf(tile[lr8 + e][cc]);
    }
  }
}

// row sums of a bf16 matrix, fp32 accumulation, one block per row, fixed order
__global__ __launch_bounds__(256) void rowsum_bf16_kernel(const bf16_t* __restrict__ X, long ld, int C,
                                                          float* __restrict__ out0, float* __restrict__ out1) {
  __shared__ float red[4];
  const bf16_t* x = X + (long)blockIdx.x * ld;
  float s = 0.f;
  const int C8 = C / 8;
  for (int c = threadIdx.x; c < C8; c += 256) {
    const bf16x8_t v = reinterpret_cast<const bf16x8_t*>(x)[c];
    float p = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) p += (float)v[j];
    s += p;
  }
  for (int c = C8 * 8 + threadIdx.x; c < C; c += 256) s += (float)*reinterpret_cast<const __bf16*>(x + c);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = (red[0] + red[1]) + (red[2] + red[3]);
    out0[blockIdx.x] = t;
    if (out1) out1[blockIdx.x] = t;
  }
}

// ============================================================================
// recurrent steps (same decomposition as the fp32 v2 kernels: 64 rows x 32 units, 8 waves)
// ============================================================================

template <int SC>
__global__ __launch_bounds__(512) void lstm_step_fwd_bf16_kernel(
    const bf16_t* __restrict__ hprev_bf, const bf16_t* __restrict__ whh_bf, bf16_t* __restrict__ gates,
    const float* __restrict__ cprev, float* __restrict__ cout, float* __restrict__ hout, bf16_t* __restrict__ hout_bf,
    bf16_t* __restrict__ hT, long ldhT, int t, int Bp, int B, int H) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ldsb = reinterpret_cast<bf16_t*>(smem);
  constexpr int BN = 4 * BF_U, LDP = BN + 4, LDH = BF_BM + 1;
  constexpr int PER = BF_BM * BF_U / 512;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * BF_U, b0 = blockIdx.y * BF_BM;
  const int wm0 = (w >> 2) * 32, wn0 = (w & 3) * 32;
  const long G = 4L * H;
  float xg[PER][4], cpv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
    const int gb = b0 + b, gj = j0 + u;
    const bool ok = gb < B && gj < H;
    const bf16_t* gp = gates + (long)gb * G + gj;
#pragma unroll
    for (int q = 0; q < 4; ++q) xg[k][q] = ok ? from_bf(gp[q * H]) : 0.f;
    cpv[k] = (ok && cprev) ? cprev[(long)gb * H + gj] : 0.f;
  }
  f32x16 acc[1][1];
  zero_acc(acc);
  if (hprev_bf)
    gemm_mainloop_step<BF_BM, BN, 512, SC, 1, 1>(hprev_bf + (long)b0 * H, H, RowMapLinear{0, B - b0}, whh_bf, H,
                                                 RowMapGates<BF_U>{j0, H}, 0, H, ldsb, tid, wm0, wn0, acc);
  float* pre = reinterpret_cast<float*>(smem);
  float* hs = pre + BF_BM * LDP;
#pragma unroll
  for (int r = 0; r < 16; ++r) pre[(wm0 + acc_row(r, lane)) * LDP + wn0 + (lane & 31)] = acc[0][0][r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    bf16_t* gp = gates + (long)gb * G + gj;
    const float* pr = pre + b * LDP + u;
    const float pv[4] = {pr[0], pr[BF_U], pr[2 * BF_U], pr[3 * BF_U]};
    float av[4], h;
    const float c = lstm_cell_fwd(pv, xg[k], cpv[k], av, h);
    gp[0] = to_bf(av[0]);
    gp[H] = to_bf(av[1]);
    gp[2 * H] = to_bf(av[2]);
    gp[3 * H] = to_bf(av[3]);
    cout[(long)gb * H + gj] = c;
    hout[(long)gb * H + gj] = h;
    hout_bf[(long)gb * H + gj] = to_bf(h);
    hs[u * LDH + b] = h;
  }
  if (!hT) return;
  __syncthreads();
  for (int e = tid; e < BF_BM * BF_U; e += 512) {
    const int u = e / BF_BM, b = e % BF_BM;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    bf16_t* row = hT + (long)gj * ldhT;
    row[(long)(t + 1) * Bp + gb] = to_bf(hs[u * LDH + b]);
    if (t == 0) row[gb] = 0;
  }
}

template <int SC>
__global__ __launch_bounds__(512) void lstm_step_bwd_bf16_kernel(
    const bf16_t* __restrict__ dgnext, const bf16_t* __restrict__ whhT, const float* __restrict__ dhup,
    const float* __restrict__ dcf_next, const bf16_t* __restrict__ acts, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, bf16_t* __restrict__ dg, float* __restrict__ dcf, bf16_t* __restrict__ dgT,
    long lddgT, int t, int Bp, int B, int H) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ldsb = reinterpret_cast<bf16_t*>(smem);
  constexpr int GBUF = 2 * (BF_BM + BF_U) * (BBK + 8);
  constexpr int LDR = BF_U + 1;
  constexpr int LDT = BF_BM + 1;
  constexpr int PER = BF_BM * BF_U / 512;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int gate = w >> 1, gt = tid & 127;
  const int j0 = blockIdx.x * BF_U, b0 = blockIdx.y * BF_BM;
  const long G = 4L * H;
  float av[PER][4], cv[PER], cpv[PER], dcfv[PER], upv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
    const int gb = b0 + b, gj = j0 + u;
    const bool ok = gb < B && gj < H;
    const long hi = (long)gb * H + gj;
    const bf16_t* ap = acts + (long)gb * G + gj;
#pragma unroll
    for (int q = 0; q < 4; ++q) av[k][q] = ok ? from_bf(ap[q * H]) : 0.f;
    cv[k] = ok ? c_t[hi] : 0.f;
    cpv[k] = (ok && c_prev) ? c_prev[hi] : 0.f;
    dcfv[k] = (ok && dcf_next) ? dcf_next[hi] : 0.f;
    upv[k] = (ok && dhup) ? dhup[hi] : 0.f;
  }
  f32x16 acc[1][1];
  zero_acc(acc);
  if (dgnext)
    gemm_mainloop_step<BF_BM, BF_U, 128, SC, 1, 1>(dgnext + (long)b0 * G, G, RowMapLinear{0, B - b0}, whhT, G,
                                                  RowMapLinear{j0, H}, gate * H, (gate + 1) * H, ldsb + gate * GBUF,
                                                  gt, (w & 1) * 32, 0, acc);
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4][64][LDR]
  float* gTs = red + 4 * BF_BM * LDR;           // [4*32][LDT]
#pragma unroll
  for (int r = 0; r < 16; ++r)
    red[(gate * BF_BM + (w & 1) * 32 + acc_row(r, lane)) * LDR + (lane & 31)] = acc[0][0][r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    const long hi = (long)gb * H + gj;
    float dh = red[(0 * BF_BM + b) * LDR + u];
    dh += red[(1 * BF_BM + b) * LDR + u];
    dh += red[(2 * BF_BM + b) * LDR + u];
    dh += red[(3 * BF_BM + b) * LDR + u];
    dh += upv[k];
    float dd[4];
    dcf[hi] = lstm_cell_bwd(dh, av[k][0], av[k][1], av[k][2], av[k][3], cv[k], cpv[k], dcfv[k], dd);
    const float d0 = dd[0], d1 = dd[1], d2 = dd[2], d3 = dd[3];
    bf16_t* dp = dg + (long)gb * G + gj;
    dp[0] = to_bf(d0);
    dp[H] = to_bf(d1);
    dp[2 * H] = to_bf(d2);
    dp[3 * H] = to_bf(d3);
    gTs[(0 * BF_U + u) * LDT + b] = d0;
    gTs[(1 * BF_U + u) * LDT + b] = d1;
    gTs[(2 * BF_U + u) * LDT + b] = d2;
    gTs[(3 * BF_U + u) * LDT + b] = d3;
  }
  if (!dgT) return;
  __syncthreads();
  for (int e = tid; e < 4 * BF_U * BF_BM; e += 512) {
    const int gu = e / BF_BM, b = e % BF_BM;
    const int gte = gu / BF_U, u = gu % BF_U;
    const int gb = b0 + b, gj = j0 + u;
    if (gb >= B || gj >= H) continue;
    dgT[((long)gte * H + gj) * lddgT + (long)t * Bp + gb] = to_bf(gTs[gu * LDT + b]);
  }
}

// ============================================================================
// host side
// ============================================================================
namespace {

struct BPlan {
  int bm, bn, splitk, kchunk;
};

// 256 x 256 kernels (sv_gemm256.h) for shapes they tile exactly
bool gemm256_ok(int M, int N, int K) { return M % G256_BM == 0 && N % G256_BM == 0 && K % G256_BK == 0; }

// the 256 x 256 tile's schedule: the 8-phase kernel (gemm_bf16_8q_kernel) where its 16-B
// epilogue stores are aligned (C rows, biases), else the two-stage gemm_bf16_256_kernel
bool g8_ok(const void* C, long ldc, const float* bias0, const float* bias1) {
  return !((((uintptr_t)C | (uintptr_t)bias0 | (uintptr_t)bias1) & 15) || ldc % 4);
}

// the 8-phase kernel with two LDS-DMA fills per phase.  Measured against one or two fill phases
// per k-tile (c3 shapes, us): dW 414 vs 445-446, dx 440 vs 471-480, K1 (bf16 out) 615 vs 626.
template <int EPI, int AF>
void launch_g8(dim3 grid, hipStream_t stream, const bf16_t* A, long lda, const bf16_t* B, long ldb, void* C, long ldc,
               long slab, int M, int N, int K, int kchunk, const float* bias0, const float* bias1, float beta,
               G256AFrag af = G256AFrag{}) {
  hipLaunchKernelGGL((gemm_bf16_8q_kernel<EPI, AF>), grid, dim3(512), G256_LDS, stream, A, lda, B, ldb, C, ldc, slab,
                     M, N, K, kchunk, bias0, bias1, beta, af);
}

template <int EPI, int AF>
void launch_g256(bool g8, dim3 grid, hipStream_t stream, const bf16_t* A, long lda, const bf16_t* B, long ldb, void* C,
                 long ldc, long slab, int M, int N, int K, int kchunk, const float* bias0, const float* bias1,
                 float beta, G256AFrag af = G256AFrag{}) {
  if (g8)
    launch_g8<EPI, AF>(grid, stream, A, lda, B, ldb, C, ldc, slab, M, N, K, kchunk, bias0, bias1, beta, af);
  else
    hipLaunchKernelGGL((gemm_bf16_256_kernel<EPI, AF>), grid, dim3(512), G256_LDS, stream, A, lda, B, ldb, (float*)C,
                       ldc, slab, M, N, K, kchunk, bias0, bias1, beta, af);
}

BPlan plan_bf16(int M, int N, int K) {
  BPlan p;
  if (gemm256_ok(M, N, K)) {  // one workgroup per CU: split K only to fill the 256 CUs
    // ... and only for the long weight-gradient reductions (K = T B): a dx GEMM (K = 4H) then sums
    // K in one order whether it runs per 32-step chunk (per-step schedule) or over all T (the
    // persistent schedule's fragment-order form), so the two schedules stay bit-identical
    const long tiles = (long)(M / G256_BM) * (N / G256_BM);
    int sk = 1;
    if (tiles < 256 && K >= 8192) sk = (int)std::max(1L, std::min(256L / tiles, (long)K / 1024));
    p.bm = p.bn = G256_BM;
    p.kchunk = ((K + sk - 1) / sk + G256_BK - 1) / G256_BK * G256_BK;
    p.splitk = (K + p.kchunk - 1) / p.kchunk;
    return p;
  }
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  const bool small = t128 < 128;
  p.bm = p.bn = small ? 64 : 128;
  const long tiles = (long)((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
  const long slots = small ? 1024 : 512;
  int sk = 1;
  if (tiles < slots) {  // the wave-quantised split-K model of plan_gemm (sv_lstm.hip), at ~600 TF/s
    const double rate = 600e12 / (double)slots, hbm = 5e12;
    const int kmax = std::max(1, std::min(32, K / 1024));
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
  p.kchunk = ((K + sk - 1) / sk + BBK - 1) / BBK * BBK;
  p.splitk = (K + p.kchunk - 1) / p.kchunk;
  return p;
}

template <int BM, int BN, int EPI>
void launch_bf(const bf16_t* A, long lda, const bf16_t* B, long ldb, void* C, long ldc, long slab, int M, int N, int K,
               int splitk, int kchunk, const float* b0, const float* b1, float beta, hipStream_t s) {
  constexpr int LDS = 2 * (BM + BN) * (BBK + 8) * (int)sizeof(bf16_t);
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, EPI>), dim3(tiles, splitk), dim3(256), LDS, s, A, lda, B, ldb, C, ldc,
                     slab, M, N, K, kchunk, b0, b1, beta);
}

constexpr int BFWD_LDS_MAIN = 2 * (BF_BM + 4 * BF_U) * (BBK + 8) * 2;
constexpr int BFWD_LDS_EPI = (BF_BM * (4 * BF_U + 4) + BF_U * (BF_BM + 1)) * 4;
constexpr int BFWD_LDS = BFWD_LDS_MAIN > BFWD_LDS_EPI ? BFWD_LDS_MAIN : BFWD_LDS_EPI;
constexpr int BBWD_LDS_MAIN = 4 * 2 * (BF_BM + BF_U) * (BBK + 8) * 2;
constexpr int BBWD_LDS_EPI = (4 * BF_BM * (BF_U + 1) + 4 * BF_U * (BF_BM + 1)) * 4;
constexpr int BBWD_LDS = BBWD_LDS_MAIN > BBWD_LDS_EPI ? BBWD_LDS_MAIN : BBWD_LDS_EPI;

// per-step forward kernel: register prefetch in super-chunks of 3 k-tiles (measured against 4, 6,
// 12 and rolling prefetch depths 4 / 6 at c3: none faster)
void launch_fwd_bf16(dim3 grid, hipStream_t s, const bf16_t* hp, const bf16_t* whh, bf16_t* g, const float* cp,
                     float* c, float* h, bf16_t* hb, bf16_t* hT, long ldhT, int t, int Bp, int B, int H) {
  hipLaunchKernelGGL(lstm_step_fwd_bf16_kernel<3>, grid, dim3(512), BFWD_LDS, s, hp, whh, g, cp, c, h, hb, hT, ldhT,
                     t, Bp, B, H);
}

// bf16 stack schedule (the `schedule` flags of sv_lstm_stack_{fwd,bwd}_bf16, include/sv_ge2e.h):
// persistent recurrences (one launch per layer, W_hh held in registers, sv_persist.hip) at
// H = 768 (measured c3 21.5 vs 22.2 ms per-step) or wherever they fit with SV_SCHED_PERSIST;
// per-step launches, layer-pipelined, with SV_SCHED_PER_STEP (bit-identical results).
bool sched_persist(int schedule, int H) {
  return !(schedule & SV_SCHED_PER_STEP) && ((schedule & SV_SCHED_PERSIST) || H == 768);
}
// the layer wavefronts (every layer in one launch, sv_wave.hip / sv_persist3.hip) where all
// layers' grids fit co-resident, unless SV_SCHED_PER_LAYER (bf16-level different sums)
bool sched_wave(int schedule, int H) { return sched_persist(schedule, H) && !(schedule & SV_SCHED_PER_LAYER); }

// per-step backward kernel: register prefetch in super-chunks of 6 k-tiles (measured against
// 2, 3 and rolling depths 3 / 4 / 6 at c3)
void launch_bwd_bf16(dim3 grid, hipStream_t s, const bf16_t* dgn, const bf16_t* whhT, const float* up,
                     const float* dcfi, const bf16_t* acts, const float* ct, const float* cp, bf16_t* dg, float* dcfo,
                     bf16_t* dgT, long lddgT, int t, int Bp, int B, int H) {
  hipLaunchKernelGGL(lstm_step_bwd_bf16_kernel<6>, grid, dim3(512), BBWD_LDS, s, dgn, whhT, up, dcfi, acts, ct, cp,
                     dg, dcfo, dgT, lddgT, t, Bp, B, H);
}

// ---- the layer wavefront's weight gradients as whole-K tiles in one launch (c4 rank) ----
// After the wavefront every layer's dG^T is final.  The per-layer split-K plan (c4 rank: K = T Bp =
// 12800 in 7 slabs of 29 k-tiles; 504 workgroups per dual GEMM, two rounds) writes 129 MB of fp32
// slabs per layer and reads them back in a reduce launch; the three layers' 256 x 256 tiles
// together (72 + 72 dual, 36 for layer 0's dW_hh) fit the CUs as ONE round of whole-K tiles, each
// stored straight into dW_hh / dW_ih.  Another fp32 summation order than the slabs' (one
// accumulator over the k-tiles): agreement with the per-layer schedule at fp32 level.
// Split form (S > 0): the CUs the tiles leave free (nsw workgroups, a multiple of 8, blocks
// 0 .. nsw - 1) compute every tile's first S k-tiles (tiles b, b + nsw, ...) and store the fp32
// partial (sc1, per-thread order) and a flag; the tile's own workgroup (block nsw + position)
// computes k-tiles S .. K/64 - 1, waits for the flag, adds the partial (its own sum first: one
// fixed order) and stores C.  The waiters are dispatched after every workgroup they wait for.
struct G8FLayer {
  const bf16_t* A;    // dG^T [4H][T Bp]
  const bf16_t* B;    // h^T (time-shifted)
  const bf16_t* B2;   // x^T (dual: columns past n1), or null
  float* C1;          // dW_hh
  float* C2;          // dW_ih (dual)
  long lda, ldb, ldb2, ldc1, ldc2;
  int N, n1, tiles;
  int f2;             // dW_ih columns (rows of x^T): layer 0's F = 40 in one partial 256-wide tile
};
struct G8Full {
  G8FLayer lay[WB_L];
  int K;             // T Bp
  int nsw, S;        // split form: first-piece workgroups and k-tiles (S = 0: whole-K tiles only)
  float* part;       // [P][256 x 256] fp32 first-piece partials
  unsigned* flag;    // [P], zero before the launch
  unsigned* status;  // the sync block's status word
  unsigned limit;
  DbFin fin;         // a deferred bias finalize: workgroups past the tiles (dbfin_blocks(fin, 512))
};
__global__ __launch_bounds__(512, 1) void gemm_bf16_8qf_kernel(const G8Full q) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const G8FLayer& L2 = q.lay[2];
  const G8FLayer& L1 = q.lay[1];
  const G8FLayer& L0 = q.lay[0];
  const int P = L2.tiles + L1.tiles + L0.tiles;
  if ((int)blockIdx.x >= q.nsw + P) {  // the deferred bias finalize (the highest blocks: nobody waits on them)
    dbfin_run(q.fin, blockIdx.x - q.nsw - P);
    return;
  }
  // tile r (top layer first) -> its operands (field-wise selects: a dynamic index into the
  // kernel-argument struct would copy it to scratch)
  auto run = [&](int r, int kbeg, int nk, g8_f32x4 (&acc)[8][4], int& l, int& tm, int& tn) {
    l = r < L2.tiles ? 2 : r < L2.tiles + L1.tiles ? 1 : 0;
    const int tile = l == 2 ? r : l == 1 ? r - L2.tiles : r - L2.tiles - L1.tiles;
    const bf16_t* A = l == 2 ? L2.A : l == 1 ? L1.A : L0.A;
    const bf16_t* Bm = l == 2 ? L2.B : l == 1 ? L1.B : L0.B;
    const bf16_t* B2 = l == 2 ? L2.B2 : l == 1 ? L1.B2 : L0.B2;
    const long lda = l == 2 ? L2.lda : l == 1 ? L1.lda : L0.lda;
    const long ldb = l == 2 ? L2.ldb : l == 1 ? L1.ldb : L0.ldb;
    const long ldb2 = l == 2 ? L2.ldb2 : l == 1 ? L1.ldb2 : L0.ldb2;
    const int N = l == 2 ? L2.N : l == 1 ? L1.N : L0.N;
    const int n1 = l == 2 ? L2.n1 : l == 1 ? L1.n1 : L0.n1;
    const int f2 = l == 2 ? L2.f2 : l == 1 ? L1.f2 : L0.f2;
    const int tiles_n = N / G256_BM;
    tn = tile % tiles_n;
    tm = tile / tiles_n;
    g8_tile<0>(A, lda, Bm, ldb, G256AFrag{}, G256Dual{B2, ldb2, n1, f2}, tm, tn, kbeg, nk, smem, acc);
  };
  g8_f32x4 acc[8][4];
  int l, tm, tn;
  if ((int)blockIdx.x < q.nsw) {  // first pieces
    for (int j = blockIdx.x; j < P; j += q.nsw) {
      run(j, 0, q.S, acc, l, tm, tn);
      const __amdgpu_buffer_rsrc_t rp = sv_rsrc(q.part + (long)j * G256_BM * G256_BM, G256_BM * G256_BM * 4u);
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const g8_f32x4 v = acc[i >> 2][i & 3];
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4_t{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])}, rp,
            (unsigned)(i * 512 + tid) * 16u, 0, 16 /* sc1 */);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(q.flag + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // position after xcd_remap (nsw % 8 == 0, so blocks nsw + i keep i's XCD): each XCD owns a
  // contiguous run, so a row tile's column tiles (the same dG^T rows) share an L2
  const int r = xcd_remap((int)blockIdx.x - q.nsw, P);
  run(r, q.S * G256_BK, q.K / G256_BK - q.S, acc, l, tm, tn);
  if (q.S > 0) {
    if (tid == 0) persist_wait(q.flag + r, 1u, q.status, q.limit, 2u);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rp = sv_rsrc(q.part + (long)r * G256_BM * G256_BM, G256_BM * G256_BM * 4u);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rp, (unsigned)(i * 512 + tid) * 16u, 0, 16 /* sc1 */);
      acc[i >> 2][i & 3] += g8_f32x4{__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]),
                                     __uint_as_float(x[3])};
    }
  }
  float* C1 = l == 2 ? L2.C1 : l == 1 ? L1.C1 : L0.C1;
  float* C2 = l == 2 ? L2.C2 : l == 1 ? L1.C2 : L0.C2;
  const long ldc1 = l == 2 ? L2.ldc1 : l == 1 ? L1.ldc1 : L0.ldc1;
  const long ldc2 = l == 2 ? L2.ldc2 : l == 1 ? L1.ldc2 : L0.ldc2;
  const int n1 = l == 2 ? L2.n1 : l == 1 ? L1.n1 : L0.n1;
  const int f2 = l == 2 ? L2.f2 : l == 1 ? L1.f2 : L0.f2;
  const bool second = tn * G256_BM >= n1;  // n1 % 256 == 0 (host): a tile is all C1 or all C2
  g8_epilogue<G8_STORE>(acc, second ? C2 : C1, second ? ldc2 : ldc1, 0, tm, second ? tn - n1 / G256_BM : tn, wr, wc,
                        lane, nullptr, nullptr, 0.f, second && f2 > 0 ? f2 : 1 << 30);
}

}  // namespace

extern "C" size_t sv_gemm_bf16_workspace(int M, int N, int K);
extern "C" int sv_gemm_bf16(int M, int N, int K, const bf16_t* A, long lda, const bf16_t* B, long ldb, float* C,
                            long ldc, const float* bias0, const float* bias1, float beta, float* workspace,
                            hipStream_t stream);
// C1 = A . B1^T and C2 = A . B2^T (fp32 out, no bias / beta) in one launch over the shared A:
// the split-K plan of sv_gemm_bf16(M, N1, K), so each product sums exactly as the single GEMM
// does (bit-identical); falls back to two calls where the fused form does not apply.
// workspace: sv_gemm_bf16_dual_workspace bytes
size_t sv_gemm_bf16_dual_workspace(int M, int N1, int N2, int K) {
  const BPlan p = plan_bf16(M, N1, K);
  size_t fused = p.splitk > 1 ? (size_t)p.splitk * M * (N1 + N2) * sizeof(float) : 0;
  return std::max(fused, std::max(sv_gemm_bf16_workspace(M, N1, K), sv_gemm_bf16_workspace(M, N2, K)));
}
int sv_gemm_bf16_dual(int M, int N1, int N2, int K, const bf16_t* A, long lda, const bf16_t* B1, long ldb1, float* C1,
                      long ldc1, const bf16_t* B2, long ldb2, float* C2, long ldc2, float* workspace,
                      hipStream_t stream) {
  const BPlan p = plan_bf16(M, N1, K);
  const bool fused = p.bm == G256_BM && p.splitk > 1 && gemm256_ok(M, N1 + N2, K) && N1 % G256_BM == 0 &&
                     N2 % G256_BM == 0 && workspace && g8_ok(workspace, N1 + N2, nullptr, nullptr) &&
                     ldb1 % 8 == 0 && ldb2 % 8 == 0 && lda % 8 == 0 && !(((uintptr_t)A | (uintptr_t)B1 | (uintptr_t)B2) & 15);
  if (!fused) {
    int rc = sv_gemm_bf16(M, N1, K, A, lda, B1, ldb1, C1, ldc1, nullptr, nullptr, 0.f, workspace, stream);
    if (rc) return rc;
    return sv_gemm_bf16(M, N2, K, A, lda, B2, ldb2, C2, ldc2, nullptr, nullptr, 0.f, workspace, stream);
  }
  const int N = N1 + N2;
  const int tiles = (M / G256_BM) * (N / G256_BM);
  const long slab = (long)M * N;
  hipLaunchKernelGGL((gemm_bf16_8q_kernel<G8_SLAB, 0>), dim3(tiles, p.splitk), dim3(512), G256_LDS, stream, A, lda, B1,
                     ldb1, (void*)workspace, (long)N, slab, M, N, K, p.kchunk, nullptr, nullptr, 0.f, G256AFrag{},
                     G256Dual{B2, ldb2, N1});
  SV_LAUNCH_CHECK();
  const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
  hipLaunchKernelGGL(slab_reduce_bf_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C1, ldc1, M, N,
                     0.f, nullptr, nullptr, nullptr, C2, ldc2, N1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// ---- narrow bf16 NT GEMM (N <= 48): layer 0's dW_ih = dG^T x (M = 4H, N = F = 40, K = T B) ----
// The 64 x 64 tiles padded N = 40 to 64 and streamed dG^T (629 MB at c3) at 4.6 TB/s (138 us).  The
// fp32 narrow kernel's layout (sv_lstm.hip) in bf16: a workgroup is 128 rows x 48 columns over a K
// chunk, v_mfma_f32_16x16x32_bf16 (B first: a lane's 4 accumulators are 4 consecutive C columns),
// each wave 32 rows (2 x 3 blocks); LDS images [rows][64 k] (128 B) with 16-B chunk c of row r at
// c ^ (r & 7), filled by LDS-DMA, two stages; split-K slabs reduced by slab_reduce_bf_kernel.
constexpr int GNB_BM = 128, GNB_BN = 48, GNB_BK = 64;
__global__ __launch_bounds__(256) void gemm_bf16_narrow_kernel(const bf16_t* __restrict__ A, long lda,
                                                               const bf16_t* __restrict__ B, long ldb,
                                                               float* __restrict__ slab, long slab_stride, int M,
                                                               int N, int K, int kchunk) {
  __shared__ __attribute__((aligned(16))) char lds[2][(GNB_BM + GNB_BN) * 128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int m0 = blockIdx.x * GNB_BM, s = blockIdx.y;
  const int kbeg = s * kchunk, nk = (min(K, kbeg + kchunk) - kbeg) / GNB_BK;
  // DMA map: 16-B chunk q of the stage: A rows 0..127 (q < 1024), then B rows 0..47
  auto fill = [&](int kt, int st) {
    const int k0 = kbeg + kt * GNB_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, c = (q & 7) ^ (row & 7);
      __builtin_amdgcn_global_load_lds((glb_vptr_t)(A + (long)(m0 + row) * lda + k0 + 8 * c),
                                       (lds_vptr_t)(&lds[st][0] + 16 * (w * 64 + 256 * i)), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && w >= 2) break;  // 384 chunks of B: waves 0-1 issue a second one (wave-uniform)
      const int q = tid + 256 * i, row = q >> 3, c = (q & 7) ^ (row & 7);
      const int n = min(row, N - 1);  // padding columns read row N - 1 (their sums are not stored)
      __builtin_amdgcn_global_load_lds((glb_vptr_t)(B + (long)n * ldb + k0 + 8 * c),
                                       (lds_vptr_t)(&lds[st][GNB_BM * 128] + 16 * (w * 64 + 256 * i)), 16, 0, 0);
    }
  };
  g8_f32x4 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = g8_f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk > 0) fill(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage st landed for every wave; stage st ^ 1 free
    if (kt + 1 < nk) fill(kt + 1, st ^ 1);
    const char* As = &lds[st][0];
    const char* Bs = &lds[st][GNB_BM * 128];
#pragma unroll
    for (int ks = 0; ks < GNB_BK / 32; ++ks) {
      const int c = 4 * ks + lq;  // lane group lq: k 8 lq .. 8 lq + 7 of the 32-k step
      bf16x8_t a[2], b[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 32 * w + 16 * i + lr;
        a[i] = *reinterpret_cast<const bf16x8_t*>(As + row * 128 + 16 * (c ^ (row & 7)));
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int row = 16 * j + lr;
        b[j] = *reinterpret_cast<const bf16x8_t*>(Bs + row * 128 + 16 * (c ^ (row & 7)));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = mfma16_bf16(b[j], a[i], acc[i][j]);
    }
  }
  // lane holds C[16 i + lr][16 j + 4 lq .. + 3] of its wave's rows
  float* Cz = slab + (long)s * slab_stride;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = 16 * j + 4 * lq;
      if (col < N)
        *reinterpret_cast<g8_f32x4*>(Cz + (long)(m0 + 32 * w + 16 * i + lr) * N + col) = acc[i][j];
    }
}
// exact plan of the narrow kernel: N <= 48 in whole 4-column groups, whole 128-row tiles, 64-k steps,
// K chunks of at least 1024 over up to 32 slabs (c3: 24 row tiles x 32 slabs = 768 workgroups)
static bool narrow_bf_ok(int M, int N, int K, long lda, long ldb) {
  return N <= GNB_BN && N % 4 == 0 && M % GNB_BM == 0 && K % GNB_BK == 0 && K >= 4096 &&
         lda % 8 == 0 && ldb % 8 == 0;
}
static int narrow_bf_splitk(int K, int& kchunk) {
  const int sk = std::max(1, std::min(32, K / 1024));
  kchunk = ((K + sk - 1) / sk + GNB_BK - 1) / GNB_BK * GNB_BK;
  return (K + kchunk - 1) / kchunk;
}

extern "C" size_t sv_gemm_bf16_workspace(int M, int N, int K) {
  const BPlan p = plan_bf16(M, N, K);
  size_t nar = 0;
  if (narrow_bf_ok(M, N, K, K, K)) {  // (the narrow kernel's slabs)
    int kchunk;
    nar = (size_t)narrow_bf_splitk(K, kchunk) * M * N * sizeof(float);
  }
  if (p.splitk <= 1) return nar;
  return std::max(nar, (size_t)p.splitk * M * N * sizeof(float));
}

extern "C" int sv_gemm_bf16(int M, int N, int K, const bf16_t* A, long lda, const bf16_t* B, long ldb, float* C,
                            long ldc, const float* bias0, const float* bias1, float beta, float* workspace,
                            hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C) return SV_EARG;
  if (K % 8 || lda % 8 || ldb % 8 || (((uintptr_t)A | (uintptr_t)B) & 15)) return SV_EALIGN;
  if (workspace && !((uintptr_t)workspace & 15) && narrow_bf_ok(M, N, K, lda, ldb)) {
    int kchunk;
    const int sk = narrow_bf_splitk(K, kchunk);
    const long slab = (long)M * N;
    hipLaunchKernelGGL(gemm_bf16_narrow_kernel, dim3(M / GNB_BM, sk), dim3(256), 0, stream, A, lda, B, ldb, workspace,
                       slab, M, N, K, kchunk);
    SV_LAUNCH_CHECK();
    const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
    hipLaunchKernelGGL(slab_reduce_bf_kernel, dim3(grid), dim3(256), 0, stream, workspace, sk, slab, C, ldc, M, N,
                       beta, bias0, bias1);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  const BPlan p = plan_bf16(M, N, K);
  if (p.bm == G256_BM) {
    const int tiles = (M / G256_BM) * (N / G256_BM);
    const long slab = (long)M * N;
    if (p.splitk == 1) {
      launch_g256<G256_STORE, 0>(g8_ok(C, ldc, bias0, bias1), dim3(tiles, 1), stream, A, lda, B, ldb, C, ldc, 0L,
                                 M, N, K, p.kchunk, bias0, bias1, beta);
      SV_LAUNCH_CHECK();
      return SV_OK;
    }
    if (!workspace) return SV_EARG;
    launch_g256<G256_SLAB, 0>(g8_ok(workspace, N, nullptr, nullptr), dim3(tiles, p.splitk), stream, A, lda, B,
                              ldb, workspace, (long)N, slab, M, N, K, p.kchunk, nullptr, nullptr, 0.f);
    SV_LAUNCH_CHECK();
    const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
    hipLaunchKernelGGL(slab_reduce_bf_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C, ldc, M, N,
                       beta, bias0, bias1);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (p.splitk == 1) {
    if (p.bm == 64)
      launch_bf<64, 64, BEPI_STORE>(A, lda, B, ldb, C, ldc, 0, M, N, K, 1, p.kchunk, bias0, bias1, beta, stream);
    else
      launch_bf<128, 128, BEPI_STORE>(A, lda, B, ldb, C, ldc, 0, M, N, K, 1, p.kchunk, bias0, bias1, beta, stream);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (!workspace) return SV_EARG;
  const long slab = (long)M * N;
  if (p.bm == 64)
    launch_bf<64, 64, BEPI_SLAB>(A, lda, B, ldb, workspace, N, slab, M, N, K, p.splitk, p.kchunk, nullptr, nullptr, 0.f,
                                 stream);
  else
    launch_bf<128, 128, BEPI_SLAB>(A, lda, B, ldb, workspace, N, slab, M, N, K, p.splitk, p.kchunk, nullptr, nullptr,
                                   0.f, stream);
  SV_LAUNCH_CHECK();
  const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
  hipLaunchKernelGGL(slab_reduce_bf_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C, ldc, M, N,
                     beta, bias0, bias1);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// C[M,N] bf16 = bf16(A . B^T + bias0 + bias1) (fp32 accumulation, one rounding): the bf16
// path's x-projection (K1), stored in the gates buffer the recurrence then overwrites with its
// bf16 activations.  The 8-phase 256 x 256 kernel where the shape tiles (no split-K), else the
// 128 x 128 / 64 x 64 kernel without split-K -- one kernel per shape, so every schedule that
// forms the same projection rounds it identically.
extern "C" int sv_gemm_bf16_bf(int M, int N, int K, const bf16_t* A, long lda, const bf16_t* B, long ldb, bf16_t* C,
                               long ldc, const float* bias0, const float* bias1, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C) return SV_EARG;
  if (K % 8 || lda % 8 || ldb % 8 || (((uintptr_t)A | (uintptr_t)B) & 15)) return SV_EALIGN;
  const BPlan p = plan_bf16(M, N, K);
  if (p.bm == G256_BM && p.splitk == 1 && g8_ok(nullptr, 0, bias0, bias1) && ldc % 8 == 0 &&
      !((uintptr_t)C & 15) && (size_t)N * 4 <= G8P_BIAS_LDS) {
    // persistent form: one workgroup per CU walks the tiles, each tile's store tail overlapping
    // the next tile's first fill
    const int tiles = (M / G256_BM) * (N / G256_BM);
    const int cus = sv_stream_cus(stream);
    const int grid = std::min(tiles, cus > 0 ? cus : 256);
    const size_t lds = G256_LDS + ((bias0 || bias1) ? (size_t)N * 4 : 0);
    hipLaunchKernelGGL((gemm_bf16_8qp_kernel<G8_STORE_BF16>), dim3(grid), dim3(512), lds, stream, A, lda, B, ldb,
                       (void*)C, ldc, M, N, K, bias0, bias1, 0.f);
  } else if ((long)((M + 127) / 128) * ((N + 127) / 128) < 128) {
    launch_bf<64, 64, BEPI_STORE_BF16>(A, lda, B, ldb, C, ldc, 0, M, N, K, 1, ((K + BBK - 1) / BBK) * BBK, bias0,
                                       bias1, 0.f, stream);
  } else {
    launch_bf<128, 128, BEPI_STORE_BF16>(A, lda, B, ldb, C, ldc, 0, M, N, K, 1, ((K + BBK - 1) / BBK) * BBK, bias0,
                                         bias1, 0.f, stream);
  }
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// dx = dG . W_ih with dG read from the persistent backward's fragment-order hand-off buffer
// (no row-major dG copy): M = T * B rows (t, b), K = 4H; needs B % 32, M % 256, N % 256, H % 64
bool gemm_afrag_ok(int T, int B, int N, int H) {
  return gemm256_ok(T * B, N, 4 * H) && B % 32 == 0 && H % G256_BK == 0 &&
         4 * H / G256_BK < 4096 && (unsigned long long)T * B * B < (1ull << 32);  // g256_af_koff / _rowoff exact
}
// (the split-K plan of sv_gemm_bf16 for the same shape)
// fin: a deferred bias finalize (sv_persist_bwd_bf16's `defer`) done by extra workgroups of the
// one-shot 8-phase launch, else by its own launch after the GEMM
int gemm_bf16_afrag(int T, int B, int H, int N, const bf16_t* dgf, int bm, const bf16_t* Bop, long ldb, float* C,
                    long ldc, float* workspace, hipStream_t stream, const DbFin& fin) {
  const int M = T * B, K = 4 * H;
  const int tiles = (M / G256_BM) * (N / G256_BM);
  const long fs = (long)((B + bm - 1) / bm) * bm * 4 * H;
  const G256AFrag af = g256_afrag(dgf, fs, B, bm, H);
  const BPlan p = plan_bf16(M, N, K);
  if (p.splitk == 1 && g8_ok(C, ldc, nullptr, nullptr)) {
    hipLaunchKernelGGL((gemm_bf16_8q_kernel<G256_STORE, 1>), dim3(tiles + dbfin_blocks(fin, 512)), dim3(512), G256_LDS,
                       stream, nullptr, 0L, Bop, ldb, (void*)C, ldc, 0L, M, N, K, p.kchunk, nullptr, nullptr, 0.f, af,
                       G256Dual{}, fin);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (int rc = sv_dbfin_launch(fin, stream)) return rc;
  if (p.splitk == 1) {
    launch_g256<G256_STORE, 1>(false, dim3(tiles, 1), stream, nullptr, 0L, Bop, ldb, C, ldc, 0L, M, N, K, p.kchunk,
                               nullptr, nullptr, 0.f, af);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (!workspace) return SV_EARG;
  const long slab = (long)M * N;
  launch_g256<G256_SLAB, 1>(g8_ok(workspace, N, nullptr, nullptr), dim3(tiles, p.splitk), stream, nullptr, 0L,
                            Bop, ldb, workspace, (long)N, slab, M, N, K, p.kchunk, nullptr, nullptr, 0.f, af);
  SV_LAUNCH_CHECK();
  const int grid = (int)std::min<long>((slab + 255) / 256, 4096);
  hipLaunchKernelGGL(slab_reduce_bf_kernel, dim3(grid), dim3(256), 0, stream, workspace, p.splitk, slab, C, ldc, M, N,
                     0.f, nullptr, nullptr);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_cast_bf16_batch(int n, const float* const* x, bf16_t* const* y, const long* count,
                                  hipStream_t stream);
extern "C" int sv_cast_bf16(const float* x, bf16_t* y, long n, hipStream_t stream) {
  if (!x || !y || n <= 0) return SV_EARG;
  return sv_cast_bf16_batch(1, &x, &y, &n, stream);
}

extern "C" int sv_cast_bf16_batch(int n, const float* const* x, bf16_t* const* y, const long* count,
                                  hipStream_t stream) {
  if (n <= 0 || n > 8 || !x || !y || !count) return SV_EARG;
  CastBatch cb{};
  cb.n = n;
  bool vec = true;
  for (int i = 0; i < n; ++i) {
    if (!x[i] || !y[i] || count[i] <= 0) return SV_EARG;
    cb.x[i] = x[i];
    cb.y[i] = y[i];
    vec = vec && count[i] % 4 == 0 && !((uintptr_t)x[i] & 15) && !((uintptr_t)y[i] & 7);
  }
  for (int i = 0; i < n; ++i) cb.start[i + 1] = cb.start[i] + (vec ? count[i] / 4 : count[i]);
  const int grid = (int)std::min<long>((cb.start[n] + 255) / 256, 8192);
  if (vec)
    hipLaunchKernelGGL(cast_bf16_batch_kernel<true>, dim3(grid), dim3(256), 0, stream, cb);
  else
    hipLaunchKernelGGL(cast_bf16_batch_kernel<false>, dim3(grid), dim3(256), 0, stream, cb);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// the transpose-casts of up to 8 matrices in one launch (dst[c ldd + r] = bf16(src[r lds + c]));
// dstr (optional, per matrix): also the row-major cast dstr[r C + c], from the same read; a null
// dst[i] with a dstr[i]: the row-major cast alone
int transpose_cast_bf16_batch(int n, const float* const* src, const long* lds, const int* R, const int* C,
                              bf16_t* const* dst, const long* ldd, hipStream_t stream, bf16_t* const* dstr = nullptr,
                              const FramesArgs* frames = nullptr) {
  if (n <= 0 || n > 8) return SV_EARG;
  TCastBatch tb{};
  tb.n = n;
  for (int i = 0; i < n; ++i) {
    if (!src[i] || !(dst[i] || (dstr && dstr[i])) || R[i] <= 0 || C[i] <= 0) return SV_EARG;
    tb.src[i] = src[i];
    tb.dst[i] = dst[i];
    tb.dstr[i] = dstr ? dstr[i] : nullptr;
    tb.lds[i] = lds[i];
    tb.ldd[i] = ldd[i];
    tb.R[i] = R[i];
    tb.C[i] = C[i];
    tb.tx[i] = (C[i] + 63) / 64;
    tb.tile0[i + 1] = tb.tile0[i] + tb.tx[i] * ((R[i] + 63) / 64);
    const bool rv = !tb.dstr[i] || (C[i] % 4 == 0 && !((uintptr_t)tb.dstr[i] & 7));
    if (lds[i] % 4 == 0 && ldd[i] % 8 == 0 && !((uintptr_t)src[i] & 15) && !((uintptr_t)dst[i] & 15) && rv)
      tb.vec |= 1u << i;
  }
  const FramesArgs fa = frames ? *frames : FramesArgs{};
  const int nfr = frames ? fa.nbx * fa.T : 0;
  hipLaunchKernelGGL(transpose_cast_batch_kernel, dim3(nfr + tb.tile0[n]), dim3(256), 0, stream, tb, fa, nfr);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// the bf16 stack's input in one launch (ABI v10; was to_time_major + a cast + a transpose-cast, and
// T transpose-casts when B % 8 != 0): frames_tile above, one workgroup per (64 rows, timestep)
__global__ __launch_bounds__(256) void frames_to_bf16_kernel(const FramesArgs fa) {
  __shared__ float tile[64][65];  // [b][f], F <= 64
  frames_tile(fa, blockIdx.x, blockIdx.y, tile);
}
static FramesArgs frames_args(const float* x, int B, int T, int F, bf16_t* x_bf, bf16_t* xT, int Bp) {
  return FramesArgs{x, x_bf, xT, B, T, F, Bp, (std::max(B, xT ? Bp : B) + 63) / 64};
}
extern "C" int sv_frames_to_bf16(const float* x, int B, int T, int F, bf16_t* x_bf, bf16_t* xT, int Bp,
                                 hipStream_t stream) {
  if (!x || !x_bf || B <= 0 || T <= 0 || F <= 0 || F > 64 || (xT && Bp < B)) return SV_EARG;
  const FramesArgs fa = frames_args(x, B, T, F, x_bf, xT, Bp);
  hipLaunchKernelGGL(frames_to_bf16_kernel, dim3(fa.nbx, T), dim3(256), 0, stream, fa);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_transpose_cast_bf16(const float* src, long ld_src, int R, int C, bf16_t* dst, long ld_dst,
                                      hipStream_t stream) {
  if (!src || !dst || R <= 0 || C <= 0) return SV_EARG;
  return transpose_cast_bf16_batch(1, &src, &ld_src, &R, &C, &dst, &ld_dst, stream);
}

extern "C" int sv_lstm_layer_fwd_bf16(const bf16_t* x_bf, int T, int B, int F, int H, const bf16_t* w_ih_bf,
                                      const bf16_t* w_hh_bf, const float* b_ih, const float* b_hh, bf16_t* gates,
                                      float* c_tm, float* h_tm, bf16_t* h_bf, bf16_t* hT, hipStream_t stream) {
  if (!x_bf || !w_ih_bf || !w_hh_bf || !gates || !c_tm || !h_tm || !h_bf) return SV_EARG;
  if (T <= 0 || B <= 0 || F <= 0 || H <= 0 || F % 8 || H % 8) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  int rc = sv_gemm_bf16_bf(T * B, 4 * H, F, x_bf, F, w_ih_bf, F, gates, 4L * H, b_ih, b_hh, stream);
  if (rc) return rc;
  hipError_t e = sv_memset0(h_tm, BH * sizeof(float), stream);
  if (e != hipSuccess) return (int)e;
  e = sv_memset0(h_bf, BH * sizeof(bf16_t), stream);
  if (e != hipSuccess) return (int)e;
  const int Bp = (B + 7) & ~7;
  const long ldhT = (long)(T + 1) * Bp;
  if (hT && Bp != B) {
    e = sv_memset0(hT, (size_t)H * ldhT * sizeof(bf16_t), stream);
    if (e != hipSuccess) return (int)e;
  }
  const dim3 grid((H + BF_U - 1) / BF_U, (B + BF_BM - 1) / BF_BM);
  for (int t = 0; t < T; ++t) {
    launch_fwd_bf16(grid, stream, t ? h_bf + t * BH : nullptr, w_hh_bf, gates + t * BG,
                    t ? c_tm + (t - 1) * BH : nullptr, c_tm + t * BH, h_tm + (t + 1) * BH, h_bf + (t + 1) * BH, hT,
                    ldhT, t, Bp, B, H);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

extern "C" size_t sv_lstm_layer_bwd_bf16_workspace(int T, int B, int F, int H) {
  const int TBp = T * ((B + 7) & ~7);
  size_t g = sv_gemm_bf16_workspace(4 * H, H, TBp);
  g = std::max(g, sv_gemm_bf16_workspace(4 * H, F, TBp));
  g = std::max(g, sv_gemm_bf16_workspace(T * B, F, 4 * H));
  return 2 * ((size_t)B * H * sizeof(float) + 256) + g + 256;
}

extern "C" int sv_lstm_layer_bwd_bf16(int T, int B, int F, int H, const bf16_t* xT_bf, long ld_xT,
                                      const bf16_t* wihT_bf, const bf16_t* whhT_bf, const bf16_t* gates,
                                      const float* c_tm, const bf16_t* hT_bf, const float* dh_up, int dh_up_full,
                                      bf16_t* dg_bf, bf16_t* dgT_bf, float* dx_tm, float* dw_ih, float* dw_hh,
                                      float* db_ih, float* db_hh, float* workspace, hipStream_t stream) {
  if (!xT_bf || !wihT_bf || !whhT_bf || !gates || !c_tm || !hT_bf || !dg_bf || !dgT_bf || !dw_ih || !dw_hh || !db_ih ||
      !workspace)
    return SV_EARG;
  if (T <= 0 || B <= 0 || F <= 0 || H <= 0 || F % 8 || H % 8 || ld_xT % 8) return SV_ESHAPE;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 7) & ~7;
  const int TBp = T * Bp;
  const size_t dcfsz = ((size_t)BH * sizeof(float) + 255) / 256 * 256 / sizeof(float);
  float* dcf0 = workspace;
  float* dcf1 = workspace + dcfsz;
  float* gws = workspace + 2 * dcfsz;
  if (Bp != B) {
    hipError_t e = sv_memset0(dgT_bf, (size_t)4 * H * TBp * sizeof(bf16_t), stream);
    if (e != hipSuccess) return (int)e;
  }
  const dim3 grid((H + BF_U - 1) / BF_U, (B + BF_BM - 1) / BF_BM);
  for (int t = T - 1; t >= 0; --t) {
    const float* up = nullptr;
    if (dh_up) up = dh_up_full ? dh_up + t * BH : (t == T - 1 ? dh_up : nullptr);
    float* dcf_out = (t & 1) ? dcf1 : dcf0;
    const float* dcf_in = (t == T - 1) ? nullptr : ((t & 1) ? dcf0 : dcf1);
    launch_bwd_bf16(grid, stream, t == T - 1 ? nullptr : dg_bf + (t + 1) * BG, whhT_bf, up, dcf_in, gates + t * BG,
                    c_tm + t * BH, t ? c_tm + (t - 1) * BH : nullptr, dg_bf + t * BG, dcf_out, dgT_bf, (long)TBp, t,
                    Bp, B, H);
    SV_LAUNCH_CHECK();
  }
  const long ldhT = (long)(T + 1) * Bp;
  int rc = sv_gemm_bf16(4 * H, H, TBp, dgT_bf, TBp, hT_bf, ldhT, dw_hh, H, nullptr, nullptr, 0.f, gws, stream);
  if (rc) return rc;
  rc = sv_gemm_bf16(4 * H, F, TBp, dgT_bf, TBp, xT_bf, ld_xT, dw_ih, F, nullptr, nullptr, 0.f, gws, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(rowsum_bf16_kernel, dim3(4 * H), dim3(256), 0, stream, dgT_bf, (long)TBp, TBp, db_ih, db_hh);
  SV_LAUNCH_CHECK();
  if (dx_tm) {
    rc = sv_gemm_bf16(T * B, F, 4 * H, dg_bf, 4L * H, wihT_bf, 4L * H, dx_tm, F, nullptr, nullptr, 0.f, gws, stream);
    if (rc) return rc;
  }
  return SV_OK;
}

// Stack forward, bf16 operands.  `schedule` (include/sv_ge2e.h): the layer wavefront (one launch
// for every layer's recurrence and input projection, sv_wave.hip) where the grids fit; else per
// layer its K1 GEMM and one persistent recurrence launch (layer 0's projection in-kernel); else
// (SV_SCHED_PER_STEP, or H without a persistent kernel) the layer-pipelined per-step schedule of
// sv_lstm_stack_fwd (sv_lstm.hip).
extern "C" int sv_lstm_stack_fwd_bf16(int L, int T, int B, int F, int H, const bf16_t* x_bf,
                                      const bf16_t* const* w_ih_bf, const bf16_t* const* w_hh_bf,
                                      const float* const* b_ih, const float* const* b_hh, bf16_t* const* gates,
                                      float* const* c_tm, float* const* h_tm, bf16_t* const* h_bf,
                                      bf16_t* const* hT, int chunk, hipStream_t main, const hipStream_t* side,
                                      hipEvent_t* ev, void* sync_block, hipEvent_t* probe, int schedule) {
  if (L <= 0 || !x_bf || !w_ih_bf || !w_hh_bf || !gates || !c_tm || !h_tm || !h_bf || !side || !ev || chunk <= 0)
    return SV_EARG;
  if (schedule & ~SV_SCHED_MASK) return SV_EARG;
  unsigned* sync = reinterpret_cast<unsigned*>(sync_block);
  if (T <= 0 || B <= 0 || F <= 0 || H <= 0 || F % 8 || H % 8) return SV_ESHAPE;
  const int nch = (T + chunk - 1) / chunk;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 7) & ~7;
  const long ldhT = (long)(T + 1) * Bp;
  hipError_t e;
  auto zero_state = [&](int l, hipStream_t s) -> int {
    if ((e = sv_memset0(h_tm[l], BH * sizeof(float), s)) != hipSuccess) return (int)e;
    if ((e = sv_memset0(h_bf[l], BH * sizeof(bf16_t), s)) != hipSuccess) return (int)e;
    if (hT[l] && Bp != B && (e = sv_memset0(hT[l], (size_t)H * ldhT * sizeof(bf16_t), s)) != hipSuccess)
      return (int)e;
    return SV_OK;
  };
  // every layer's state reset in one launch (the schedules that run on `main`); cnt: also the
  // counter channels 0..L-1 of the sync block (the layer wavefront's), in the same launch
  auto zero_states = [&](hipStream_t s, bool cnt) -> int {
    void* p[SV_ZB_MAX];
    size_t b[SV_ZB_MAX];
    int n = 0;
    for (int l = 0; l < L; ++l) {
      if (n + 3 > SV_ZB_MAX) {
        if (int rc = sv_zero_bytes_multi(n, p, b, s)) return rc;
        n = 0;
      }
      p[n] = h_tm[l], b[n++] = BH * sizeof(float);
      p[n] = h_bf[l], b[n++] = BH * sizeof(bf16_t);
      if (hT[l] && Bp != B) p[n] = hT[l], b[n++] = (size_t)H * ldhT * sizeof(bf16_t);
    }
    if (cnt) {  // every counter channel: this forward's and the backward's that follows
      if (n == SV_ZB_MAX) {
        if (int rc = sv_zero_bytes_multi(n, p, b, s)) return rc;
        n = 0;
      }
      p[n] = sync + SV_SYNC_CNT, b[n++] = (size_t)SV_SYNC_CHANNELS * SV_PCNT_ROWS * SV_PCNT_STRIDE * sizeof(unsigned);
    }
    return sv_zero_bytes_multi(n, p, b, s);
  };
  int rc;
  if (sched_wave(schedule, H) && sv_wave_fwd_fits(L, T, B, F, H, sv_stream_cus(main))) {
    // layer-wavefront schedule (sv_wave.hip): every layer's recurrence and input projection in
    // one launch on `main`
    if (!sync || L > SV_SYNC_CHANNELS) return SV_EARG;
    if ((rc = zero_states(main, true))) return rc;
    return sv_wave_fwd_bf16(L, T, B, F, H, x_bf, w_ih_bf, w_hh_bf, b_ih, b_hh, gates, c_tm, h_tm, h_bf, hT, sync, main,
                            sv_persist_limit(), sv_persist_fault(0), probe ? probe[0] : nullptr,
                            probe ? probe[1] : nullptr, 1);
  }
  if (sched_persist(schedule, H) && sv_persist_fwd_fits(B, H, sv_stream_cus(main))) {
    if (!sync) return SV_EARG;
    // persistent schedule on `main`: per layer the whole-T K1 GEMM, then one launch for the
    // recurrence (sv_persist.hip); layers run one after another, layer l on counter channel l
    // (zeroed, with the backward's, in the state-reset launch) where L <= SV_BWD_CH0, else all on
    // channel 0, each launch zeroing it
    const bool own = L <= SV_BWD_CH0;
    if ((rc = zero_states(main, true))) return rc;
    for (int l = 0; l < L; ++l) {
      const int Fl = l == 0 ? F : H;
      const bf16_t* in = l == 0 ? x_bf : h_bf[l - 1] + BH;
      if (l == 0 && sv_persist_fwd_fusex_ok(H, F)) {  // layer 0's input projection inside the recurrence
        if ((rc = sv_persist_fwd_bf16(T, B, H, w_hh_bf[l], gates[l], c_tm[l], h_tm[l], h_bf[l], hT[l], main, sync,
                                      own ? l : 0, x_bf, F, w_ih_bf[l], b_ih[l], b_hh[l],
                                      probe ? probe[2 * l] : nullptr, probe ? probe[2 * l + 1] : nullptr, own)))
          return rc;
        continue;
      }
      rc = sv_gemm_bf16_bf(T * B, 4 * H, Fl, in, Fl, w_ih_bf[l], Fl, gates[l], 4L * H, b_ih[l], b_hh[l], main);
      if (rc) return rc;
      if ((rc = sv_persist_fwd_bf16(T, B, H, w_hh_bf[l], gates[l], c_tm[l], h_tm[l], h_bf[l], hT[l], main, sync,
                                    own ? l : 0, nullptr, 0, nullptr, nullptr, nullptr,
                                    probe ? probe[2 * l] : nullptr, probe ? probe[2 * l + 1] : nullptr, own)))
        return rc;
    }
    return SV_OK;
  }
  // per-step schedule: no counters of its own, but the backward's zeroed all the same (the
  // caller may pass SV_SCHED_CNT_READY to a persistent backward after any stack forward)
  if (sync && (rc = sv_zero_bytes(sync + SV_SYNC_CNT + (size_t)SV_BWD_CH0 * SV_PCNT_ROWS * SV_PCNT_STRIDE,
                                  (size_t)(SV_SYNC_CHANNELS - SV_BWD_CH0) * SV_PCNT_ROWS * SV_PCNT_STRIDE *
                                      sizeof(unsigned),
                                  main)))
    return rc;
  hipEvent_t ev_start = ev[L * nch];
  e = hipEventRecord(ev_start, main);
  if (e != hipSuccess) return (int)e;
  for (int l = 0; l < L; ++l) {
    hipStream_t s = side[l];
    if ((e = hipStreamWaitEvent(s, ev_start, 0)) != hipSuccess) return (int)e;
    if ((rc = zero_state(l, s))) return rc;
  }
  const dim3 grid((H + BF_U - 1) / BF_U, (B + BF_BM - 1) / BF_BM);
  for (int c = 0; c < nch + L - 1; ++c) {
    for (int l = 0; l < L; ++l) {
      const int cc = c - l;
      if (cc < 0 || cc >= nch) continue;
      hipStream_t s = side[l];
      const int t0 = cc * chunk, t1 = std::min(T, t0 + chunk);
      const int Fl = l == 0 ? F : H;
      const bf16_t* in = l == 0 ? x_bf + (long)t0 * B * F : h_bf[l - 1] + (long)(t0 + 1) * BH;
      if (l > 0 && (e = hipStreamWaitEvent(s, ev[(l - 1) * nch + cc], 0)) != hipSuccess) return (int)e;
      rc = sv_gemm_bf16_bf((t1 - t0) * B, 4 * H, Fl, in, Fl, w_ih_bf[l], Fl, gates[l] + t0 * BG, 4L * H, b_ih[l],
                           b_hh[l], s);
      if (rc) return rc;
      for (int t = t0; t < t1; ++t) {
        launch_fwd_bf16(grid, s, t ? h_bf[l] + t * BH : nullptr, w_hh_bf[l], gates[l] + t * BG,
                        t ? c_tm[l] + (t - 1) * BH : nullptr, c_tm[l] + t * BH, h_tm[l] + (t + 1) * BH,
                        h_bf[l] + (t + 1) * BH, hT[l], ldhT, t, Bp, B, H);
        SV_LAUNCH_CHECK();
      }
      if ((e = hipEventRecord(ev[l * nch + cc], s)) != hipSuccess) return (int)e;
    }
  }
  for (int l = 0; l < L; ++l)
    if ((e = hipStreamWaitEvent(main, ev[l * nch + nch - 1], 0)) != hipSuccess) return (int)e;
  return SV_OK;
}

// Layer-pipelined stack backward, bf16 operands (see sv_lstm_stack_bwd in sv_lstm.hip).
namespace {
struct BBwdWs {
  float *dcf0, *dcf1, *gws;
  bf16_t *whhT, *wihT;
  size_t gbytes, total;  // gws bytes; the region's
};
BBwdWs carve_bbwd(char* base, int T, int B, int F, int H) {
  BBwdWs w;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~size_t(255);
    return p;
  };
  w.dcf0 = (float*)take((size_t)B * H * 4);
  w.dcf1 = (float*)take((size_t)B * H * 4);
  w.whhT = (bf16_t*)take((size_t)4 * H * H * 2);
  w.wihT = (bf16_t*)take((size_t)bf16_wiht_ld(H) * F * 2);
  const int TBp = T * ((B + 7) & ~7);
  size_t g = sv_gemm_bf16_workspace(4 * H, H, TBp);
  g = std::max(g, sv_gemm_bf16_workspace(4 * H, F, TBp));
  g = std::max(g, sv_gemm_bf16_workspace(T * B, F, 4 * H));
  g = std::max(g, sv_gemm_bf16_dual_workspace(4 * H, H, F, TBp));
  w.gws = (float*)take(g);
  w.gbytes = g;
  w.total = off;
  return w;
}
}  // namespace

// L per-layer regions, then the persistent backward's hand-off scratch (shared by the layers,
// whose recurrences run one after another)
// W_hh^T of every layer and W_ih^T of layers >= 1 (bf16 [K, 4H]) in one or two launches
static int wbf_transposes(int L, int F, int H, const float* const* w_ih, const float* const* w_hh,
                          const bf16_t* const* whhT, const bf16_t* const* wihT, hipStream_t s) {
  const float* src[8];
  bf16_t* dst[8];
  long lds[8], ldd[8];
  int R[8], C[8], n = 0;
  auto flush = [&]() -> int {
    const int rc = n ? transpose_cast_bf16_batch(n, src, lds, R, C, dst, ldd, s) : 0;
    n = 0;
    return rc;
  };
  for (int l = 0; l < L; ++l) {
    for (int m = 0; m < (l > 0 ? 2 : 1); ++m) {
      if (n == 8)
        if (int rc = flush()) return rc;
      const int K = m == 0 ? H : (l == 0 ? F : H);
      src[n] = m == 0 ? w_hh[l] : w_ih[l];
      dst[n] = const_cast<bf16_t*>(m == 0 ? whhT[l] : wihT[l]);
      lds[n] = K;
      ldd[n] = m == 0 ? 4L * H : bf16_wiht_ld(H);
      R[n] = 4 * H;
      C[n] = K;
      ++n;
    }
  }
  return flush();
}

// ABI v10: every layer's bf16 weights in one launch (transpose_cast_batch_kernel, each fp32 weight
// read once): the forward's row-major operands w_ih_bf / w_hh_bf and, when bwd_workspace is given
// (a stack-backward workspace, sv_lstm_bwd_workspace(SV_DTYPE_BF16, ...)), the transposes the stack
// backward reads -- W_hh^T of every layer, W_ih^T of layers >= 1 -- in that workspace's per-layer
// regions, so that sv_lstm_bwd with SV_SCHED_WT_READY on the same workspace launches none (at the
// c4 rank shape: the forward's cast and the backward's transposes, 13 + 20 us, read every weight
// twice)
static int weights_bf16(int L, int T, int B, int F, int H, const float* const* w_ih, const float* const* w_hh,
                        bf16_t* const* w_ih_bf, bf16_t* const* w_hh_bf, void* bwd_workspace, hipStream_t stream,
                        const FramesArgs* frames);
extern "C" int sv_lstm_weights_bf16(int L, int T, int B, int F, int H, const float* const* w_ih,
                                    const float* const* w_hh, bf16_t* const* w_ih_bf, bf16_t* const* w_hh_bf,
                                    void* bwd_workspace, hipStream_t stream) {
  return weights_bf16(L, T, B, F, H, w_ih, w_hh, w_ih_bf, w_hh_bf, bwd_workspace, stream, nullptr);
}
// ABI v11: sv_frames_to_bf16 and sv_lstm_weights_bf16 as ONE launch (the frames' workgroups beside
// the weight tiles: at the c4 rank shape 10 + 17 us one after the other)
extern "C" int sv_lstm_prep_bf16(int L, int T, int B, int F, int H, const float* x, bf16_t* x_bf, bf16_t* xT, int Bp,
                                 const float* const* w_ih, const float* const* w_hh, bf16_t* const* w_ih_bf,
                                 bf16_t* const* w_hh_bf, void* bwd_workspace, hipStream_t stream) {
  if (!x || !x_bf || F > 64 || (xT && Bp < B)) return SV_EARG;
  const FramesArgs fa = frames_args(x, B, T, F, x_bf, xT, Bp);
  return weights_bf16(L, T, B, F, H, w_ih, w_hh, w_ih_bf, w_hh_bf, bwd_workspace, stream, &fa);
}
static int weights_bf16(int L, int T, int B, int F, int H, const float* const* w_ih, const float* const* w_hh,
                        bf16_t* const* w_ih_bf, bf16_t* const* w_hh_bf, void* bwd_workspace, hipStream_t stream,
                        const FramesArgs* frames) {
  if (L <= 0 || !w_ih || !w_hh || !w_ih_bf || !w_hh_bf) return SV_EARG;
  if (T <= 0 || B <= 0 || F <= 0 || H <= 0 || F % 8 || H % 8) return SV_ESHAPE;
  const size_t per = carve_bbwd(nullptr, T, B, std::max(F, H), H).total;
  const float* src[8];
  bf16_t *dst[8], *dstr[8];
  long lds[8], ldd[8];
  int R[8], C[8], n = 0;
  for (int l = 0; l < L; ++l) {
    if (!w_ih[l] || !w_hh[l] || !w_ih_bf[l] || !w_hh_bf[l]) return SV_EARG;
    BBwdWs ws{};
    if (bwd_workspace) ws = carve_bbwd((char*)bwd_workspace + per * l, T, B, std::max(F, H), H);
    for (int m = 0; m < 2; ++m) {  // m = 0: W_ih [4H][F_l], m = 1: W_hh [4H][H]
      if (n == 8) {
        if (int rc = transpose_cast_bf16_batch(n, src, lds, R, C, dst, ldd, stream, dstr)) return rc;
        n = 0;
      }
      const int K = (m == 0 && l == 0) ? F : H;
      src[n] = m == 0 ? w_ih[l] : w_hh[l];
      dstr[n] = m == 0 ? w_ih_bf[l] : w_hh_bf[l];
      dst[n] = !bwd_workspace ? nullptr : m == 1 ? ws.whhT : (l > 0 ? ws.wihT : nullptr);
      ldd[n] = m == 1 ? 4L * H : bf16_wiht_ld(H);
      lds[n] = K;
      R[n] = 4 * H;
      C[n] = K;
      ++n;
    }
  }
  return transpose_cast_bf16_batch(n, src, lds, R, C, dst, ldd, stream, dstr, frames);  // frames: the last launch
}

#ifndef SV_PERSIST_FULLK
#define SV_PERSIST_FULLK 1  // the persistent schedule's weight gradients as one whole-K launch (A/B)
#endif
// the hand-off scratch shared by the layers (persistent or wavefront backward), behind the L
// per-layer regions
static size_t bbwd_scratch(int L, int T, int B, int H) {
  size_t scratch = sv_persist_bwd_fits(B, H, 1 << 30) ? sv_persist_bwd_scratch(T, B, H) : 0;
  if (sv_wave_bwd_fits(L, B, H, 1 << 30)) scratch = std::max(scratch, sv_wave_bwd_scratch(L, T, B, H));
  return (scratch + 255) & ~size_t(255);
}
extern "C" size_t sv_lstm_stack_bwd_bf16_workspace(int L, int T, int B, int F, int H) {
  const size_t per = (size_t)L * carve_bbwd(nullptr, T, B, std::max(F, H), H).total;
  return per + bbwd_scratch(L, T, B, H);
}

extern "C" int sv_lstm_stack_bwd_bf16(int L, int T, int B, int F, int H, const bf16_t* const* xT, const long* ld_xT,
                                      const float* const* w_ih, const float* const* w_hh, const bf16_t* const* gates,
                                      const float* const* c_tm, const bf16_t* const* hT, const float* dh_last,
                                      bf16_t* const* dg, bf16_t* const* dgT, float* const* dx, float* const* dw_ih,
                                      float* const* dw_hh, float* const* db_ih, float* const* db_hh, void* workspace,
                                      int chunk, hipStream_t main, const hipStream_t* side, hipEvent_t* ev,
                                      void* sync_block, hipEvent_t* probe, int schedule) {
  if (L <= 0 || !xT || !ld_xT || !w_ih || !w_hh || !gates || !c_tm || !hT || !dh_last || !dg || !dgT || !dx ||
      !dw_ih || !dw_hh || !db_ih || !workspace || !side || !ev || chunk <= 0)
    return SV_EARG;
  if (schedule & ~SV_SCHED_MASK) return SV_EARG;
  unsigned* sync = reinterpret_cast<unsigned*>(sync_block);
  if (T <= 0 || B <= 0 || F <= 0 || H <= 0 || F % 8 || H % 8) return SV_ESHAPE;
  const int nch = (T + chunk - 1) / chunk;
  const long BH = (long)B * H, BG = 4L * B * H;
  const int Bp = (B + 7) & ~7;
  const int TBp = T * Bp;
  const long ldhT = (long)(T + 1) * Bp;
  const size_t per = carve_bbwd(nullptr, T, B, std::max(F, H), H).total;
  hipError_t e;
  // the per-layer completion events (a caller's gradient buckets wait on them) of the persistent and
  // wavefront schedules; SV_SCHED_NO_EVENTS: nobody waits, record none (each record idles the GPU)
  const bool evs = !(schedule & SV_SCHED_NO_EVENTS);
  // SV_SCHED_WT_READY: sv_lstm_weights_bf16 already wrote the transposes into this workspace
  const bool wt_ready = schedule & SV_SCHED_WT_READY;
  // SV_SCHED_CNT_READY: the stack forward zeroed the backward's counter channels and no backward
  // has used this sync block since (the caller tracks that): no zeroing launches here
  const bool cnt_ready = schedule & SV_SCHED_CNT_READY;
  // every layer's whole-K weight-gradient tiles in one launch where they fit one round of the CUs
  // (gemm_bf16_8qf_kernel; layer 0's N = F dW_ih after it on the narrow kernel), the split form
  // (first pieces on the CUs the tiles leave free, their flags on channel SV_BWD_CH0 + WB_L) where
  // at least 8 CUs are left over and the partials fit the GEMM scratch
  auto plan_fullk = [&](G8Full& f, int& fP) -> bool {
    const int cus = sv_stream_cus(main);
    f = G8Full{};
    fP = 0;
    if (!(L == WB_L && gemm256_ok(4 * H, H, TBp) && TBp % 8 == 0 && ldhT % 8 == 0)) return false;
    bool fullk = true;
    f.K = TBp;
    for (int l = 0; l < L; ++l) {
      // upper layers: dW_ih beside dW_hh (input width H, 3 column tiles); layer 0 too (x0 tile):
      // its F <= 256 columns as one partial column tile (x^T rows clamped, F columns stored) --
      // the narrow GEMM after the launch re-read all of dG^T_0 for them (c5 rank 76 + 10 us)
      const bool x0 = l == 0 && F <= G256_BM && F % 4 == 0;
      const bool dual = l > 0 || x0;
      G8FLayer& fl = f.lay[l];
      fl.A = dgT[l];
      fl.lda = TBp;
      fl.B = hT[l];
      fl.ldb = ldhT;
      fl.B2 = dual ? xT[l] : nullptr;
      fl.ldb2 = dual ? ld_xT[l] : 0;
      fl.C1 = dw_hh[l];
      fl.ldc1 = H;
      fl.C2 = dual ? dw_ih[l] : nullptr;
      fl.ldc2 = l > 0 ? H : F;
      fl.n1 = H;
      fl.N = l > 0 ? 2 * H : x0 ? H + G256_BM : H;
      fl.f2 = x0 ? F : 0;
      fl.tiles = (4 * H / G256_BM) * (fl.N / G256_BM);
      fP += fl.tiles;
      if (((uintptr_t)dgT[l] | (uintptr_t)hT[l] | (uintptr_t)dw_hh[l]) & 15) fullk = false;
      if (dual && ((((uintptr_t)xT[l] | (uintptr_t)dw_ih[l]) & 15) || ld_xT[l] % 8 || fl.ldc2 % 4)) fullk = false;
    }
    fullk = fullk && fP <= cus;
    const BBwdWs wsp = carve_bbwd((char*)workspace + per * (L - 1), T, B, std::max(F, H), H);
    const int KT = TBp / G256_BK;
    f.nsw = fullk ? (cus - fP) / 8 * 8 : 0;
    if (f.nsw > 0) {
      const int per_wg = (fP + f.nsw - 1) / f.nsw;  // first pieces per workgroup
      f.S = KT / (per_wg + 1) - 2;    // (their stores and prologues: a little less)
    }
    if (f.nsw <= 0 || f.S < 4 || (size_t)fP * G256_BM * G256_BM * 4 > wsp.gbytes) f.nsw = f.S = 0;
    if (f.S > 0) {
      f.part = wsp.gws;
      f.flag = sync + SV_SYNC_CNT + (size_t)(SV_BWD_CH0 + WB_L) * SV_PCNT_ROWS * SV_PCNT_STRIDE;
      f.status = sync;
      f.limit = sv_persist_limit();
    }
    return fullk;
  };
  // the whole-K launch, then layer 0's dW_ih and the layers' completion events
  auto run_fullk = [&](const G8Full& f, int fP) -> int {
    hipLaunchKernelGGL(gemm_bf16_8qf_kernel, dim3(f.nsw + fP + dbfin_blocks(f.fin, 512)), dim3(512), G256_LDS, main, f);
    SV_LAUNCH_CHECK();
    for (int l = L - 1; l >= 1 && evs; --l)
      if ((e = hipEventRecord(ev[L * nch + l], main)) != hipSuccess) return (int)e;
    if (!f.lay[0].f2) {  // layer 0's dW_ih (F > 256) on its own
      const BBwdWs ws = carve_bbwd((char*)workspace, T, B, std::max(F, H), H);
      if (int rc = sv_gemm_bf16(4 * H, F, TBp, dgT[0], TBp, xT[0], ld_xT[0], dw_ih[0], F, nullptr, nullptr, 0.f, ws.gws,
                                main))
        return rc;
    }
    if (evs && (e = hipEventRecord(ev[L * nch], main)) != hipSuccess) return (int)e;
    return SV_OK;
  };
  if (sched_wave(schedule, H) && sv_wave_bwd_fits(L, B, H, sv_stream_cus(main))) {
    if (!sync) return SV_EARG;
    // layer-wavefront schedule: every layer's recurrence and upstream gradient dx in one launch
    // (sv_persist3.hip, no dx GEMMs; bias gradients summed in the kernel), then per layer the
    // weight gradients on `main`
    const bf16_t* whhT_l[WB_L];
    const bf16_t* wihT_l[WB_L];
    for (int l = 0; l < L; ++l) {
      const BBwdWs ws = carve_bbwd((char*)workspace + per * l, T, B, std::max(F, H), H);
      whhT_l[l] = ws.whhT;
      wihT_l[l] = l > 0 ? ws.wihT : nullptr;
    }
    int rc = wt_ready ? 0 : wbf_transposes(L, F, H, w_ih, w_hh, whhT_l, wihT_l, main);
    if (rc) return rc;
    G8Full f;
    int fP;
    const bool fullk = plan_fullk(f, fP);
    // with the whole-K launch after it, the bias finalize rides on that launch (G8Full::fin)
    rc = sv_wave_bwd_bf16(L, T, B, H, whhT_l, wihT_l, gates, c_tm, dh_last, dx, dgT, (char*)workspace + per * L,
                              sync, main, db_ih, db_hh, probe ? probe[0] : nullptr, probe ? probe[1] : nullptr,
                              bf16_wiht_ld(H), f.S > 0 ? fP : 0, SV_BWD_CH0, cnt_ready, fullk ? &f.fin : nullptr);
    if (rc) return rc;
    if (fullk) return run_fullk(f, fP);
    for (int l = L - 1; l >= 0; --l) {
      const int Fl = l == 0 ? F : H;
      const BBwdWs ws = carve_bbwd((char*)workspace + per * l, T, B, std::max(F, H), H);
      if ((rc = sv_gemm_bf16_dual(4 * H, H, Fl, TBp, dgT[l], TBp, hT[l], ldhT, dw_hh[l], H, xT[l], ld_xT[l], dw_ih[l],
                                  Fl, ws.gws, main)))
        return rc;
      // layer l's gradients are complete: its all-reduce bucket (grad_ready) overlaps the lower
      // layers' weight-gradient GEMMs (the recurrences are all done)
      if (evs && (e = hipEventRecord(ev[L * nch + l], main)) != hipSuccess) return (int)e;
    }
    return SV_OK;
  }
  if (sched_persist(schedule, H) && sv_persist_bwd_fits(B, H, sv_stream_cus(main))) {
    if (!sync) return SV_EARG;
    // persistent schedule on `main`: per layer (top first) the whole-T recurrence in one launch
    // (sv_persist.hip; bias gradients summed in the kernel), the whole-T dx GEMM straight from its
    // fragment-order hand-off, then the layer's weight gradients (measured: on a side stream
    // beside the next layer's recurrence 16.8 vs 16.6 ms at c3 -- the GEMM workgroups contend
    // with the co-resident recurrence)
    {  // every layer's W_hh^T / W_ih^T (bf16) in one launch
      std::vector<const bf16_t*> whhT_l(L), wihT_l(L);  // any L (wbf_transposes batches 8 at a time)
      for (int l = 0; l < L; ++l) {
        const BBwdWs ws = carve_bbwd((char*)workspace + per * l, T, B, std::max(F, H), H);
        whhT_l[l] = ws.whhT;
        wihT_l[l] = l > 0 ? ws.wihT : nullptr;
      }
      if (int rc = wt_ready ? 0 : wbf_transposes(L, F, H, w_ih, w_hh, whhT_l.data(), wihT_l.data(), main)) return rc;
    }
    // the weight gradients of every layer after the last recurrence, as the layer wavefront's one
    // whole-K launch (plan_fullk), where it applies; else per layer, split-K, after its recurrence
    G8Full f;
    int fP;
    const bool fullk = SV_PERSIST_FULLK && plan_fullk(f, fP);
    if (fullk && f.S > 0 && !cnt_ready) {  // the first pieces' flags (else zeroed by the forward)
      if (int rc = sv_zero_counters(f.flag, 1, 0, fP, main)) return rc;
    }
    for (int l = L - 1; l >= 0; --l) {
      const int Fl = l == 0 ? F : H;
      const BBwdWs ws = carve_bbwd((char*)workspace + per * l, T, B, std::max(F, H), H);
      int rc = 0;
      const float* up = l == L - 1 ? dh_last : dx[l + 1];
      bf16_t* dgf = (bf16_t*)((char*)workspace + per * L);
      const bool afr = l > 0 && gemm_afrag_ok(T, B, Fl, H);  // dx reads dgf: no row-major dG
      // layer l on channel SV_BWD_CH0 + l, pre-zeroed by the forward (cnt_ready) where the layers fit
      // the channels, else each launch zeroing its own
      const bool own = L <= SV_SYNC_CHANNELS - SV_BWD_CH0;
      // the bias-gradient finalize rides on the next launch (the dx GEMM; layer 0's: the whole-K
      // weight-gradient launch), before the next recurrence reuses the partials' slots in dgf
      DbFin fin{};
      if ((rc = sv_persist_bwd_bf16(T, B, H, ws.whhT, gates[l], c_tm[l], up, l < L - 1,
                                    (afr || l == 0) ? nullptr : dg[l],  // layer 0 has no dx GEMM
                                    dgT[l], dgf, main, sync, db_ih[l], db_hh ? db_hh[l] : nullptr,
                                    probe ? probe[2 * l] : nullptr, probe ? probe[2 * l + 1] : nullptr,
                                    SV_BWD_CH0 + (own ? l : 0), own && cnt_ready, &fin)))
        return rc;
      // the completion events of layers >= 1 (grad_ready: a caller's bucketed all-reduce) fire once
      // the last recurrence is done, so collectives never share the device with a persistent launch
      // (whose grid must be co-resident; a concurrent RCCL kernel would hold CUs it waits for) but
      // overlap layer 0's weight-gradient GEMMs
      for (int k = 1; l == 0 && k < L && evs && !fullk; ++k)
        if ((e = hipEventRecord(ev[L * nch + k], main)) != hipSuccess) return (int)e;
      if (afr) {
        if ((rc = gemm_bf16_afrag(T, B, H, Fl, dgf, sv_persist_bm(B, H, sv_stream_cus(main)), ws.wihT, bf16_wiht_ld(H), dx[l],
                                  Fl, ws.gws, main, fin)))
          return rc;
      } else if (l == 0 && fullk) {
        f.fin = fin;
      } else {
        if ((rc = sv_dbfin_launch(fin, main))) return rc;
        if (l > 0 && (rc = sv_gemm_bf16(T * B, Fl, 4 * H, dg[l], 4L * H, ws.wihT, bf16_wiht_ld(H), dx[l], Fl, nullptr,
                                        nullptr, 0.f, ws.gws, main)))
          return rc;
      }
      if (fullk) continue;
      // dW_hh and dW_ih in one pass over dG^T (falls back to two GEMMs for layer 0's F = 40)
      rc = sv_gemm_bf16_dual(4 * H, H, Fl, TBp, dgT[l], TBp, hT[l], ldhT, dw_hh[l], H, xT[l], ld_xT[l], dw_ih[l], Fl,
                             ws.gws, main);
      if (rc) return rc;
    }
    if (fullk) return run_fullk(f, fP);
    if (evs && (e = hipEventRecord(ev[L * nch], main)) != hipSuccess) return (int)e;
    return SV_OK;
  }
  // per-step schedule, layer-pipelined (sv_lstm_stack_bwd, sv_lstm.hip): each layer on side[l]
  hipEvent_t ev_start = ev[L * nch + L];
  if ((e = hipEventRecord(ev_start, main)) != hipSuccess) return (int)e;
  const dim3 grid((H + BF_U - 1) / BF_U, (B + BF_BM - 1) / BF_BM);
  for (int l = L - 1; l >= 0; --l) {
    hipStream_t s = side[l];
    const int Fl = l == 0 ? F : H;
    const BBwdWs ws = carve_bbwd((char*)workspace + per * l, T, B, std::max(F, H), H);
    if ((e = hipStreamWaitEvent(s, ev_start, 0)) != hipSuccess) return (int)e;
    int rc = wt_ready ? 0 : sv_transpose_cast_bf16(w_hh[l], H, 4 * H, H, ws.whhT, 4L * H, s);
    if (rc) return rc;
    if (!wt_ready && l > 0 && (rc = sv_transpose_cast_bf16(w_ih[l], Fl, 4 * H, Fl, ws.wihT, bf16_wiht_ld(H), s)))
      return rc;
    if (Bp != B && (e = sv_memset0(dgT[l], (size_t)4 * H * TBp * sizeof(bf16_t), s)) != hipSuccess)
      return (int)e;
    for (int c = nch - 1; c >= 0; --c) {
      const int t0 = c * chunk, t1 = std::min(T, t0 + chunk);
      if (l < L - 1 && (e = hipStreamWaitEvent(s, ev[(l + 1) * nch + c], 0)) != hipSuccess) return (int)e;
      for (int t = t1 - 1; t >= t0; --t) {
        const float* up = (l == L - 1) ? (t == T - 1 ? dh_last : nullptr) : dx[l + 1] + t * BH;
        float* dcf_out = (t & 1) ? ws.dcf1 : ws.dcf0;
        const float* dcf_in = (t == T - 1) ? nullptr : ((t & 1) ? ws.dcf0 : ws.dcf1);
        launch_bwd_bf16(grid, s, t == T - 1 ? nullptr : dg[l] + (t + 1) * BG, ws.whhT, up, dcf_in, gates[l] + t * BG,
                        c_tm[l] + t * BH, t ? c_tm[l] + (t - 1) * BH : nullptr, dg[l] + t * BG, dcf_out, dgT[l],
                        (long)TBp, t, Bp, B, H);
        SV_LAUNCH_CHECK();
      }
      if (l > 0) {
        rc = sv_gemm_bf16((t1 - t0) * B, Fl, 4 * H, dg[l] + t0 * BG, 4L * H, ws.wihT, bf16_wiht_ld(H),
                          dx[l] + (long)t0 * B * Fl, Fl, nullptr, nullptr, 0.f, ws.gws, s);
        if (rc) return rc;
      }
      if ((e = hipEventRecord(ev[l * nch + c], s)) != hipSuccess) return (int)e;
    }
    rc = sv_gemm_bf16(4 * H, H, TBp, dgT[l], TBp, hT[l], ldhT, dw_hh[l], H, nullptr, nullptr, 0.f, ws.gws, s);
    if (rc) return rc;
    rc = sv_gemm_bf16(4 * H, Fl, TBp, dgT[l], TBp, xT[l], ld_xT[l], dw_ih[l], Fl, nullptr, nullptr, 0.f, ws.gws, s);
    if (rc) return rc;
    hipLaunchKernelGGL(rowsum_bf16_kernel, dim3(4 * H), dim3(256), 0, s, dgT[l], (long)TBp, TBp, db_ih[l],
                       db_hh ? db_hh[l] : nullptr);
    SV_LAUNCH_CHECK();
    if ((e = hipEventRecord(ev[L * nch + l], s)) != hipSuccess) return (int)e;
  }
  for (int l = 0; l < L; ++l)
    if ((e = hipStreamWaitEvent(main, ev[L * nch + l], 0)) != hipSuccess) return (int)e;
  return SV_OK;
}
