// Persistent recurrences: one launch runs all T timesteps of one LSTM layer.
//
// Why: a per-step launch pays a kernel boundary, a grid fill/drain and a cold-L2 start (TCC
// misses per bf16 step launch ~ the per-XCD W_hh + h footprint).  Here each workgroup keeps the
// same (row block, unit block) tile for the whole sequence: its W_hh slice stays in the XCD's
// L2, its cell state stays in registers, and only h_{t-1} crosses workgroups.  Selected by
// (see persist_fwd() in sv_bf16.hip for when the stack forward uses it).
//
// Hand-off of h between timesteps (MI355X_MICROARCH.md, inter-workgroup visibility, hand-off
// table row 1): every store of the handed-off bytes (h_bf[t+1], 4-B packed pairs) is an `sc1`
// write-through store, every storing wave drains with s_waitcnt vmcnt(0), a workgroup barrier
// follows, then ONE lane adds 1 to its row block's agent-scope counter.  A consumer's lane 0
// polls that counter with `sc1` loads until all producers of its row block have arrived for the
// step, the workgroup barrier releases the other waves, and every load of h_bf is a
// buffer_load_dwordx4 `sc1`.  Each h_bf slot is written once per launch (slot t+1 at step t).
//
// Residency: the grid must be co-resident (one workgroup per CU at most), which the host checks
// against the CU count of the stream's device; the spin is bounded: a timeout sets the sticky
// status word of the caller's sync block (sv_sync_size, include/sv_ge2e.h) and every later wait
// on that block returns at once, so the launch drains instead of hanging, and the caller sees
// the status (the trainer raises and its clip + SGD kernel skips the update).  Counters and
// status live in the caller's block, not in device globals: calls with different blocks may
// run concurrently; launches sharing one block (the layers of a stack call) are serialised on
// one stream.
#include <algorithm>
#include <atomic>
#include "sv_bf16.h"
#include "../../include/sv_ge2e.h"

#include "sv_persist_dev.h"

// A-operand tile of a handed-off buffer: [R][BK] bf16 rows (row stride ld elements) read with
// buffer_load_dwordx4 sc1 (bypasses the CU's L1, L2-served; rows past the buffer end read 0)
template <int R, int NT, int BK>
struct BTileStageSC1 {
  static constexpr int LD = BK + 8;
  static constexpr int C8 = BK / 8;
  static constexpr int NV = (R * C8) / NT;
  static_assert(NV >= 1 && NV * NT == R * C8, "tile/thread mismatch");
  uint4 v[NV];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int row0, int ld, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      const int r = q / C8, c = (q % C8) * 8;
      const unsigned off = ((unsigned)(row0 + r) * (unsigned)ld + (unsigned)(k0 + c)) * 2u;
      const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */);
      v[i] = (k0 + c < K) ? uint4{x.x, x.y, x.z, x.w} : uint4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      *reinterpret_cast<uint4*>(lds + (q / C8) * LD + (q % C8) * 8) = v[i];
    }
  }
};

// rolling-prefetch main loop (depth D) with the A operand from a handed-off buffer
template <int BM, int BN, int NT, int D, class MapB>
__device__ __forceinline__ void persist_mainloop(__amdgpu_buffer_rsrc_t ra, int row0, int lda,
                                                 const bf16_t* __restrict__ B, long ldb, const MapB& mapB, int K,
                                                 bf16_t* lds, int tid, int wm0, int wn0, f32x16 (&acc)[1][1]) {
  using SA = BTileStageSC1<BM, NT, BBK>;
  using SB = BTileStage<BN, NT, BBK>;
  constexpr int LD = BBK + 8;
  constexpr int BUF = (BM + BN) * LD;
  const int lane = tid & 63;
  const int nk = (K + BBK - 1) / BBK;
  SA sa[D];
  SB sb[D];
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nk) {
      sa[j].load(ra, row0, lda, j * BBK, K, tid);
      sb[j].load(B, ldb, mapB, j * BBK, K, tid);
    }
  for (int k0 = 0; k0 < nk; k0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int kt = k0 + j;
      if (kt < nk) {
        bf16_t* buf = lds + (kt & 1) * BUF;
        sa[j].store(buf, tid);
        sb[j].store(buf + BM * LD, tid);
        if (kt + D < nk) {
          sa[j].load(ra, row0, lda, (kt + D) * BBK, K, tid);
          sb[j].load(B, ldb, mapB, (kt + D) * BBK, K, tid);
        }
        __syncthreads();
        mfma_ktile_bf<1, 1, BBK, LD>(buf, buf + BM * LD, wm0, wn0, lane, acc);
      }
    }
  }
  __syncthreads();
}

// ============================================================================
// bf16 forward recurrence of one layer, all T steps.  Tile (b0, j0): 64 batch rows x 32
// units x 4 gates; 8 waves, one 32x32 accumulator each (as lstm_step_fwd_bf16_kernel).
//   gates [T,B,4H] bf16: in = bf16(x W_ih^T + b_ih + b_hh) (K1), out = bf16 activated i,f,g,o
//   c_tm [T,B,H], h_tm [T+1,B,H] (slot 0 = 0), h_bf [T+1,B,H] (slot 0 = 0, the hand-off),
//   hT [H,(T+1)Bp] or NULL.  cnt: this launch's zeroed row-block counters.
// ============================================================================
template <int D>
__global__ __launch_bounds__(512) void lstm_persist_fwd_bf16_kernel(const bf16_t* __restrict__ whh_bf,
                                                                    bf16_t* __restrict__ gates,
                                                                    float* __restrict__ c_tm,
                                                                    float* __restrict__ h_tm, bf16_t* h_bf,
                                                                    bf16_t* __restrict__ hT, long ldhT, int T,
                                                                    int Bp, int B, int H, unsigned* cnt,
                                                                    unsigned* status, unsigned limit, int fault,
                                                                    int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* ldsb = reinterpret_cast<bf16_t*>(smem);
  constexpr int BN = 4 * BF_U, LDP = BN + 4, LDH = BF_BM + 1;
  constexpr int PER = BF_BM * BF_U / 512;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.x * BF_U, b0 = blockIdx.y * BF_BM;
  const int wm0 = (w >> 2) * 32, wn0 = (w & 3) * 32;
  const long G = 4L * H, BH = (long)B * H;
  unsigned* my_cnt = cnt + blockIdx.y * SV_PCNT_STRIDE;
  const unsigned producers = gridDim.x;
  float cst[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) cst[k] = 0.f;
  float* pre = reinterpret_cast<float*>(smem);
  float* hs = pre + BF_BM * LDP;
  for (int t = 0; t < T; ++t) {
    bf16_t* gt = gates + (long)t * B * G;
    float xg[PER][4];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      const bool ok = gb < B && gj < H;
      const bf16_t* gp = gt + (long)gb * G + gj;
#pragma unroll
      for (int q = 0; q < 4; ++q) xg[k][q] = ok ? from_bf(gp[q * H]) : 0.f;
    }
    f32x16 acc[1][1];
    zero_acc(acc);
    if (t > 0 && !(dbg & 2)) {
      if (tid == 0 && !(dbg & 1)) persist_wait(my_cnt, producers * (unsigned)t, status, limit, 1u);
      __syncthreads();
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(h_bf + (long)t * BH, (unsigned)(BH * 2));
      persist_mainloop<BF_BM, BN, 512, D>(ra, b0, H, whh_bf, H, RowMapGates<BF_U>{j0, H}, H, ldsb, tid, wm0, wn0,
                                          acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) pre[(wm0 + acc_row(r, lane)) * LDP + wn0 + (lane & 31)] = acc[0][0][r];
    __syncthreads();
    float* ct = c_tm + (long)t * BH;
    float* ht = h_tm + (long)(t + 1) * BH;
    bf16_t* hb = h_bf + (long)(t + 1) * BH;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      const bool ok = gb < B && gj < H;
      const float* pr = pre + b * LDP + u;
      const float pv[4] = {pr[0], pr[BF_U], pr[2 * BF_U], pr[3 * BF_U]};
      float av[4], h;
      const float c = lstm_cell_fwd(pv, xg[k], cst[k], av, h);
      const float i = av[0], f = av[1], g = av[2], o = av[3];
      cst[k] = c;
      // h_bf hand-off: lanes (u, u+1) pair up, the even lane stores both as one 4-B sc1 store
      const unsigned hbits = to_bf(h);
      const unsigned nb = __shfl_down(hbits, 1, 64);
      if (ok) {
        bf16_t* gp = gt + (long)gb * G + gj;
        gp[0] = to_bf(i);
        gp[H] = to_bf(f);
        gp[2 * H] = to_bf(g);
        gp[3 * H] = to_bf(o);
        ct[(long)gb * H + gj] = c;
        ht[(long)gb * H + gj] = h;
        if (!(u & 1))
          __hip_atomic_store(reinterpret_cast<unsigned*>(hb + (long)gb * H + gj), hbits | (nb << 16),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      hs[u * LDH + b] = h;
    }
    __syncthreads();
    if (hT) {
      for (int e = tid; e < BF_BM * BF_U; e += 512) {
        const int u = e / BF_BM, b = e % BF_BM;
        const int gb = b0 + b, gj = j0 + u;
        if (gb >= B || gj >= H) continue;
        bf16_t* row = hT + (long)gj * ldhT;
        row[(long)(t + 1) * Bp + gb] = to_bf(hs[u * LDH + b]);
        if (t == 0) row[gb] = 0;
      }
    }
    // publish: every wave drains its stores, barrier, one lane arrives on the row block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && persist_arrive_ok(fault, t == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ============================================================================
// W-stationary variant (H = 16 NS): 4 waves, wave g owns gate g of the tile's 32 units for all
// 64 rows (two 32x32 accumulators) and keeps its W_hh rows -- 32 x H bf16, the MFMA B
// fragments of every k-step -- in registers for the whole sequence.  Per step only h_{t-1}
// (64 rows x H) is staged into LDS (two halves of sc1 buffer loads); each wave reads it as A
// fragments: 1 LDS fragment per MFMA instead of 2, no W traffic at all after the prologue.
// Epilogue: each thread owns 4 consecutive units of 2 rows (16-B operand loads and stores);
// only the h_bf hand-off (16-B sc1 stores from an LDS-staged tile) precedes the arrival, the
// activations, c, h and hT (16-B transposed chunks) are stored after it.
// ============================================================================
// XF > 0 (layer 0, F = 8 * XF <= 48 input features): the input projection x_t W_ih^T + b_ih + b_hh
// is computed in the kernel from x_bf [T,B,F] and W_ih [4H,F] (held in registers beside W_hh:
// 3 k-steps of 16, zero-padded), so the layer needs no K1 GEMM and its step loads 80 B per row
// instead of 4 x 4H fp32 pre-activations; the sum (MFMA over the zero-padded k range, then the
// two biases, rounded to bf16 as the K1 GEMM stores it) matches the K1 path bit for bit.
template <int NS, int BM, int XF>
__global__ __launch_bounds__(256, 1) void lstm_persist2_fwd_bf16_kernel(const bf16_t* __restrict__ whh_bf,
                                                                       bf16_t* __restrict__ gates,
                                                                       float* __restrict__ c_tm,
                                                                       float* __restrict__ h_tm, bf16_t* h_bf,
                                                                       bf16_t* __restrict__ hT, long ldhT, int T,
                                                                       int Bp, int B, int H, unsigned* cnt, int nub,
                                                                       int xcd, unsigned* status, unsigned limit,
                                                                       int fault, int pipe,
                                                                       const bf16_t* __restrict__ x_bf,
                                                                       const bf16_t* __restrict__ wih_bf,
                                                                       const float* __restrict__ b_ih,
                                                                       const float* __restrict__ b_hh) {
  if (!SV_PDBG) pipe = 1;  // (the non-pipelined k-loop: A/B builds only)
  constexpr int K = NS * 16, LDA = K + 8, HALF = NS / 2 * 16;
  constexpr int LDP = 4 * BF_U + 4;      // pre [BM][LDP] fp32
  constexpr int LDB = BF_U + 8;          // hsb [BM][LDB] bf16 (h tile, row-major)
  constexpr int LDT = BM + 8;            // hts [32][LDT] bf16 (h tile, transposed)
  constexpr int KR = BM / 32;            // 32-row halves of the tile (rows per thread)
  static_assert(NS % 2 == 0, "two staging halves");
  static_assert(BM == 32 || BM == 64, "row tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);                          // [BM][LDA]
  float* pre = reinterpret_cast<float*>(smem + BM * LDA * 2);            // [BM][LDP]
  bf16_t* hsb = reinterpret_cast<bf16_t*>(pre + BM * LDP);               // [BM][LDB]
  bf16_t* hts = hsb + BM * LDB;                                          // [32][LDT]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * BF_U, b0 = rb * BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  // this wave's W_hh fragments: B[k][n] = W[g H + j0 + n][k], lane (n = r, k = 16 s + 8 hh .. +7)
  bf16x8_t wreg[NS];
  {
    const bool wok = j0 + r < H;
    const bf16_t* wrow = whh_bf + ((long)g * H + j0 + r) * K + 8 * hh;
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      bf16x8_t z = {};
      wreg[s2] = wok ? *reinterpret_cast<const bf16x8_t*>(wrow + 16 * s2) : z;
    }
    // the weights live in AGPRs (MFMA reads B from them directly): the VGPRs stay free for the
    // x-projection prefetch and the A-fragment ring of the recurrent MFMAs
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) asm volatile("" : "+a"(wreg[s2]));
  }
  // fused input projection (XF > 0): W_ih fragments of this wave's 32 gate columns (k = 16 s +
  // 8 hh .. +7, zero past F = 8 XF) and the column's bias b_ih + b_hh
  constexpr int XS = (XF + 1) / 2;  // k-steps of 16
  constexpr int F = 8 * XF;
  bf16x8_t wx[XS > 0 ? XS : 1];
  float xbias = 0.f;
  if constexpr (XF > 0) {
    const int col = g * H + j0 + r;
    const bool wok = j0 + r < H;
#pragma unroll
    for (int s2 = 0; s2 < XS; ++s2) {
      bf16x8_t z = {};
      wx[s2] = (wok && 16 * s2 + 8 * hh < F) ? *reinterpret_cast<const bf16x8_t*>(wih_bf + (long)col * F + 16 * s2 + 8 * hh)
                                             : z;
    }
    if (wok) {
      if (b_ih) xbias += b_ih[col];
      if (b_hh) xbias += b_hh[col];
    }
  }
  // x_t A fragments (rows b0 + r (+32), k = 16 s + 8 hh), prefetched a step ahead; rows past B
  // and k past F read zeros
  u32x4_t xa[XS > 0 ? XS : 1][BM / 32];
  auto load_x = [&](int tt) {
    if constexpr (XF > 0) {
      const __amdgpu_buffer_rsrc_t rxs = sv_rsrc(x_bf + (long)tt * B * F, (unsigned)((long)B * F * 2));
#pragma unroll
      for (int s2 = 0; s2 < XS; ++s2)
#pragma unroll
        for (int m = 0; m < BM / 32; ++m) {
          const unsigned off = 16 * s2 + 8 * hh < F ? ((unsigned)(b0 + 32 * m + r) * (unsigned)F + 16 * s2 + 8 * hh) * 2u
                                                    : 0xFFFFFFF0u;
          xa[s2][m] = __builtin_amdgcn_raw_buffer_load_b128(rxs, off, 0, 0);
        }
    }
  };
  // elementwise map: thread -> 4 consecutive units (u4) x rows brow (+ 32)
  const int u4 = (tid & 7) * 4, brow = tid >> 3;
  const long Bv = B;
  float cst[KR][4];
#pragma unroll
  for (int k = 0; k < KR; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v) cst[k][v] = 0.f;
  // staging map of one half (BM rows x HALF bf16 = BM * HALF / 8 16-B chunks over 256 threads)
  constexpr int CH = BM * HALF / 8 / 256;
  // bf16(x W_ih^T + b) of step t (K1 output): 8-B buffer loads of 4 units, rows past B read zeros
  uint2 xg[KR][4];
  auto load_xg = [&](int tt) {
    if constexpr (XF > 0) {
      load_x(tt);
      return;
    }
    const __amdgpu_buffer_rsrc_t rx = sv_rsrc(gates + (long)tt * BG, (unsigned)(BG * 2));
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + brow + 32 * k;
      const long gbv = gb < Bv ? gb : Bv + 64;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x2_t x = __builtin_amdgcn_raw_buffer_load_b64(rx, (unsigned)((gbv * G + q * H + j0 + u4) * 2), 0, 0);
        xg[k][q] = uint2{x.x, x.y};
      }
    }
  };
  for (int t = 0; t < T; ++t) {
    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
    if (t > 0) {
      if (tid == 0) persist_wait(my_cnt, producers * (unsigned)t, status, limit, 1u);
      __syncthreads();
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(h_bf + (long)t * BH, (unsigned)(BH * 2));
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        uint4 v[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {  // chunk q: row q / (HALF/8), column chunk q % (HALF/8)
          const int q = tid + 256 * i, row = q / (HALF / 8), c = (q % (HALF / 8)) * 8 + half * HALF;
          const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(
              ra, ((unsigned)(b0 + row) * (unsigned)H + (unsigned)c) * 2u, 0, 16 /* sc1 */);
          v[i] = uint4{x.x, x.y, x.z, x.w};
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int q = tid + 256 * i, row = q / (HALF / 8), c = (q % (HALF / 8)) * 8 + half * HALF;
          *reinterpret_cast<uint4*>(As + row * LDA + c) = v[i];
        }
      }
      __syncthreads();
      // this step's x-projection, in flight behind the recurrent MFMAs (which read only LDS);
      // loaded in the step that uses it, so it is no loop-carried register set (those were
      // copied right after the loads, exposing the whole round trip)
      load_xg(t);
      __builtin_amdgcn_sched_barrier(0);
      if (pipe) {  // A fragments P k-steps ahead of the MFMAs (sv_bf16.h)
        f32x16 accs[KR];
        accs[0] = acc0;
        if constexpr (BM == 64) accs[KR - 1] = acc1;
        mfma_lds_pipe<NS, KR, (BM == 64 ? 3 : 4)>(As + r * LDA + 8 * hh, 32 * LDA, wreg, accs);
        acc0 = accs[0];
        if constexpr (BM == 64) acc1 = accs[KR - 1];
      } else {
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
          const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(As + r * LDA + 16 * s2 + 8 * hh);
          acc0 = mfma_bf16(a0, wreg[s2], acc0);
          if constexpr (BM == 64) {
            const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(As + (32 + r) * LDA + 16 * s2 + 8 * hh);
            acc1 = mfma_bf16(a1, wreg[s2], acc1);
          }
        }
      }
    } else {
      load_xg(0);
    }
    if constexpr (XF > 0) {  // pre-activation = recurrent part + (x_t W_ih^T + b_ih + b_hh)
      f32x16 x0, x1;
#pragma unroll
      for (int i = 0; i < 16; ++i) x0[i] = x1[i] = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < XS; ++s2) {
        x0 = mfma_bf16(__builtin_bit_cast(bf16x8_t, xa[s2][0]), wx[s2], x0);
        if constexpr (BM == 64) x1 = mfma_bf16(__builtin_bit_cast(bf16x8_t, xa[s2][1]), wx[s2], x1);
      }
      add_round_bf16x(acc0, x0, xbias);
      if constexpr (BM == 64) add_round_bf16x(acc1, x1, xbias);
    }
    // gate exchange: wave g's [BM rows][32 units] -> pre[row][g * 32 + unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pre[acc_row(i, lane) * LDP + g * BF_U + r] = acc0[i];
      if constexpr (BM == 64) pre[(32 + acc_row(i, lane)) * LDP + g * BF_U + r] = acc1[i];
    }
    __syncthreads();
    uint2 act[KR][4];
    float4 cv[KR], hv[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = brow + 32 * k;
      float4 pq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pq[q] = *reinterpret_cast<const float4*>(pre + b * LDP + q * BF_U + u4);
      float ao[4][4], co[4], ho[4];
      unsigned pk[2] = {0u, 0u};
      float4 xf[4];
      if constexpr (XF == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) xf[q] = unpack_bf4(xg[k][q]);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float pv[4] = {pq[0][v], pq[1][v], pq[2][v], pq[3][v]};
        float xv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (XF == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) xv[q] = xf[q][v];
        }
        float a4[4], h;
        const float c = lstm_cell_fwd(pv, xv, cst[k][v], a4, h);
        cst[k][v] = c;
#pragma unroll
        for (int q = 0; q < 4; ++q) ao[q][v] = a4[q];
        co[v] = c;
        ho[v] = h;
      }
      pk[0] = pack_bf2(ho[0], ho[1]);
      pk[1] = pack_bf2(ho[2], ho[3]);
#pragma unroll
      for (int v = 0; v < 4; ++v) hts[(u4 + v) * LDT + b] = (bf16_t)(pk[v >> 1] >> (16 * (v & 1)));
      *reinterpret_cast<uint2*>(hsb + b * LDB + u4) = uint2{pk[0], pk[1]};
#pragma unroll
      for (int q = 0; q < 4; ++q) act[k][q] = pack_bf4(ao[q][0], ao[q][1], ao[q][2], ao[q][3]);
      cv[k] = float4{co[0], co[1], co[2], co[3]};
      hv[k] = float4{ho[0], ho[1], ho[2], ho[3]};
    }
    __syncthreads();  // hsb, hts complete
    // the hand-off: h_t bf16, BM rows x 4 chunks of 8 units, 16-B sc1 stores
    {
      const int row = tid >> 2, c = tid & 3, gb = b0 + row;
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(h_bf + (long)(t + 1) * BH, (unsigned)(BH * 2));
      if (row < BM && gb < B && j0 + 8 * c < H) {
        const uint4 v = *reinterpret_cast<const uint4*>(hsb + row * LDB + 8 * c);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw,
                                               ((unsigned)gb * (unsigned)H + (unsigned)(j0 + 8 * c)) * 2u, 0,
                                               16 /* sc1 */);
      }
    }
    // publish h_t: the hand-off stores drained, barrier, one lane arrives
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && persist_arrive_ok(fault, t == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // off the critical chain: activations, c, h and hT of step t
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + brow + 32 * k;
      if (gb < Bv) {
        bf16_t* gp = gates + (long)t * BG + gb * G + j0 + u4;
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(gp + q * H) = act[k][q];
        *reinterpret_cast<float4*>(c_tm + (long)t * BH + gb * H + j0 + u4) = cv[k];
        // fp32 h: only h_{T-1} is read (the projection); the next layer and the backward take
        // the bf16 copies
        if (t == T - 1) *reinterpret_cast<float4*>(h_tm + (long)(t + 1) * BH + gb * H + j0 + u4) = hv[k];
      }
    }
    if (hT) {  // 32 unit rows x BM/8 chunks of 8 batch columns (padding columns get zeros)
      constexpr int CPR = BM / 8;
      const int u = tid / CPR, c = tid % CPR, gb = b0 + 8 * c;
      if (u < BF_U && gb < Bp && j0 + u < H) {
        bf16_t* row = hT + (long)(j0 + u) * ldhT;
        *reinterpret_cast<uint4*>(row + (long)(t + 1) * Bp + gb) = *reinterpret_cast<const uint4*>(hts + u * LDT + 8 * c);
        if (t == 0) *reinterpret_cast<uint4*>(row + gb) = uint4{0u, 0u, 0u, 0u};
      }
    }
  }
}

// ============================================================================
// W-stationary backward recurrence of one layer (reverse time, all T steps).  Tile (b0, j0):
// 64 batch rows x 32 hidden units.  Wave g owns gate g's K range of the recurrent product
//   dh_rec[b][j] = sum_g sum_k dG_{t+1}[b][g H + k] * W_hh[g H + k][j]
// and keeps its W_hh slice (K = H rows x 32 units, the MFMA B fragments of every k-step) in
// registers for the whole sequence.  Each wave's A operand (64 rows x H of dG_{t+1}, used by no
// other wave of the workgroup) streams from the hand-off buffer straight into registers, P
// fragment pairs in flight.  The hand-off buffer `dgf` holds dG in MFMA A-fragment order --
// [slot t][row block][gate][row half][k-step][lane][8] -- so every wave load instruction reads
// one contiguous KB (row-major rows would give 32-B pieces of 32 rows per instruction, which
// measured at under a third of the CU's L2 read rate).  The four per-gate partials meet in LDS
// and are summed in gate order 0..3 (the per-step kernel's order, each gate accumulated over k
// in one accumulator as there), so results are bit-identical to lstm_step_bwd_bf16_kernel.
// dc * f (the cell-gradient carry) and c_{t-1} stay in registers; the elementwise operands of
// step t-1 load as 16-B vectors right after step t's arrival.  Only the hand-off stores precede
// the arrival; dG_t row-major (the dx GEMM's operand, skipped when the dx GEMM reads dgf) and
// transposed (dgT, the dW GEMMs') are stored after it.
//   acts [T,B,4H] bf16 activated gates, c_tm [T,B,H]; dhup: [T,B,H] (up_full) or [B,H] at t = T-1.
// Hand-off: hand-off table row 1 of MI355X_MICROARCH.md, as the forward kernel above.
// ============================================================================
template <int NS, int P, int BM, bool agpr_w = true, bool EWD = true>
__global__ __launch_bounds__(256, 1) void lstm_persist2_bwd_bf16_kernel(
    const bf16_t* __restrict__ whhT, const bf16_t* __restrict__ acts, const float* __restrict__ c_tm,
    const float* __restrict__ dhup, int up_full, bf16_t* __restrict__ dg, bf16_t* __restrict__ dgT, long lddgT,
    bf16_t* dgf, int T, int Bp, int B, int H, unsigned* cnt, int nub, int xcd, unsigned* status, unsigned limit,
    int fault, int dbg, float* __restrict__ dbp, unsigned long long* __restrict__ stamps) {
  dbg &= SV_PDBG;
  constexpr int LDR = BF_U + 4;          // red [4][BM][LDR] fp32 (16-B aligned rows)
  constexpr int LDG = 4 * BF_U + 8;      // dgs [BM][LDG] bf16 (row-major dG tile)
  constexpr int LDT = BM + 8;            // gts [128][LDT] bf16 (transposed dG tile)
  constexpr int FRAG = NS * 64 * 8;      // dgf elements of one (row block, gate, row half)
  constexpr int KR = BM / 32;            // 32-row halves of the tile
  static_assert(P >= 1 && P <= NS, "prefetch depth");
  static_assert(BM == 32 || BM == 64, "row tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);
  bf16_t* dgs = reinterpret_cast<bf16_t*>(smem + 4 * BM * LDR * 4);
  bf16_t* gts = dgs + BM * LDG;
  // step operands staged by LDS-DMA (EWD): activations [BM][16 x 16 B] (gate blocks rotated by
  // row), c_{t-1} and dh_up [BM][32] fp32
  char* ewa = reinterpret_cast<char*>(gts + 4 * BF_U * LDT);
  float* ewc = reinterpret_cast<float*>(ewa + BM * 256);
  float* ewu = ewc + BM * BF_U;
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * BF_U, b0 = rb * BM;
  const int nrb = gridDim.x / nub;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  const long FS = (long)nrb * BM * G;  // dgf slot (elements)
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  // W_hh fragments of gate g: B[k][n] = W_hh[g H + k][j0 + n] = whhT[j0 + n][g H + k]
  bf16x8_t wreg[NS];
  {
    const bool wok = j0 + r < H;
    const bf16_t* wrow = whhT + (long)(j0 + r) * G + (long)g * H + 8 * hh;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      bf16x8_t z = {};
      wreg[s] = wok ? *reinterpret_cast<const bf16x8_t*>(wrow + 16 * s) : z;
    }
    if (agpr_w) {  // weights in AGPRs (MFMA B operand): VGPRs free for the A stream and operands
#pragma unroll
      for (int s = 0; s < NS; ++s) asm volatile("" : "+a"(wreg[s]));
    }
  }
  // elementwise map: thread -> 4 consecutive units (u4) x rows brow, brow + 32
  const int u4 = (tid & 7) * 4, brow = tid >> 3;
  uint2 av[KR][4];  // 4 units of each gate, bf16
  float4 cv[KR], cpv[KR], upv[KR];
  float dcf[KR][4];
  // bias-gradient partial sums over t of this thread's bf16 dG values (dbp: per row block)
  float dbs[KR][4][4];
#pragma unroll
  for (int k = 0; k < KR; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) dbs[k][q][v] = 0.f;
  // step tt's operands except c_tt (carried): 16-B buffer loads, rows past B read zeros (offsets
  // beyond the slice's range), as do absent operands (zero-size ranges)
  auto ld4 = [](__amdgpu_buffer_rsrc_t rs, long off_elems) {
    const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(off_elems * 4), 0, 0);
    return float4{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
  };
  const long Bv = B;
  // EWD: step tt's operands into LDS by buffer_load ... lds (no destination registers, so the
  // issuing wave does not wait for them; rows past B and absent operands read zeros).  Wave g's
  // instruction j stages 1 KB at LDS position p = (g * n + j) * 64 + lane (16-B units):
  //   acts: row p / 16, slot s = p % 16 holds gate ((s / 4) - row) & 3, 8-unit chunk s % 4
  //   c_{t-1}, dh_up: row p / 8, 4-unit chunk p % 8
  auto load_ew_lds = [&](int tt) {
    const float* up = dhup ? (up_full ? dhup + (long)tt * BH : (tt == T - 1 ? dhup : nullptr)) : nullptr;
    const __amdgpu_buffer_rsrc_t ra_ = sv_rsrc(acts + (long)tt * BG, (unsigned)(BG * 2));
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(c_tm + (long)(tt > 0 ? tt - 1 : 0) * BH, tt > 0 ? (unsigned)(BH * 4) : 0u);
    const __amdgpu_buffer_rsrc_t ru_ = sv_rsrc(up ? up : c_tm, up ? (unsigned)(BH * 4) : 0u);
    constexpr int NA = BM / 16, NC = BM / 32;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int p = (g * NA + j) * 64 + lane, row = p >> 4, sl = p & 15;
      const int q = ((sl >> 2) - row) & 3, c = sl & 3;
      const long gb = b0 + row, gbv = gb < Bv ? gb : Bv + 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (lds_ptr_t)(ewa + (g * NA + j) * 1024), 16,
                                               (unsigned)((gbv * G + q * H + j0 + 8 * c) * 2), 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int p = (g * NC + j) * 64 + lane, row = p >> 3, c = p & 7;
      const long gb = b0 + row, gbv = gb < Bv ? gb : Bv + 64;
      const unsigned off = (unsigned)((gbv * H + j0 + 4 * c) * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rc_, (lds_ptr_t)((char*)ewc + (g * NC + j) * 1024), 16, off, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ru_, (lds_ptr_t)((char*)ewu + (g * NC + j) * 1024), 16, off, 0, 0, 0);
    }
  };
  auto load_ew = [&](int tt) {
    if (EWD) {
      load_ew_lds(tt);
      return;
    }
    const float* up = dhup ? (up_full ? dhup + (long)tt * BH : (tt == T - 1 ? dhup : nullptr)) : nullptr;
    const __amdgpu_buffer_rsrc_t ra_ = sv_rsrc(acts + (long)tt * BG, (unsigned)(BG * 2));
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(c_tm + (long)(tt > 0 ? tt - 1 : 0) * BH, tt > 0 ? (unsigned)(BH * 4) : 0u);
    const __amdgpu_buffer_rsrc_t ru_ = sv_rsrc(up ? up : c_tm, up ? (unsigned)(BH * 4) : 0u);
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + brow + 32 * k;
      const long gbv = gb < Bv ? gb : Bv + 64;  // rows past B: offsets past every range
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x2_t x = __builtin_amdgcn_raw_buffer_load_b64(ra_, (unsigned)((gbv * G + q * H + j0 + u4) * 2), 0, 0);
        av[k][q] = uint2{x.x, x.y};
      }
      cpv[k] = ld4(rc_, gbv * H + j0 + u4);
      upv[k] = ld4(ru_, gbv * H + j0 + u4);
    }
  };
  {
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(c_tm + (long)(T - 1) * BH, (unsigned)(BH * 4));
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + brow + 32 * k;
      cv[k] = ld4(rc_, (gb < Bv ? gb : Bv + 64) * H + j0 + u4);
#pragma unroll
      for (int v = 0; v < 4; ++v) dcf[k][v] = 0.f;
    }
  }
  load_ew(T - 1);
  // phase stamps (dbg & 32): wait, GEMM + partial exchange, cell epilogue, hand-off + arrival,
  // post-arrival issue
  const bool stamp = dbg & 32;
  unsigned long long ph[5] = {0, 0, 0, 0, 0}, tlast = stamp ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {
    if (stamp) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      ph[i] += now - tlast;
      tlast = now;
    }
  };
  for (int t = T - 1; t >= 0; --t) {
    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
    if (t < T - 1 && !(dbg & 4)) {
      if (tid == 0 && !(dbg & 1)) persist_wait(my_cnt, producers * (unsigned)(T - 1 - t), status, limit, 2u);
      __syncthreads();
      mark(0);
      // A fragments of dG_{t+1}: (row half m, k-step s) is the KB at ((rb 4 + g) 2 + m) FRAG + s 512
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(dgf + (long)(t + 1) * FS, (unsigned)(FS * 2));
      constexpr unsigned kstep = 1024u;
      const unsigned base0 = ((unsigned)((rb * 4 + g) * KR) * (unsigned)FRAG + (unsigned)lane * 8u) * 2u;
      const unsigned base1 = base0 + (unsigned)FRAG * 2u;
      u32x4_t fa[P][2];
#pragma unroll
      for (int s = 0; s < P; ++s) {
        fa[s][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * s, 0, 16 /* sc1 */);
        if constexpr (BM == 64) fa[s][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, base1 + kstep * s, 0, 16);
      }
      // the scheduler would sink every load next to its MFMA (one exposed round trip per
      // k-step); scheduling barriers pin the P-deep software pipeline in program order
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        acc0 = mfma_bf16(__builtin_bit_cast(bf16x8_t, fa[s % P][0]), wreg[s], acc0);
        if constexpr (BM == 64) acc1 = mfma_bf16(__builtin_bit_cast(bf16x8_t, fa[s % P][1]), wreg[s], acc1);
        if (s + P < NS) {
          fa[s % P][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * (s + P), 0, 16);
          if constexpr (BM == 64)
            fa[s % P][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, base1 + kstep * (s + P), 0, 16);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // per-gate partials -> red[g][row][unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      red[(g * BM + acc_row(i, lane)) * LDR + r] = acc0[i];
      if constexpr (BM == 64) red[(g * BM + 32 + acc_row(i, lane)) * LDR + r] = acc1[i];
    }
    if (EWD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's operand DMA landed
    __syncthreads();
    mark(1);
    if (EWD) {  // step t's operands from the LDS image (every wave's DMA retired before the barrier)
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        const int b = brow + 32 * k;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          av[k][q] = *reinterpret_cast<const uint2*>(ewa + b * 256 + (((q + b) & 3) * 4 + (u4 >> 3)) * 16 + (u4 & 7) * 2);
        cpv[k] = *reinterpret_cast<const float4*>(ewc + b * BF_U + u4);
        upv[k] = *reinterpret_cast<const float4*>(ewu + b * BF_U + u4);
      }
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = brow + 32 * k;
      const float4 r0 = *reinterpret_cast<const float4*>(red + (0 * BM + b) * LDR + u4);
      const float4 r1 = *reinterpret_cast<const float4*>(red + (1 * BM + b) * LDR + u4);
      const float4 r2 = *reinterpret_cast<const float4*>(red + (2 * BM + b) * LDR + u4);
      const float4 r3 = *reinterpret_cast<const float4*>(red + (3 * BM + b) * LDR + u4);
      const float rs0[4] = {r0.x, r0.y, r0.z, r0.w}, rs1[4] = {r1.x, r1.y, r1.z, r1.w};
      const float rs2[4] = {r2.x, r2.y, r2.z, r2.w}, rs3[4] = {r3.x, r3.y, r3.z, r3.w};
      const float ups[4] = {upv[k].x, upv[k].y, upv[k].z, upv[k].w};
      const float cs[4] = {cv[k].x, cv[k].y, cv[k].z, cv[k].w}, cps[4] = {cpv[k].x, cpv[k].y, cpv[k].z, cpv[k].w};
      const float4 f0 = unpack_bf4(av[k][0]), f1 = unpack_bf4(av[k][1]), f2 = unpack_bf4(av[k][2]),
                   f3 = unpack_bf4(av[k][3]);
      const float a0[4] = {f0.x, f0.y, f0.z, f0.w};
      const float a1[4] = {f1.x, f1.y, f1.z, f1.w};
      const float a2[4] = {f2.x, f2.y, f2.z, f2.w};
      const float a3[4] = {f3.x, f3.y, f3.z, f3.w};
      unsigned pk[4][2];
      float dh4[4];  // (elementwise, the scalar order)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        dh4[v] = rs0[v];
        dh4[v] += rs1[v];
        dh4[v] += rs2[v];
        dh4[v] += rs3[v];
        dh4[v] += ups[v];
      }
      float ddv[4][4];
      lstm_cell_bwd_x4(dh4, a0, a1, a2, a3, cs, cps, dcf[k], ddv);
      pack_dg4(ddv, pk, dbs[k]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) gts[(q * BF_U + u4 + v) * LDT + b] = (bf16_t)(pk[q][v >> 1] >> (16 * (v & 1)));
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(dgs + b * LDG + q * BF_U + u4) = uint2{pk[q][0], pk[q][1]};
      cv[k] = cpv[k];  // c_{t-1} is the next step's c_t
    }
    __syncthreads();
    mark(2);
    // the hand-off: dG_t in fragment order, BM/4 KB per workgroup as contiguous KB pieces
    // (gate, row half, k-step), 16-B sc1 stores (dbg & 8, profiling only: no global stores)
    if (!(dbg & 8)) {
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(dgf + (long)t * FS, (unsigned)(FS * 2));
#pragma unroll
      for (int i = 0; i < 2 * KR; ++i) {
        const int p = tid + 256 * i, c = p >> 6, l = p & 63;
        const int gq = c / (2 * KR), m = (c >> 1) % KR, sl = c & 1;
        const uint4 v = *reinterpret_cast<const uint4*>(dgs + (32 * m + (l & 31)) * LDG + gq * BF_U + 16 * sl +
                                                        8 * (l >> 5));
        const unsigned off =
            ((unsigned)((rb * 4 + gq) * KR + m) * (unsigned)FRAG + (unsigned)(2 * ub + sl) * 512u + (unsigned)l * 8u) *
            2u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw, off, 0, 16 /* sc1 */);
      }
    }
    // publish dG_t: every store of the hand-off drained, barrier, one lane arrives.  With no
    // row-major dG: the dx GEMM reads the hand-off): the BM / 16 dG^T stores per thread (buffer
    // stores; a piece past Bp to a dropped offset) go out first, and the drain counts them
    // (vmcnt(BM / 16): this wave's older hand-off stores done; a raw barrier: __syncthreads' fence
    // would drain them)
    const bool ovl = !dbg && !dg && dgT && 4L * H * lddgT * 2 < (1L << 32) - 64;
    if (ovl) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // (the dG^T stores stay younger than the hand-off's)
      const __amdgpu_buffer_rsrc_t rt = sv_rsrc(dgT, (unsigned)(4L * H * lddgT * 2));
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
        const int q = tid + 256 * i, gu = q / (BM / 8), c = q % (BM / 8);
        const int gq = gu / BF_U, gj = j0 + gu % BF_U, gb = b0 + 8 * c;
        const uint4 v = *reinterpret_cast<const uint4*>(gts + gu * LDT + 8 * c);
        const unsigned off =
            gb < Bp && gj < H ? (unsigned)((((long)gq * H + gj) * lddgT + (long)t * Bp + gb) * 2) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rt, off, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(BM / 16) : "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (tid == 0 && persist_arrive_ok(fault, t == T - 1))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mark(3);
    // dG_t row-major (BM rows x 4 gates x 4 chunks of 8 units) and transposed (128 gate-unit
    // rows x BM/8 chunks of 8 batch columns; padding columns get zeros): 16-B plain stores
    // (dbg & 8, profiling only: skipped).  Before the operand DMA below: LDS reads issued behind
    // an LDS-DMA wait for it to land (the compiler puts vmcnt(0) before them)
    if (!(dbg & 8)) {
      bf16_t* dgt = dg ? dg + (long)t * BG : nullptr;  // NULL: the dx GEMM reads dgf itself
#pragma unroll
      for (int i = 0; i < BM / 16; ++i) {
        const int q = tid + 256 * i, row = q >> 4, gq = (q >> 2) & 3, c = q & 3;
        const int gb = b0 + row, gj = j0 + 8 * c;
        if (dgt && gb < B && gj < H)
          *reinterpret_cast<uint4*>(dgt + (long)gb * G + (long)gq * H + gj) =
              *reinterpret_cast<const uint4*>(dgs + row * LDG + gq * BF_U + 8 * c);
      }
      if (dgT && !ovl) {
#pragma unroll
        for (int i = 0; i < BM / 16; ++i) {
          const int q = tid + 256 * i, gu = q / (BM / 8), c = q % (BM / 8);
          const int gq = gu / BF_U, gj = j0 + gu % BF_U, gb = b0 + 8 * c;
          if (gb < Bp && gj < H)
            *reinterpret_cast<uint4*>(dgT + ((long)gq * H + gj) * lddgT + (long)t * Bp + gb) =
                *reinterpret_cast<const uint4*>(gts + gu * LDT + 8 * c);
        }
      }
    }
    // step t-1's elementwise operands, in flight during the next hand-off wait (dbg & 16,
    // profiling only: skipped)
    if (t > 0 && !(dbg & 16)) load_ew(t - 1);
    mark(4);
  }
  if (stamp && tid == 0 && blockIdx.x < SV_NSTAMP_WG)
    for (int i = 0; i < 5; ++i) stamps[blockIdx.x * SV_NSTAMP + i] = ph[i];
  // bias gradients: this tile's column sums (rows in order 0..BM-1), one partial per row block;
  // sv_persist_db_finalize adds the row blocks in order
  if (dbp) {
    __syncthreads();
    float* dsum = red;  // [BM][4 * BF_U] fp32 (fits in the red region)
#pragma unroll
    for (int k = 0; k < KR; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(dsum + (brow + 32 * k) * (4 * BF_U) + q * BF_U + u4) =
            float4{dbs[k][q][0], dbs[k][q][1], dbs[k][q][2], dbs[k][q][3]};
    __syncthreads();
    if (tid < 4 * BF_U) {
      const int q = tid / BF_U, gj = j0 + tid % BF_U;
      float sum = 0.f;
      for (int b = 0; b < BM; ++b) sum += dsum[b * (4 * BF_U) + tid];
      if (gj < H) dbp[(long)rb * G + (long)q * H + gj] = sum;
    }
  }
}

// db_ih = db_hh = sum over row blocks (in order) of the persistent backward's partials [nrb][G]
__global__ void persist_db_finalize_kernel(const float* __restrict__ dbp, int nrb, int G, float* __restrict__ db_ih,
                                           float* __restrict__ db_hh) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= G) return;
  float s = 0.f;
  for (int r = 0; r < nrb; ++r) s += dbp[(long)r * G + c];
  db_ih[c] = s;
  if (db_hh) db_hh[c] = s;
}

// the same for up to 4 layers in one launch (grid y = layer): the layer wavefront's biases
struct DbMulti {
  const float* dbp[4];
  float* db_ih[4];
  float* db_hh[4];
};
__global__ void persist_db_finalize_multi_kernel(const DbMulti m, int nrb, int G) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y;
  if (c >= G) return;
  const float* dbp = m.dbp[l];
  float s = 0.f;
  for (int r = 0; r < nrb; ++r) s += dbp[(long)r * G + c];
  m.db_ih[l][c] = s;
  if (m.db_hh[l]) m.db_hh[l][c] = s;
}

int sv_persist_db_finalize(const float* dbp, int nrb, int G, float* db_ih, float* db_hh, hipStream_t stream) {
  if (!dbp || !db_ih || nrb <= 0 || G <= 0) return SV_EARG;
  hipLaunchKernelGGL(persist_db_finalize_kernel, dim3((G + 255) / 256), dim3(256), 0, stream, dbp, nrb, G, db_ih, db_hh);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// ============================================================================
// host side
// ============================================================================
namespace {
constexpr int PFWD_LDS_MAIN = 2 * (BF_BM + 4 * BF_U) * (BBK + 8) * 2;
constexpr int PFWD_LDS_EPI = (BF_BM * (4 * BF_U + 4) + BF_U * (BF_BM + 1)) * 4;
constexpr int PFWD_LDS = PFWD_LDS_MAIN > PFWD_LDS_EPI ? PFWD_LDS_MAIN : PFWD_LDS_EPI;

// CU count per device, cached (device attributes do not change while the process runs)
std::atomic<int> g_cus[64];
int device_cus(int dev) {
  if (dev < 0 || dev >= 64) return 0;
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  g_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}
int current_cus() {
  int dev = 0;
  return hipGetDevice(&dev) == hipSuccess ? device_cus(dev) : 0;
}
// XCD-grouped tile order for the W-stationary kernels (persist_tile)
constexpr int kPersistXcd = 1;
#ifdef SV_FAULT_INJECTION
// test build only (libsv_ge2e_faultinj.so, `make faultinj`): sv_test_set_fault(1) (every
// persistent launch) or (2) (backward launches only) makes workgroup 0 withhold its first arrival
// and shortens the spin limit, so the launch times out deterministically and quickly.  The
// shipped library has no such state: persist_fault() is the constant 0.
std::atomic<int> g_fault{0};
int persist_fault() { return g_fault.load(std::memory_order_relaxed); }
#else
constexpr int persist_fault() { return 0; }
#endif
int fwd_fault() { return persist_fault() == 1; }
// polls before a hand-off wait gives up (each poll = one L2 round trip + s_sleep 2: ~2^21 polls
// is seconds, far beyond any legitimate wait)
unsigned persist_limit() { return persist_fault() ? (1u << 12) : (1u << 21); }
unsigned* sync_cnt(unsigned* sync, int chan) {
  return sync + SV_SYNC_CNT + (size_t)chan * SV_PCNT_ROWS * SV_PCNT_STRIDE;
}
}  // namespace

#ifdef SV_FAULT_INJECTION
extern "C" int sv_test_set_fault(int mode) {
  if (mode < 0 || mode > 2) return SV_EARG;
  g_fault.store(mode, std::memory_order_relaxed);
  return SV_OK;
}
#endif

unsigned sv_persist_limit() { return persist_limit(); }
int sv_persist_fault(int bwd) { return bwd ? persist_fault() != 0 : fwd_fault(); }

__global__ void sv_zero_counters_kernel(unsigned* cnt, int nchan, long chan_stride, int words) {
  for (int i = threadIdx.x; i < nchan * words; i += blockDim.x) cnt[(i / words) * chan_stride + i % words] = 0u;
}

int sv_zero_counters(unsigned* cnt, int nchan, long chan_stride, int words, hipStream_t stream) {
  if (!cnt || nchan <= 0 || words <= 0) return SV_EARG;
  hipLaunchKernelGGL(sv_zero_counters_kernel, dim3(1), dim3(256), 0, stream, cnt, nchan, chan_stride, words);
  return (int)hipGetLastError();
}

// head bytes up to 16-B alignment, 16-B body, tail bytes
__global__ void sv_zero_bytes_kernel(char* p, size_t head, size_t n16, size_t tail) {
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  if (i0 < head) p[i0] = 0;
  uint4* b = reinterpret_cast<uint4*>(p + head);
  for (size_t i = i0; i < n16; i += stride) b[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i0 < tail) p[head + 16 * n16 + i0] = 0;
}

int sv_zero_bytes(void* p, size_t bytes, hipStream_t stream) {
  if (!bytes) return SV_OK;
  if (!p) return SV_EARG;
  const size_t head = std::min(bytes, (size_t)((16 - ((uintptr_t)p & 15)) & 15));
  const size_t n16 = (bytes - head) / 16, tail = bytes - head - 16 * n16;
  const size_t blocks = std::max<size_t>(1, std::min<size_t>(2048, (n16 + 255) / 256));
  hipLaunchKernelGGL(sv_zero_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (char*)p, head, n16, tail);
  return (int)hipGetLastError();
}

// up to SV_ZB_MAX zeroings in one launch (blockIdx.y = buffer): the per-step state resets of the
// bf16 stack (and, for the layer wavefront, its counter channels)
struct ZeroBatch {
  char* p[SV_ZB_MAX];
  size_t head[SV_ZB_MAX], n16[SV_ZB_MAX], tail[SV_ZB_MAX];
};
__global__ void sv_zero_bytes_multi_kernel(const ZeroBatch zb) {
  const int b = blockIdx.y;
  char* p = zb.p[b];
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  if (i0 < zb.head[b]) p[i0] = 0;
  uint4* q = reinterpret_cast<uint4*>(p + zb.head[b]);
  for (size_t i = i0; i < zb.n16[b]; i += stride) q[i] = make_uint4(0u, 0u, 0u, 0u);
  if (i0 < zb.tail[b]) p[zb.head[b] + 16 * zb.n16[b] + i0] = 0;
}
int sv_zero_bytes_multi(int n, void* const* ptrs, const size_t* bytes, hipStream_t stream) {
  if (n <= 0) return SV_OK;
  if (n > SV_ZB_MAX) return SV_EARG;
  ZeroBatch zb{};
  size_t most = 0;
  for (int i = 0; i < n; ++i) {
    if (!ptrs[i] && bytes[i]) return SV_EARG;
    char* p = static_cast<char*>(ptrs[i]);
    zb.p[i] = p;
    zb.head[i] = std::min(bytes[i], (size_t)((16 - ((uintptr_t)p & 15)) & 15));
    zb.n16[i] = (bytes[i] - zb.head[i]) / 16;
    zb.tail[i] = bytes[i] - zb.head[i] - 16 * zb.n16[i];
    most = std::max(most, zb.n16[i]);
  }
  const size_t blocks = std::max<size_t>(1, std::min<size_t>(2048, (most + 255) / 256));
  hipLaunchKernelGGL(sv_zero_bytes_multi_kernel, dim3((unsigned)blocks, n), dim3(256), 0, stream, zb);
  return (int)hipGetLastError();
}

int sv_stream_cus(hipStream_t stream) {
  int dev = -1;
  if (stream && hipStreamGetDevice(stream, &dev) == hipSuccess) return device_cus(dev);
  return current_cus();
}

extern "C" size_t sv_sync_size(void) { return (size_t)SV_SYNC_WORDS * sizeof(unsigned); }

// can the persistent forward recurrence run these dims co-resident on a device of `cus` CUs?
int sv_persist_fwd_fits(int B, int H, int cus) {
  const long grid = (long)((H + BF_U - 1) / BF_U) * ((B + BF_BM - 1) / BF_BM);
  return H % 8 == 0 && (B + BF_BM - 1) / BF_BM <= SV_PCNT_ROWS && grid <= cus && (long)B * H * 2 < (1L << 31);
}
int sv_persist_bwd_fits(int B, int H, int cus) {
  return (H == 768 || H == 64 || H == 96) && sv_persist_fwd_fits(B, H, cus) && (long)B * 4 * H * 2 < (1L << 31);
}
// ... on the current device
extern "C" int sv_persist_fwd_ok(int B, int H) { return sv_persist_fwd_fits(B, H, current_cus()); }
extern "C" int sv_wave_ok(int L, int T, int B, int F, int H) {
  const int cus = current_cus();
  return sv_wave_fwd_fits(L, T, B, F, H, cus) && sv_wave_bwd_fits(L, B, H, cus);
}

namespace {
// row tile of the W-stationary kernels: 32 rows when twice the 64-row grid still fits on the
// device (B <= 320 at H = 768: c5's per-GPU batch; measured 13.4 -> 10.1 ms at the c5 rank
// shape), else 64
int persist_bm(int B, int H, int cus) {
  const long grid32 = (long)((H + BF_U - 1) / BF_U) * ((B + 31) / 32);
  return (grid32 <= cus && (B + 31) / 32 <= SV_PCNT_ROWS) ? 32 : 64;
}
}  // namespace

// the 16-row wide forward (sv_persist16_fwd_launch): H = 768, whole 16-row blocks, B > 256 (below, the
// 32 x 32 tile keeps its bit-identity with the per-step schedule), (B / 16) x (H / 64) co-resident
int pfwd16_ok(int B, int H, int cus) {
  return H == 768 && B % 16 == 0 && B > 256 && B / 16 <= SV_PCNT_ROWS && (long)(B / 16) * (H / 64) <= cus;
}

// can the persistent forward compute layer 0's input projection in-kernel (F = 40 features)?
int sv_persist_fwd_fusex_ok(int H, int F) { return H == 768 && F == 40; }

// one layer's recurrence (K2 for all t) after its K1 has filled `gates`; on `stream`.  With x_bf
// (layer 0, sv_persist_fwd_fusex_ok): no K1 -- the kernel forms x_t W_ih^T + b_ih + b_hh itself.
int pbwd3_ok(int B, int H, int cus);
int sv_persist_fwd_bf16(int T, int B, int H, const bf16_t* whh_bf, bf16_t* gates, float* c_tm, float* h_tm,
                        bf16_t* h_bf, bf16_t* hT, hipStream_t stream, unsigned* sync, int chan, const bf16_t* x_bf,
                        int F, const bf16_t* wih_bf, const float* b_ih, const float* b_hh, hipEvent_t pre,
                        hipEvent_t post, int counters_zeroed) {
  const int cus = sv_stream_cus(stream);
  if (!sv_persist_fwd_fits(B, H, cus)) return SV_ESHAPE;
  if (!sync || chan < 0 || chan >= SV_SYNC_CHANNELS) return SV_EARG;
  if (x_bf && (!wih_bf || !sv_persist_fwd_fusex_ok(H, F))) return SV_EARG;
  unsigned* cnt = sync_cnt(sync, chan);
  unsigned* status = sync;
  const int Bp = (B + 7) & ~7;
  const long ldhT = (long)(T + 1) * Bp;
  const bool wst = H == 768;  // W_hh held in registers (else the LDS-staged persistent kernel)
  // wide tile (32 rows x 64 units, sv_persist3.hip) where the wide backward runs, with or without
  // the fused layer-0 projection
  const bool wide = wst && pbwd3_ok(B, H, cus);
  // 16-row wide tile (sv_persist3.hip, with or without the fused layer-0 projection) where it keeps
  // the 32-row tile's workgroup count (B in (256, 320] at H = 768 on 256 CUs: c5's rank shape)
  const bool p16 = wst && !wide && pfwd16_ok(B, H, cus);
  const int bm = wide ? 32 : p16 ? 16 : wst ? persist_bm(B, H, cus) : BF_BM;
  const dim3 grid(wide || p16 ? H / 64 : (H + BF_U - 1) / BF_U, (B + bm - 1) / bm);
  hipError_t e = counters_zeroed ? hipSuccess : (hipError_t)sv_zero_counters(cnt, 1, 0, grid.y * SV_PCNT_STRIDE, stream);
  if (e != hipSuccess) return (int)e;
  const unsigned limit = persist_limit();
  const int fault = fwd_fault();
  constexpr int dbg = 0, pipe = 1;  // (no diagnostic skips: the kernels' dbg bits are for A/B edits); LDS-pipelined A fragments
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;  // timing probe
  if (p16) {
    const int rc = sv_persist16_fwd_launch((int)grid.y, (int)grid.x, stream, whh_bf, gates, c_tm, h_tm, h_bf, hT, ldhT,
                                           T, Bp, B, H, cnt, kPersistXcd, status, limit, fault, x_bf, F, wih_bf, b_ih,
                                           b_hh);
    if (rc) return rc;
  } else if (wide) {
    const int rc = sv_persist3_fwd_launch(dim3(grid.x * grid.y), (int)grid.x, stream, whh_bf, gates, c_tm, h_tm, h_bf,
                                          hT, ldhT, T, Bp, B, H, cnt, kPersistXcd, status, limit, fault, x_bf, F,
                                          wih_bf, b_ih, b_hh, dbg);
    if (rc) return rc;
  } else if (wst) {
    constexpr int NS = 48, LDA = NS * 16 + 8;
    const size_t lds = (size_t)bm * LDA * 2 + (size_t)bm * (4 * BF_U + 4) * 4 + (size_t)bm * (BF_U + 8) * 2 +
                       (size_t)BF_U * (bm + 8) * 2;
    const dim3 g1(grid.x * grid.y);
    const int nub = (int)grid.x, xcd = kPersistXcd;
    if (x_bf && bm == 32)
      hipLaunchKernelGGL((lstm_persist2_fwd_bf16_kernel<NS, 32, 5>), g1, dim3(256), lds, stream, whh_bf, gates, c_tm,
                         h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, pipe, x_bf, wih_bf, b_ih,
                         b_hh);
    else if (x_bf)
      hipLaunchKernelGGL((lstm_persist2_fwd_bf16_kernel<NS, 64, 5>), g1, dim3(256), lds, stream, whh_bf, gates, c_tm,
                         h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, pipe, x_bf, wih_bf, b_ih,
                         b_hh);
    else if (bm == 32)
      hipLaunchKernelGGL((lstm_persist2_fwd_bf16_kernel<NS, 32, 0>), g1, dim3(256), lds, stream, whh_bf, gates, c_tm,
                         h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, pipe, nullptr, nullptr,
                         nullptr, nullptr);
    else
      hipLaunchKernelGGL((lstm_persist2_fwd_bf16_kernel<NS, 64, 0>), g1, dim3(256), lds, stream, whh_bf, gates, c_tm,
                         h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, pipe, nullptr, nullptr,
                         nullptr, nullptr);
  } else {
    hipLaunchKernelGGL(lstm_persist_fwd_bf16_kernel<4>, grid, dim3(512), PFWD_LDS, stream, whh_bf, gates, c_tm, h_tm,
                       h_bf, hT, ldhT, T, Bp, B, H, cnt, status, limit, fault, dbg);
  }
  SV_LAUNCH_CHECK();
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  return SV_OK;
}

// ---- W-stationary persistent backward recurrence ----
namespace {
constexpr size_t pbwd_lds(int bm) {
  return (size_t)4 * bm * (BF_U + 4) * 4 + (size_t)bm * (4 * BF_U + 8) * 2 + (size_t)4 * BF_U * (bm + 8) * 2 +
         (size_t)bm * 512;  // + the LDS-DMA operand image (EWD)
}
// the backward kernels' diagnostic bits: 0 in the product library (an A/B edit sets e.g. 32 = per-phase
// cycle stamps into the caller's sync block, read by scripts/persist_ab.py, in a build with
// FLAGS=-DSV_PDBG=-1: the kernels fold the bits away otherwise)
constexpr int kPbwdDebug = 0;
template <int NS, int P>
void launch_pbwd(dim3 grid, int bm, hipStream_t s, const bf16_t* whhT, const bf16_t* acts, const float* c_tm,
                 const float* dhup, int up_full, bf16_t* dg, bf16_t* dgT, long lddgT, bf16_t* dgf, int T, int Bp, int B,
                 int H, unsigned* cnt, unsigned* sync, float* dbp) {
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(sync + SV_SYNC_STAMP);
#define SV_PBWD_LAUNCH(BMV, AG, EW)                                                                               \
  hipLaunchKernelGGL((lstm_persist2_bwd_bf16_kernel<NS, P, BMV, AG, EW>), dim3(grid.x * grid.y), dim3(256), pbwd_lds(BMV), s, \
                     whhT, acts, c_tm, dhup, up_full, dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, (int)grid.x, kPersistXcd, \
                     sync, persist_limit(), persist_fault(), kPbwdDebug, dbp, stamps)
  // weight fragments in AGPRs, step operands staged by LDS-DMA (EWD)
  if (bm == 32)
    SV_PBWD_LAUNCH(32, true, true);
  else
    SV_PBWD_LAUNCH(64, true, true);
#undef SV_PBWD_LAUNCH
}
}  // namespace

// row tile the persistent kernels use for this batch on a device of `cus` CUs (the dgf layout's
// row-block size)
// wide-tile backward (lstm_persist3_bwd_bf16_kernel): H = 768, (H / 64) x (B / 32) co-resident,
// and only where the 32-unit tile would need 64-row blocks (B > 320 on 256 CUs: c3); at smaller
// B the 32 x 32 tile's twice-as-many workgroups win (c5 rank 8.30 vs 9.48 ms, c4 rank 4.36 vs
// 5.65).
int pbwd3_ok(int B, int H, int cus) {
  const int nrb = (B + 31) / 32;
  return H == 768 && nrb <= SV_PCNT_ROWS && (long)(H / 64) * nrb <= cus && persist_bm(B, H, cus) == 64;
}
// row-block size of the backward's fragment-order hand-off (the dx GEMM's A layout)
int sv_persist_bm(int B, int H, int cus) { return pbwd3_ok(B, H, cus) ? 32 : persist_bm(B, H, cus); }

// can the persistent backward recurrence run these dims (W_hh slice in registers: H in {64, 96, 768})?
extern "C" int sv_persist_bwd_ok(int B, int H) { return sv_persist_bwd_fits(B, H, current_cus()); }

// fragment-order hand-off scratch of the persistent backward (bytes; T slots of nrb*BM x 4H
// bf16; the 64-row count bounds the 32-row one)
extern "C" size_t sv_persist_bwd_scratch(int T, int B, int H) {
  const size_t frag = (size_t)T * (size_t)((B + BF_BM - 1) / BF_BM) * BF_BM * 4 * H * sizeof(bf16_t);
  return frag + (size_t)((B + 15) / 16) * 4 * H * sizeof(float);  // + bias-gradient partials (16-row blocks)
}

// one layer's backward recurrence for all t (reverse), on `stream`: dG (bf16, row-major and
// transposed) from the activations, cell states and the upstream dh (dhup [T,B,H] if up_full,
// else [B,H] at t = T-1 only, or NULL).  dgT: [4H][T*Bp] (padding columns written as zeros).
// dgf: sv_persist_bwd_scratch(T, B, H) bytes.  Counter channel `chan` of `sync` (zeroed here unless
// counters_zeroed).
int sv_persist_bwd_bf16(int T, int B, int H, const bf16_t* whhT, const bf16_t* acts, const float* c_tm,
                        const float* dhup, int up_full, bf16_t* dg, bf16_t* dgT, bf16_t* dgf, hipStream_t stream,
                        unsigned* sync, float* db_ih, float* db_hh, hipEvent_t pre, hipEvent_t post, int chan,
                        int counters_zeroed, DbFin* defer) {
  const int cus = sv_stream_cus(stream);
  if (!sv_persist_bwd_fits(B, H, cus)) return SV_ESHAPE;
  if (!dgf || ((uintptr_t)dgf & 15) || !sync || chan < 0 || chan >= SV_SYNC_CHANNELS) return SV_EARG;
  unsigned* cnt = sync_cnt(sync, chan);
  const int Bp = (B + 7) & ~7;
  const long lddgT = (long)T * Bp;
  const bool wide = pbwd3_ok(B, H, cus);
  const int bm = wide ? 32 : persist_bm(B, H, cus);
  const dim3 grid(wide ? H / 64 : (H + BF_U - 1) / BF_U, (B + bm - 1) / bm);
  // bias-gradient partials [nrb][4H] after the fragment-order slots (db_ih NULL: not computed)
  float* dbp = db_ih ? reinterpret_cast<float*>(reinterpret_cast<char*>(dgf) +
                                                (size_t)T * ((B + BF_BM - 1) / BF_BM) * BF_BM * 4 * H * sizeof(bf16_t))
                     : nullptr;
  hipError_t e = counters_zeroed ? hipSuccess : (hipError_t)sv_zero_counters(cnt, 1, 0, grid.y * SV_PCNT_STRIDE, stream);
  if (e != hipSuccess) return (int)e;
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;  // timing probe
  // A-fragment prefetch depth 8 at H = 768 (measured: 4 / 16 no better)
  if (wide) {
    const int rc = sv_persist3_bwd_launch(dim3(grid.x * grid.y), (int)grid.x, stream, whhT, acts, c_tm, dhup, up_full,
                                          dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, kPersistXcd, sync, persist_limit(),
                                          persist_fault(), kPbwdDebug, dbp);
    if (rc) return rc;
  } else if (H == 768)
    launch_pbwd<48, 8>(grid, bm, stream, whhT, acts, c_tm, dhup, up_full, dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, sync,
                       dbp);
  else if (H == 96)
    launch_pbwd<6, 4>(grid, bm, stream, whhT, acts, c_tm, dhup, up_full, dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, sync,
                      dbp);
  else
    launch_pbwd<4, 4>(grid, bm, stream, whhT, acts, c_tm, dhup, up_full, dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, sync,
                      dbp);
  SV_LAUNCH_CHECK();
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  if (dbp && defer) {  // the caller's next launch sums the partials (dbfin_run)
    *defer = DbFin{};
    defer->dbp[0] = dbp;
    defer->db_ih[0] = db_ih;
    defer->db_hh[0] = db_hh;
    defer->n = 1;
    defer->nrb = (int)grid.y;
    defer->G = 4 * H;
  } else if (dbp) {
    hipLaunchKernelGGL(persist_db_finalize_kernel, dim3((4 * H + 255) / 256), dim3(256), 0, stream, dbp, (int)grid.y,
                       4 * H, db_ih, db_hh);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

__global__ void dbfin_kernel(const DbFin f) { dbfin_run(f, blockIdx.x); }
int sv_dbfin_launch(const DbFin& f, hipStream_t stream) {
  if (f.n <= 0) return SV_OK;
  hipLaunchKernelGGL(dbfin_kernel, dim3(dbfin_blocks(f, 256)), dim3(256), 0, stream, f);
  return (int)hipGetLastError();
}

// ---- layer-wavefront backward (lstm_wave_bwd_bf16_kernel, sv_persist3.hip) ----
// L = 3, H = 768 and all L x (H/32) x (B/32) workgroups co-resident (c4's 80 rows per rank: 216
// of 256 CUs).  SV_SCHED_PER_LAYER keeps the per-layer schedule.
int sv_wave_bwd_fits(int L, int B, int H, int cus) {
  const int nrb = (B + 31) / 32;
  return L == WB_L && H == 768 && nrb <= SV_PCNT_ROWS && (long)L * (H / 32) * nrb <= cus &&
         (long)(B + 64) * 4 * H * 2 < (1L << 31);
}
namespace {
size_t wave_frag_bytes(int T, int B, int H) {
  return ((size_t)T * ((B + 31) / 32) * 32 * 4 * H * sizeof(bf16_t) + 255) & ~size_t(255);
}
size_t wave_dbp_bytes(int B, int H) { return ((size_t)((B + 31) / 32) * 4 * H * sizeof(float) + 255) & ~size_t(255); }
}  // namespace
// per layer: the fragment-order dG hand-off ([T][nrb][4][32][H] bf16) and the bias partials
size_t sv_wave_bwd_scratch(int L, int T, int B, int H) {
  return (size_t)L * (wave_frag_bytes(T, B, H) + wave_dbp_bytes(B, H));
}
// dx[l] (l >= 1): layer l's upstream gradient for layer l-1, [T][B][H] fp32 (written whole);
// dgT[l]: [4H][T*Bp] (padding columns written as zeros); db_ih NULL: bias gradients not computed.
// Counter channels ch0 .. ch0 + L - 1 of `sync` (+ channel ch0 + L for zero_next), zeroed here unless
// counters_zeroed.
int sv_wave_bwd_bf16(int L, int T, int B, int H, const bf16_t* const* whhT, const bf16_t* const* wihT,
                     const bf16_t* const* acts, const float* const* c_tm, const float* dh_last, float* const* dx,
                     bf16_t* const* dgT, void* scratch, unsigned* sync, hipStream_t stream, float* const* db_ih,
                     float* const* db_hh, hipEvent_t pre, hipEvent_t post, long ldwih,
                     int zero_next, int ch0, int counters_zeroed, DbFin* defer) {
  if (!sv_wave_bwd_fits(L, B, H, sv_stream_cus(stream))) return SV_ESHAPE;
  if (!scratch || ((uintptr_t)scratch & 15) || !sync || !dh_last || !whhT || !wihT || !acts || !c_tm || !dx || !dgT)
    return SV_EARG;
  WaveBwdArgs a{};
  a.nub = H / 32;
  a.nrb = (B + 31) / 32;
  a.ldwih = ldwih ? ldwih : 4L * H;
  char* p = static_cast<char*>(scratch);
  for (int l = 0; l < L; ++l) {
    if (!whhT[l] || !acts[l] || !c_tm[l] || !dgT[l] || (l > 0 && (!wihT[l] || !dx[l]))) return SV_EARG;
    a.whhT[l] = whhT[l];
    a.wihT[l] = l > 0 ? wihT[l] : nullptr;
    a.acts[l] = acts[l];
    a.c[l] = c_tm[l];
    a.dx[l] = l > 0 ? dx[l] : nullptr;
    a.dgT[l] = dgT[l];
    a.dgf[l] = reinterpret_cast<bf16_t*>(p);
    p += wave_frag_bytes(T, B, H);
    a.dbp[l] = db_ih ? reinterpret_cast<float*>(p) : nullptr;
    p += wave_dbp_bytes(B, H);
    a.cnt[l] = sync_cnt(sync, ch0 + l);
  }
  if (ch0 < 0 || ch0 + L + (zero_next > 0 ? 1 : 0) > SV_SYNC_CHANNELS ||
      zero_next > SV_PCNT_ROWS * SV_PCNT_STRIDE)
    return SV_EARG;
  // zero_next > 0: channel ch0 + L's first zero_next words too (the flags of the weight-gradient
  // launch that follows, gemm_bf16_8qf_kernel), in the same launch
  if (!counters_zeroed)
    if (int rc = sv_zero_counters(a.cnt[0], zero_next > 0 ? L + 1 : L, (long)SV_PCNT_ROWS * SV_PCNT_STRIDE,
                                  std::max(a.nrb * SV_PCNT_STRIDE, zero_next), stream))
      return rc;
  a.dh_last = dh_last;
  a.status = sync;
  a.limit = persist_limit();
  a.fault = persist_fault() != 0;
  a.T = T;
  a.B = B;
  a.Bp = (B + 7) & ~7;
  a.H = H;
  a.lddgT = (long)T * a.Bp;
  hipError_t e;
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;
  const int rc = sv_wave_bwd_launch(a, stream);
  if (rc) return rc;
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  if (db_ih && defer && L <= SV_DBF_MAX) {  // the caller's next launch sums the partials (dbfin_run)
    *defer = DbFin{};
    for (int l = 0; l < L; ++l) {
      defer->dbp[l] = a.dbp[l];
      defer->db_ih[l] = db_ih[l];
      defer->db_hh[l] = db_hh ? db_hh[l] : nullptr;
    }
    defer->n = L;
    defer->nrb = a.nrb;
    defer->G = 4 * H;
  } else if (db_ih) {  // every layer's bias gradients in one launch
    DbMulti m{};
    for (int l = 0; l < L; ++l) {
      m.dbp[l] = a.dbp[l];
      m.db_ih[l] = db_ih[l];
      m.db_hh[l] = db_hh ? db_hh[l] : nullptr;
    }
    hipLaunchKernelGGL(persist_db_finalize_multi_kernel, dim3((4 * H + 255) / 256, L), dim3(256), 0, stream, m, a.nrb,
                       4 * H);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

// (status guard) loss := NaN when the sync block's status is set: a training step whose
// recurrences timed out reports a NaN loss instead of a finite wrong one
__global__ void status_poison_kernel(const unsigned* __restrict__ status, float* __restrict__ x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) x[i] = __builtin_nanf("");
}
extern "C" int sv_status_poison(const void* sync, float* x, int n, hipStream_t stream) {
  if (!sync || !x || n <= 0) return SV_EARG;
  hipLaunchKernelGGL(status_poison_kernel, dim3((n + 255) / 256), dim3(256), 0, stream,
                     reinterpret_cast<const unsigned*>(sync), x, n);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// sv_status_poison + the status word reported to the host without a copy or an event (ABI v9):
// thread 0 stores ((seq << 32) | status) into a slot of caller-owned pinned host memory mapped into
// the device's address space (system scope, release), so the host reads the outcome of step `seq`
// by comparing the slot's high word -- the device->pinned copy and the event it needed idled the
// GPU ~10 us per step
__global__ void status_report_kernel(const unsigned* __restrict__ status, float* __restrict__ x, int n,
                                     unsigned long long* slot, unsigned seq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned s = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (i < n && s) x[i] = __builtin_nanf("");
  if (i == 0)
    __hip_atomic_store(slot, ((unsigned long long)seq << 32) | s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
extern "C" int sv_status_report(const void* sync, float* x, int n, void* host_slot_dev, unsigned seq,
                                hipStream_t stream) {
  if (!sync || !host_slot_dev || n < 0 || (n > 0 && !x) || ((uintptr_t)host_slot_dev & 7)) return SV_EARG;
  hipLaunchKernelGGL(status_report_kernel, dim3(n > 0 ? (n + 255) / 256 : 1), dim3(256), 0, stream,
                     reinterpret_cast<const unsigned*>(sync), x, n,
                     reinterpret_cast<unsigned long long*>(host_slot_dev), seq);
  SV_LAUNCH_CHECK();
  return SV_OK;
}
// the device address of pinned host memory (hipHostGetDevicePointer), for sv_status_report's slot
extern "C" int sv_host_device_ptr(void* host, void** dev) {
  if (!host || !dev) return SV_EARG;
  return (int)hipHostGetDevicePointer(dev, host, 0);
}

// data-parallel status agreement: flag[0..1] := the status's forward / backward bits as floats
// (two words of the SUM-reduced gradient buffer: a sum over ranks stays nonzero iff any rank set
// the bit), then status |= the reduced bits on every rank
__global__ void status_to_flag_kernel(const unsigned* __restrict__ status, float* __restrict__ flag) {
  if (threadIdx.x == 0) {
    const unsigned s = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = (s & 1u) ? 1.f : 0.f;
    flag[1] = (s & 2u) ? 1.f : 0.f;
  }
}
__global__ void status_merge_kernel(unsigned* __restrict__ status, const float* __restrict__ flag) {
  if (threadIdx.x == 0) {
    const unsigned bits = (flag[0] != 0.f ? 1u : 0u) | (flag[1] != 0.f ? 2u : 0u);
    if (bits) __hip_atomic_fetch_or(status, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
extern "C" int sv_status_to_flag(const void* sync, float* flag, hipStream_t stream) {
  if (!sync || !flag) return SV_EARG;
  hipLaunchKernelGGL(status_to_flag_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<const unsigned*>(sync), flag);
  SV_LAUNCH_CHECK();
  return SV_OK;
}
extern "C" int sv_status_merge(void* sync, const float* flag, hipStream_t stream) {
  if (!sync || !flag) return SV_EARG;
  hipLaunchKernelGGL(status_merge_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<unsigned*>(sync), flag);
  SV_LAUNCH_CHECK();
  return SV_OK;
}
