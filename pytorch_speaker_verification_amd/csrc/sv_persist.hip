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
// Residency: the grid must be co-resident (one 512-thread workgroup per CU at most), which the
// host checks against the CU count; the spin is bounded (a timeout sets the status flag and
// the kernel drains instead of hanging), and the recurrences of different layers never run
// concurrently (the host serialises them on one stream).
#include <algorithm>
#include <stdlib.h>
#include "sv_bf16.h"
#include "../../include/sv_ge2e.h"

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define SV_PCNT_ROWS 64      // max row blocks per launch
#define SV_PCNT_STRIDE 32    // one 128-B line per counter
__device__ unsigned sv_pcnt[SV_PCNT_ROWS * SV_PCNT_STRIDE];
__device__ unsigned sv_perr;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sv_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

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

// lane 0 of the workgroup: wait until *c >= target (bounded; a timeout raises sv_perr and every
// later wait returns at once, so a broken launch drains instead of hanging the GPU)
__device__ __forceinline__ void persist_wait(unsigned* c, unsigned target) {
  unsigned spins = 0;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(&sv_perr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 21)) {
      __hip_atomic_store(&sv_perr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

// ============================================================================
// bf16 forward recurrence of one layer, all T steps.  Tile (b0, j0): 64 batch rows x 32
// units x 4 gates; 8 waves, one 32x32 accumulator each (as lstm_step_fwd_bf16_kernel).
//   gates [T,B,4H]: in = x W_ih^T + b_ih + b_hh (K1), out = activated i,f,g,o
//   c_tm [T,B,H], h_tm [T+1,B,H] (slot 0 = 0), h_bf [T+1,B,H] (slot 0 = 0, the hand-off),
//   hT [H,(T+1)Bp] or NULL.  cnt: this launch's zeroed row-block counters.
// ============================================================================
template <int D>
__global__ __launch_bounds__(512) void lstm_persist_fwd_bf16_kernel(const bf16_t* __restrict__ whh_bf,
                                                                    float* __restrict__ gates,
                                                                    float* __restrict__ c_tm,
                                                                    float* __restrict__ h_tm, bf16_t* h_bf,
                                                                    bf16_t* __restrict__ hT, long ldhT, int T,
                                                                    int Bp, int B, int H, unsigned* cnt,
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
    float* gt = gates + (long)t * B * G;
    float xg[PER][4];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 512 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      const bool ok = gb < B && gj < H;
      const float* gp = gt + (long)gb * G + gj;
#pragma unroll
      for (int q = 0; q < 4; ++q) xg[k][q] = ok ? gp[q * H] : 0.f;
    }
    f32x16 acc[1][1];
    zero_acc(acc);
    if (t > 0 && !(dbg & 2)) {
      if (tid == 0 && !(dbg & 1)) persist_wait(my_cnt, producers * (unsigned)t);
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
      const float i = sv_sigmoid(pr[0] + xg[k][0]);
      const float f = sv_sigmoid(pr[BF_U] + xg[k][1]);
      const float g = tanhf(pr[2 * BF_U] + xg[k][2]);
      const float o = sv_sigmoid(pr[3 * BF_U] + xg[k][3]);
      const float c = f * cst[k] + i * g;
      const float h = o * tanhf(c);
      cst[k] = c;
      // h_bf hand-off: lanes (u, u+1) pair up, the even lane stores both as one 4-B sc1 store
      const unsigned hbits = to_bf(h);
      const unsigned nb = __shfl_down(hbits, 1, 64);
      if (ok) {
        float* gp = gt + (long)gb * G + gj;
        gp[0] = i;
        gp[H] = f;
        gp[2 * H] = g;
        gp[3 * H] = o;
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
    if (tid == 0) __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ============================================================================
// W-stationary variant (H = 16 NS): 4 waves, wave g owns gate g of the tile's 32 units for all
// 64 rows (two 32x32 accumulators) and keeps its W_hh rows -- 32 x H bf16, the MFMA B
// fragments of every k-step -- in registers for the whole sequence.  Per step only h_{t-1}
// (64 rows x H) is staged into LDS (two halves of sc1 buffer loads); each wave reads it as A
// fragments: 1 LDS fragment per MFMA instead of 2, no W traffic at all after the prologue.
// ============================================================================
template <int NS>
__global__ __launch_bounds__(256, 1) void lstm_persist2_fwd_bf16_kernel(const bf16_t* __restrict__ whh_bf,
                                                                       float* __restrict__ gates,
                                                                       float* __restrict__ c_tm,
                                                                       float* __restrict__ h_tm, bf16_t* h_bf,
                                                                       bf16_t* __restrict__ hT, long ldhT, int T,
                                                                       int Bp, int B, int H, unsigned* cnt) {
  constexpr int K = NS * 16, LDA = K + 8, HALF = NS / 2 * 16;
  constexpr int LDP = 4 * BF_U + 4, LDH = BF_BM + 1;
  constexpr int PER = BF_BM * BF_U / 256;  // epilogue elements per thread
  static_assert(NS % 2 == 0, "two staging halves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);                          // [64][LDA]
  float* pre = reinterpret_cast<float*>(smem + BF_BM * LDA * 2);         // [64][LDP]
  float* hs = pre + BF_BM * LDP;                                         // [32][LDH]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int j0 = blockIdx.x * BF_U, b0 = blockIdx.y * BF_BM;
  const long G = 4L * H, BH = (long)B * H;
  unsigned* my_cnt = cnt + blockIdx.y * SV_PCNT_STRIDE;
  const unsigned producers = gridDim.x;
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
  }
  float cst[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) cst[k] = 0.f;
  // staging map of one half (64 rows x HALF bf16 = 64 * HALF / 8 16-B chunks over 256 threads)
  constexpr int CH = BF_BM * HALF / 8 / 256;
  // x W_ih^T + b of step t (K1 output), prefetched one step ahead: independent of the recurrence
  float xg[PER][4];
  auto load_xg = [&](int tt) {
    const float* gt = gates + (long)tt * B * G;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      const bool ok = gb < B && gj < H;
      const float* gp = gt + (long)gb * G + gj;
#pragma unroll
      for (int q = 0; q < 4; ++q) xg[k][q] = ok ? gp[q * H] : 0.f;
    }
  };
  load_xg(0);
  for (int t = 0; t < T; ++t) {
    float* gt = gates + (long)t * B * G;
    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
    if (t > 0) {
      if (tid == 0) persist_wait(my_cnt, producers * (unsigned)t);
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
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) {
        const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(As + r * LDA + 16 * s2 + 8 * hh);
        const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(As + (32 + r) * LDA + 16 * s2 + 8 * hh);
        acc0 = mfma_bf16(a0, wreg[s2], acc0);
        acc1 = mfma_bf16(a1, wreg[s2], acc1);
      }
    }
    // gate exchange: wave g's [64 rows][32 units] -> pre[row][g * 32 + unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pre[acc_row(i, lane) * LDP + g * BF_U + r] = acc0[i];
      pre[(32 + acc_row(i, lane)) * LDP + g * BF_U + r] = acc1[i];
    }
    __syncthreads();
    float* ct = c_tm + (long)t * BH;
    float* ht = h_tm + (long)(t + 1) * BH;
    bf16_t* hb = h_bf + (long)(t + 1) * BH;
    float act[PER][4], hv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      const bool ok = gb < B && gj < H;
      const float* pr = pre + b * LDP + u;
      act[k][0] = sv_sigmoid(pr[0] + xg[k][0]);
      act[k][1] = sv_sigmoid(pr[BF_U] + xg[k][1]);
      act[k][2] = tanhf(pr[2 * BF_U] + xg[k][2]);
      act[k][3] = sv_sigmoid(pr[3 * BF_U] + xg[k][3]);
      const float c = act[k][1] * cst[k] + act[k][0] * act[k][2];
      const float h = act[k][3] * tanhf(c);
      cst[k] = c;
      hv[k] = h;
      // the hand-off first: lanes (u, u+1) pair up, the even lane stores both (4-B sc1 store)
      const unsigned hbits = to_bf(h);
      const unsigned nb = __shfl_down(hbits, 1, 64);
      if (ok && !(u & 1))
        __hip_atomic_store(reinterpret_cast<unsigned*>(hb + (long)gb * H + gj), hbits | (nb << 16),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hs[u * LDH + b] = h;
    }
    __syncthreads();  // hs complete
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + 256 * k, b = e / BF_U, u = e % BF_U;
      const int gb = b0 + b, gj = j0 + u;
      if (gb < B && gj < H) {
        float* gp = gt + (long)gb * G + gj;
        gp[0] = act[k][0];
        gp[H] = act[k][1];
        gp[2 * H] = act[k][2];
        gp[3 * H] = act[k][3];
        ct[(long)gb * H + gj] = cst[k];
        ht[(long)gb * H + gj] = hv[k];
      }
    }
    if (hT) {
      for (int e = tid; e < BF_BM * BF_U; e += 256) {
        const int u = e / BF_BM, b = e % BF_BM;
        const int gb = b0 + b, gj = j0 + u;
        if (gb >= B || gj >= H) continue;
        bf16_t* row = hT + (long)gj * ldhT;
        row[(long)(t + 1) * Bp + gb] = to_bf(hs[u * LDH + b]);
        if (t == 0) row[gb] = 0;
      }
    }
    // publish h_t (every store of this step drained first), then prefetch the next x-projection
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 < T) load_xg(t + 1);
  }
}

// ============================================================================
// host side
// ============================================================================
namespace {
constexpr int PFWD_LDS_MAIN = 2 * (BF_BM + 4 * BF_U) * (BBK + 8) * 2;
constexpr int PFWD_LDS_EPI = (BF_BM * (4 * BF_U + 4) + BF_U * (BF_BM + 1)) * 4;
constexpr int PFWD_LDS = PFWD_LDS_MAIN > PFWD_LDS_EPI ? PFWD_LDS_MAIN : PFWD_LDS_EPI;

int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return n;
}
// W_hh held in registers (lstm_persist2_fwd_bf16_kernel) when H = 768; SV_PERSIST_W=0 forces the
// LDS-staged persistent kernel
int persist_wregs() {
  static int v = [] {
    const char* e = getenv("SV_PERSIST_W");
    return (e && *e == '0') ? 0 : 1;
  }();
  return v;
}
unsigned* pcnt_ptr() {
  void* p = nullptr;
  return hipGetSymbolAddress(&p, HIP_SYMBOL(sv_pcnt)) == hipSuccess ? (unsigned*)p : nullptr;
}
}  // namespace

// can the persistent forward recurrence run these dims co-resident on this device?
extern "C" int sv_persist_fwd_ok(int B, int H) {
  const long grid = (long)((H + BF_U - 1) / BF_U) * ((B + BF_BM - 1) / BF_BM);
  return H % 8 == 0 && (B + BF_BM - 1) / BF_BM <= SV_PCNT_ROWS && grid <= cu_count() && (long)B * H * 2 < (1L << 31);
}

// status of the persistent kernels since the last call (0 = ok, 1 = a hand-off wait timed out);
// synchronises the device, clears the flag
extern "C" int sv_persist_status(void) {
  unsigned v = 0, z = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(sv_perr), sizeof(v)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(sv_perr), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)v;
}

// one layer's recurrence (K2 for all t) after its K1 has filled `gates`; on `stream`
int sv_persist_fwd_bf16(int T, int B, int H, const bf16_t* whh_bf, float* gates, float* c_tm, float* h_tm,
                        bf16_t* h_bf, bf16_t* hT, hipStream_t stream) {
  if (!sv_persist_fwd_ok(B, H)) return SV_ESHAPE;
  unsigned* cnt = pcnt_ptr();
  if (!cnt) return SV_EARG;
  const int Bp = (B + 7) & ~7;
  const long ldhT = (long)(T + 1) * Bp;
  const dim3 grid((H + BF_U - 1) / BF_U, (B + BF_BM - 1) / BF_BM);
  hipError_t e = hipMemsetAsync(cnt, 0, (size_t)grid.y * SV_PCNT_STRIDE * sizeof(unsigned), stream);
  if (e != hipSuccess) return (int)e;
  // SV_PERSIST_DEBUG (profiling only, results invalid): 1 = skip the hand-off waits, 2 = skip the GEMM
  static const int dbg = [] {
    const char* v = getenv("SV_PERSIST_DEBUG");
    return v ? atoi(v) : 0;
  }();
  if (H == 768 && persist_wregs()) {
    constexpr int NS = 48, LDA = NS * 16 + 8;
    constexpr size_t lds = (size_t)BF_BM * LDA * 2 + (size_t)(BF_BM * (4 * BF_U + 4) + BF_U * (BF_BM + 1)) * 4;
    hipLaunchKernelGGL(lstm_persist2_fwd_bf16_kernel<NS>, grid, dim3(256), lds, stream, whh_bf, gates, c_tm, h_tm,
                       h_bf, hT, ldhT, T, Bp, B, H, cnt);
  } else {
    hipLaunchKernelGGL(lstm_persist_fwd_bf16_kernel<4>, grid, dim3(512), PFWD_LDS, stream, whh_bf, gates, c_tm, h_tm,
                       h_bf, hT, ldhT, T, Bp, B, H, cnt, dbg);
  }
  SV_LAUNCH_CHECK();
  return SV_OK;
}
