// 256 x BN x 32 exact-fp32 GEMM tile for the big NT GEMMs of the fp32 path (K1 input projection,
// dx, dW at c2): C[M,N] fp32 = A[M,K] . B[N,K]^T (+ bias0 + bias1 + beta C, or split-K slabs).
//
// Why a second fp32 kernel: the 128 x 128 register-staged kernel (gemm_km_kernel) moves every
// operand through VGPRs and ds_write, and re-reads the A panel once per column sweep (K1: 7.1 GB
// of HBM traffic per launch against 1.58 GB algorithmic).  Here:
//   * operands go global -> LDS by LDS-DMA (global_load_lds, 16 B per lane, no VGPR round trip),
//     two stages of [256][32] fp32 per operand; a row is 128 B = 8 slots of 16 B and row `row`
//     holds logical slot s at physical slot s ^ ((row >> 1) & 7) (the swizzle is applied to the
//     per-lane global source, as in sv_gemm256.h), so the MFMA fragment reads below are
//     conflict-free;
//   * 8 waves as 2 (M) x 4 (N); a 256 x 256 tile halves the operand bytes per FLOP of 128 x 128;
//   * exact fp32 products on v_mfma_f32_32x32x2_f32 (MF = 32) or v_mfma_f32_16x16x4_f32 (MF = 16),
//     B fragment as the MFMA's first operand, so each lane's accumulator holds 4 consecutive C
//     columns of one row (16-B stores).
// A k-tile is 32 k = 8192 MFMA cycles per wave: the next tile's DMA (8 instructions per wave) is
// issued before the current tile's MFMAs and waited for (vmcnt(0) + one barrier) after them.
// Reduction order: per k-tile, k-groups in order; within a group the MFMA sequence of the fp32
// k-major tiles (mfma_ktile_km / _km16 in sv_gemm.h): a fixed permutation, deterministic.
#pragma once
#include <type_traits>
#include "sv_gemm.h"

#define GF_BM 256
#define GF_BK 32

typedef __attribute__((address_space(3))) void* gf_lds_ptr_t;
typedef unsigned int gf_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void* gf_glb_ptr_t;

__device__ __forceinline__ int gf_phys_slot(int row, int slot) { return slot ^ ((row >> 1) & 7); }

// one operand's R x 32 fp32 k-tile: thread chunk q = tid + 512 i -> LDS byte q * 16 = row q >> 3,
// physical slot q & 7, holding logical slot (q & 7) ^ ((row >> 1) & 7) of that row
template <int R>
struct GfStage {
  static constexpr int NI = R * 8 / 512;
  const float* src[NI];
  __device__ __forceinline__ void init(const float* base, long ld, int row0, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = tid + 512 * i, row = q >> 3, ls = gf_phys_slot(row, q & 7);
      src[i] = base + (long)(row0 + row) * ld + k0 + ls * 4;
    }
  }
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_global_load_lds((gf_glb_ptr_t)(src[i] + kt * GF_BK),
                                       (gf_lds_ptr_t)(lds + (wave * 64 + 512 * i) * 16), 16, 0, 0);
  }
};

enum { GF_STORE = 0, GF_SLAB = 1 };

// MFMA geometry of a wave's 128 x BN/4 block
template <int BN, int MF>
struct GfGeom {
  static constexpr int WN = BN / 4;                 // wave's columns (64 or 32)
  static constexpr int TM = 128 / MF, TN = WN / MF;  // MFMA blocks per wave
  static constexpr int NR = MF == 32 ? 16 : 4;
  static constexpr int OPA = GF_BM * GF_BK * 4, OPB = BN * GF_BK * 4;  // bytes per operand per stage
  using Acc = typename std::conditional<MF == 32, f32x16, f32x4>::type;
};

// bias0 / bias1 of a lane's C columns (column of (j, q): tn BN + wc WN + MF j + c0(q)), loaded in
// one batch per pointer (zeros for a null one): a null test around each load made the compiler
// wait for every load on its own (64 serial round trips per tile, each also waiting for the stores
// issued before it).  Added as (acc + bias0) + bias1, the order of the other fp32 kernels.
template <int BN, int MF>
struct GfBias {
  using Gm = GfGeom<BN, MF>;
  f32x4 b0[Gm::TN][Gm::NR / 4], b1[Gm::TN][Gm::NR / 4];
  __device__ __forceinline__ void load(const float* bias0, const float* bias1, int tn, int wc, int fh) {
    auto col = [&](int j, int q) { return tn * BN + wc * Gm::WN + MF * j + (MF == 32 ? 8 * q + 4 * fh : 4 * fh); };
    ld(bias0, b0, col);
    ld(bias1, b1, col);
  }
  template <class F>
  __device__ __forceinline__ static void ld(const float* p, f32x4 (&d)[Gm::TN][Gm::NR / 4], F col) {
    if (p) {
#pragma unroll
      for (int j = 0; j < Gm::TN; ++j)
#pragma unroll
        for (int q = 0; q < Gm::NR / 4; ++q) d[j][q] = *reinterpret_cast<const f32x4*>(p + col(j, q));
    } else {
#pragma unroll
      for (int j = 0; j < Gm::TN; ++j)
#pragma unroll
        for (int q = 0; q < Gm::NR / 4; ++q) d[j][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ f32x4 add(f32x4 v, int j, int q) const { return v + b0[j][q] + b1[j][q]; }
};

// A operand in the fp32 persistent backward's fragment-order hand-off layout (sv_persist_f32.hip,
// dgf): row m = t * bsl + b of A is (slot t, batch row b); its 32-row group (row block b / 64, half
// (b / 32) & 1) and 8-wide k-group of gate q form one contiguous KB [64 lanes][4] -- lane r + 32 h
// holds row r at k 8 kg + 4 h .. + 3, exactly this kernel's 32x32x2 A fragment -- at slot t, block
// ((b / 64) * 4 + q) * 2 + half, k-group kg.  A 256 x 32 k-tile is 8 row groups x 4 k-groups = 32
// whole KB, copied to LDS as is (wave w: row group w); every fragment read is lane-linear.
struct GfAFrag {
  const float* base;  // dgf
  long fs;            // slot size (floats)
  int bsl, kh;        // batch rows per slot (a multiple of 32), gate width H (k per gate)
  // x / d as umulhi(x, ceil(2^32 / d)) (exact for x d < 2^32: the host checks T B x B and 4H x H):
  // a runtime division per k-tile sat in the k-loop (sv_gemm256.h's G256AFrag)
  unsigned bsl_div, kh_div;
};
__host__ inline GfAFrag gf_afrag(const float* base, long fs, int bsl, int kh) {
  auto magic = [](unsigned d) { return (unsigned)((((unsigned long long)1 << 32) + d - 1) / d); };
  return GfAFrag{base, fs, bsl, kh, magic((unsigned)bsl), magic((unsigned)kh)};
}

// the k-loop of one tile (rows tm GF_BM, columns tn BN, k-tiles [kbeg / GF_BK, + nk)) into acc
// (zeroed here); shared by the one-shot and stream-K kernels.  Ends with every wave past its last
// LDS read (the stages may be refilled).
template <int BN, int MF, int AF>
__device__ __forceinline__ void gf_mainloop(const float* __restrict__ A, long lda, const float* __restrict__ B,
                                            long ldb, int tm, int tn, int kbeg, int nk, const GfAFrag& af,
                                            char* smem,
                                            typename GfGeom<BN, MF>::Acc (&acc)[128 / MF][BN / 4 / MF]) {
  constexpr int WN = BN / 4;                 // wave's columns (64 or 32)
  constexpr int TM = 128 / MF, TN = WN / MF;  // MFMA blocks per wave
  constexpr int NR = MF == 32 ? 16 : 4;
  constexpr int OPA = GF_BM * GF_BK * 4, OPB = BN * GF_BK * 4;  // bytes per operand per stage
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  GfStage<GF_BM> sa;
  GfStage<BN> sb;
  if constexpr (!AF) sa.init(A, lda, tm * GF_BM, kbeg, tid);
  sb.init(B, ldb, tn * BN, kbeg, tid);
  auto stage = [&](int kt) { return smem + (kt & 1) * (OPA + OPB); };
  // fragment-order A: wave w copies row group w's 4 k-groups of each k-tile (KB c = 4 w + i)
  long af_row = 0;
  if constexpr (AF) {
    const int m0 = tm * GF_BM + 32 * w, t = (int)__umulhi((unsigned)m0, af.bsl_div), b = m0 - t * af.bsl;
    af_row = (long)t * af.fs + (long)((b / 64) * 8 + ((b / 32) & 1)) * (af.kh / 8 * 256) + lane * 4;
  }
  auto issue_a = [&](char* lds, int kt) {
    if constexpr (AF) {
      // the k-tile's 4 k-groups lie in one gate q (H % 32 == 0: the host checks)
      const int k0 = kbeg + kt * GF_BK, q = (int)__umulhi((unsigned)k0, af.kh_div), kg0 = (k0 - q * af.kh) / 8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_global_load_lds(
            (gf_glb_ptr_t)(af.base + af_row + (long)q * 2 * (af.kh / 8 * 256) + (kg0 + i) * 256),
            (gf_lds_ptr_t)(lds + (4 * w + i) * 1024), 16, 0, 0);
      }
    } else {
      sa.issue(lds, kt, w);
    }
  };
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < NR; ++e) acc[i][j][e] = 0.f;
  if (nk > 0) {
    issue_a(stage(0), 0);
    sb.issue(stage(0) + OPA, 0, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // fragment reads: MF = 32 -> lane (r = lane & 31, h = lane >> 5), k-group g of 8: slot 2 g + h;
  // MF = 16 -> lane (r = lane & 15, q = lane >> 4), k-group g of 16: slot 4 g + q
  constexpr int RM = MF == 32 ? 31 : 15;
  const int fr = lane & RM, fh = MF == 32 ? lane >> 5 : lane >> 4;
  constexpr int NG = MF == 32 ? GF_BK / 8 : GF_BK / 16;  // k-groups per k-tile
  auto rd = [&](const char* As, const char* Bs, int g, f32x4 (&a)[TM], f32x4 (&b)[TN]) {
    const int sl = MF == 32 ? 2 * g + fh : 4 * g + fh;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * 128 + MF * i + fr;
      if constexpr (AF)
        a[i] = *reinterpret_cast<const f32x4*>(As + ((wr * 4 + i) * 4 + g) * 1024 + lane * 16);
      else
        a[i] = *reinterpret_cast<const f32x4*>(As + row * 128 + gf_phys_slot(row, sl) * 16);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wc * WN + MF * j + fr;
      b[j] = *reinterpret_cast<const f32x4*>(Bs + row * 128 + gf_phys_slot(row, sl) * 16);
    }
  };
  auto mm = [&](const f32x4 (&a)[TM], const f32x4 (&b)[TN]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (MF == 32)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[j][c], a[i][c], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][c], a[i][c], acc[i][j], 0, 0, 0);
        }
  };
  f32x4 a0[TM], b0[TN], a1[TM], b1[TN];
  for (int kt = 0; kt < nk; ++kt) {
    const char* As = stage(kt);
    const char* Bs = As + OPA;
    if (kt + 1 < nk) {
      issue_a(stage(kt + 1), kt + 1);
      sb.issue(stage(kt + 1) + OPA, kt + 1, w);
    }
    rd(As, Bs, 0, a0, b0);
#pragma unroll
    for (int g = 0; g < NG; g += 2) {
      rd(As, Bs, g + 1, a1, b1);
      mm(a0, b0);
      if (g + 2 < NG) rd(As, Bs, g + 2, a0, b0);
      mm(a1, b1);
    }
    // the next k-tile landed (this wave's DMA) and every wave is done with this one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// C tile store of acc: acc[i][j][e] = C[row][4 consecutive cols] (+ bias0 + bias1 + beta C for
// GF_STORE; slab `sl` of the split-K workspace for GF_SLAB)
template <int BN, int MF, int EPI>
__device__ __forceinline__ void gf_store_tile(const typename GfGeom<BN, MF>::Acc (&acc)[128 / MF][BN / 4 / MF],
                                              float* __restrict__ C, long ldc, long slab, int sl, int tm, int tn,
                                              const float* __restrict__ bias0, const float* __restrict__ bias1,
                                              float beta) {
  constexpr int WN = BN / 4, TM = 128 / MF, TN = WN / MF, NR = MF == 32 ? 16 : 4;
  constexpr int RM = MF == 32 ? 31 : 15;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 2, wc = w & 3;
  const int fr = lane & RM, fh = MF == 32 ? lane >> 5 : lane >> 4;
  float* Cz = C + (EPI == GF_SLAB ? (long)sl * slab : 0);
  GfBias<BN, MF> bias;
  if (EPI == GF_STORE) bias.load(bias0, bias1, tn, wc, fh);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long row = (long)tm * GF_BM + wr * 128 + MF * i + fr;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < NR / 4; ++q) {
        // MF = 32: elements 4 q .. 4 q + 3 are columns (4 q & 3) + 8 (q) + 4 h .. + 3 of the block,
        // i.e. 8 q' + 4 h with q' = q; MF = 16: columns 4 fq .. 4 fq + 3
        const int c0 = MF == 32 ? 8 * q + 4 * fh : 4 * fh;
        const int col = tn * BN + wc * WN + MF * j + c0;
        f32x4 v = f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
        float* dst = Cz + row * ldc + col;
        if (EPI == GF_STORE) {
          v = bias.add(v, j, q);
          if (beta != 0.f) v += beta * *reinterpret_cast<const f32x4*>(dst);
        }
        *reinterpret_cast<f32x4*>(dst) = v;
      }
  }
}

template <int BN, int MF, int EPI, int AF = 0>
__global__ __launch_bounds__(512, 1) void gemm_f32_256_kernel(const float* __restrict__ A, long lda,
                                                             const float* __restrict__ B, long ldb,
                                                             float* __restrict__ C, long ldc, long slab, int M, int N,
                                                             int K, int kchunk, const float* __restrict__ bias0,
                                                             const float* __restrict__ bias1, float beta,
                                                             GfAFrag af = GfAFrag{}) {
  static_assert(!AF || MF == 32, "fragment-order A: the 32x32x2 fragment layout");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = N / BN;
  const int nwg = tiles_n * (M / GF_BM);
  int id, sl = 0, tn, tm;
  if (gridDim.y == 1) {
    // one-shot launches: column-grouped tile order (4 fp32 B panels of 256 x 768 = 3.1 MB per XCD
    // L2 at the K1 shape)
    id = xcd_remap(blockIdx.x, nwg);
    grouped_tile(id, M / GF_BM, tiles_n, 4, tm, tn);
  } else {
    splitk_tile(nwg, id, sl);
    tn = id % tiles_n;
    tm = id / tiles_n;
  }
  const int kbeg = sl * kchunk;
  const int nk = (min(K, kbeg + kchunk) - kbeg) / GF_BK;
  typename GfGeom<BN, MF>::Acc acc[128 / MF][BN / 4 / MF];
  gf_mainloop<BN, MF, AF>(A, lda, B, ldb, tm, tn, kbeg, nk, af, smem, acc);
  gf_store_tile<BN, MF, EPI>(acc, C, ldc, slab, sl, tm, tn, bias0, bias1, beta);
}

// ---- stream-K form (C = A . B^T, plain stores, no bias / beta; 32x32x2 MFMA) ----
// A one-shot launch with tiles % CUs != 0 leaves the last round partly idle: the c2 dx GEMM
// (fragment-order A) is 1200 tiles of 96 k-tiles on 256 CUs, 4.69 rounds run as 5.  Here a grid of
// G workgroups (one per CU) first runs R = tiles / G whole tiles each (data-parallel part, the
// one-shot kernel's tile order), then the remaining rem tiles' rem x nk k-tiles, cut into G equal
// contiguous ranges of L k-tiles (tile-major, k-minor).  A range's pieces of a tile are partial
// sums; each is written (sc1, drained) to the workgroup's partial slot and counted on the tile's
// arrival counter, and the workgroup that arrives last reads the others (sc1 loads) and stores the
// tile's sum -- summed in segment order (k order), so the result is deterministic.  No workgroup
// ever waits for another (no co-residency requirement).  The counters are left at zero.
struct GfSK {
  int R, rem, L;   // whole-tile rounds, stream-K tiles, k-tiles per workgroup range
  float* part;     // 2 G partial slots of 512 threads x 128 fp32 (slot 2 i: the piece opening i's range)
  unsigned* cnt;   // [rem] arrival counters, zero at the launch
};
constexpr int GF_SK_MAXSEG = 4;  // segments per stream-K tile (the host checks)

template <int BN, int AF>
__global__ __launch_bounds__(512, 1) void gemm_f32_256sk_kernel(const float* __restrict__ A, long lda,
                                                               const float* __restrict__ B, long ldb,
                                                               float* __restrict__ C, long ldc, int M, int N, int K,
                                                               GfSK sk, GfAFrag af = GfAFrag{}) {
  constexpr int MF = 32, TM = 128 / MF, TN = BN / 4 / MF, NR = 16, NV = TM * TN * NR;
  constexpr unsigned SLOT = 512u * NV * 4u;  // bytes per partial slot
  using Acc = typename GfGeom<BN, MF>::Acc;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned arrived;
  const int tid = threadIdx.x, G = gridDim.x, i = blockIdx.x;
  const int tiles_m = M / GF_BM, tiles_n = N / BN, nk = K / GF_BK;
  const long S = (long)sk.rem * nk, p1 = min(S, (long)(i + 1) * sk.L);
  long p = (long)i * sk.L;  // stream-K cursor (tile-major, k-minor)
  // partial slots: one buffer descriptor over all of them (uniform); lane offset (chunk 512 + tid) 16
  const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(sk.part, 0, 2u * G * SLOT, 0x00020000);
  Acc acc[TM][TN];
  // work items: R whole tiles (positions i + G r of [0, R G), the one-shot kernel's order), then
  // this workgroup's stream-K range -- one call site of the k-loop
  for (int r = 0;; ++r) {
    int tm, tn, ka = 0, kb = nk, j = -1;
    if (r < sk.R) {
      grouped_tile(xcd_remap(i + G * r, sk.R * G), tiles_m, tiles_n, 4, tm, tn);
    } else {
      if (p >= p1) break;
      j = (int)(p / nk);
      ka = (int)(p - (long)j * nk);
      kb = (int)min((long)nk, p1 - (long)j * nk);
      p = (long)j * nk + kb;
      grouped_tile(sk.R * G + j, tiles_m, tiles_n, 4, tm, tn);
    }
    gf_mainloop<BN, MF, AF>(A, lda, B, ldb, tm, tn, ka * GF_BK, kb - ka, af, smem, acc);
    if (ka == 0 && kb == nk) {  // a whole tile
      gf_store_tile<BN, MF, GF_STORE>(acc, C, ldc, 0L, 0, tm, tn, nullptr, nullptr, 0.f);
      continue;
    }
    // a piece of stream-K tile j: the tile's pieces are workgroups s0 .. s1's (k order)
    const int s0 = (int)(((long)j * nk) / sk.L), s1 = (int)(((long)j * nk + nk - 1) / sk.L);
    auto slot = [&](int wg) {  // slot of workgroup wg's piece of tile j: 0 if it opens wg's range
      return (unsigned)(2 * wg + ((long)wg * sk.L >= (long)j * nk ? 0 : 1)) * SLOT;
    };
    {
      const unsigned base = slot(i);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int q = 0; q < NR / 4; ++q) {
            const unsigned off = base + (unsigned)((((a * TN + b) * (NR / 4) + q) * 512 + tid) * 16);
            const f32x4 v = {acc[a][b][4 * q], acc[a][b][4 * q + 1], acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gf_u32x4, v), rpart, off, 0, 16 /* sc1 */);
          }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) arrived = __hip_atomic_fetch_add(sk.cnt + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (arrived != (unsigned)(s1 - s0)) continue;  // not the last piece to arrive
    // the last piece: the tile's pieces summed in segment order (this one from registers)
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int q = 0; q < NR / 4; ++q) {
          const unsigned off = (unsigned)((((a * TN + b) * (NR / 4) + q) * 512 + tid) * 16);
          const f32x4 own = {acc[a][b][4 * q], acc[a][b][4 * q + 1], acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]};
          f32x4 sum = own;
          for (int wg = s0; wg <= s1; ++wg) {
            const f32x4 v = wg == i ? own
                                    : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                    rpart, slot(wg) + off, 0, 16 /* sc1 */));
            sum = wg == s0 ? v : sum + v;
          }
          acc[a][b][4 * q] = sum[0];
          acc[a][b][4 * q + 1] = sum[1];
          acc[a][b][4 * q + 2] = sum[2];
          acc[a][b][4 * q + 3] = sum[3];
        }
    gf_store_tile<BN, MF, GF_STORE>(acc, C, ldc, 0L, 0, tm, tn, nullptr, nullptr, 0.f);
    if (tid == 0) __hip_atomic_store(sk.cnt + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- persistent form (plain stores, no split-K, beta = 0) ----
// At the K1 shape (4800 tiles of 24 k-tiles) the one-shot launch ran at 0.76 of the fp32 peak
// against 0.88 for the split-K dW launches of the same k-loop: its CUs finish their tiles in lock
// step, so every round starts with a cold, chip-wide k-tile-0 fill and ends in a chip-wide store
// burst (256 KB per CU).  Here one workgroup per CU walks the tiles in the one-shot order (virtual
// block v = blockIdx.x + i gridDim.x); the next tile's k-tile 0 is DMA'd during this tile's last
// k-tile (into the stage that k-tile leaves idle), so the next tile starts on landed data and its
// first k-tile runs while this tile's stores drain.  Same k-loop and summation order as
// gemm_f32_256_kernel: bit-identical results.
// (The next tile's k-tile 1 DMA'd too, before this tile's C stores, with k-tile 0's closing wait
// counting the stores, measured no faster and was deleted: DESIGN §4.)
template <int BN, int MF>
__global__ __launch_bounds__(512, 1) void gemm_f32_256p_kernel(const float* __restrict__ A, long lda,
                                                              const float* __restrict__ B, long ldb,
                                                              float* __restrict__ C, long ldc, int M, int N, int K,
                                                              const float* __restrict__ bias0,
                                                              const float* __restrict__ bias1) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Gm = GfGeom<BN, MF>;
  constexpr int TM = Gm::TM, TN = Gm::TN, WN = Gm::WN, NR = Gm::NR, OPA = Gm::OPA;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int tiles_m = M / GF_BM, tiles_n = N / BN;
  const int nwg = tiles_n * tiles_m;
  const int nk = K / GF_BK;
  constexpr int RM = MF == 32 ? 31 : 15;
  const int fr = lane & RM, fh = MF == 32 ? lane >> 5 : lane >> 4;
  int v = blockIdx.x;
  if (v >= nwg || nk <= 0) return;
  int tm, tn;
  grouped_tile(xcd_remap(v, nwg), tiles_m, tiles_n, 4, tm, tn);
  GfStage<GF_BM> sa;
  GfStage<BN> sb;
  sa.init(A, lda, tm * GF_BM, 0, tid);
  sb.init(B, ldb, tn * BN, 0, tid);
  sa.issue(smem, 0, w);
  sb.issue(smem + OPA, 0, w);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // fragment reads and MFMAs: gemm_f32_256_kernel's, verbatim (same order: bit-identical)
  constexpr int OPB = Gm::OPB;
  constexpr int NG = MF == 32 ? GF_BK / 8 : GF_BK / 16;  // k-groups per k-tile
  int base = 0;
  auto stage = [&](int kt) { return smem + ((kt + base) & 1) * (OPA + OPB); };
  typename Gm::Acc acc[TM][TN];
  auto rd = [&](const char* As, const char* Bs, int g, f32x4 (&a)[TM], f32x4 (&b)[TN]) {
    const int sl = MF == 32 ? 2 * g + fh : 4 * g + fh;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * 128 + MF * i + fr;
      a[i] = *reinterpret_cast<const f32x4*>(As + row * 128 + gf_phys_slot(row, sl) * 16);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wc * WN + MF * j + fr;
      b[j] = *reinterpret_cast<const f32x4*>(Bs + row * 128 + gf_phys_slot(row, sl) * 16);
    }
  };
  auto mm = [&](const f32x4 (&a)[TM], const f32x4 (&b)[TN]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (MF == 32)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[j][c], a[i][c], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][c], a[i][c], acc[i][j], 0, 0, 0);
        }
  };
  f32x4 a0[TM], b0[TN], a1[TM], b1[TN];
  while (true) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < NR; ++e) acc[i][j][e] = 0.f;
    const int vn = v + gridDim.x;
    const bool more = vn < nwg;
    int tmn = 0, tnn = 0;
    if (more) grouped_tile(xcd_remap(vn, nwg), tiles_m, tiles_n, 4, tmn, tnn);
    for (int kt = 0; kt < nk; ++kt) {
      const char* As = stage(kt);
      const char* Bs = As + OPA;
      if (kt + 1 < nk) {
        sa.issue(stage(kt + 1), kt + 1, w);
        sb.issue(stage(kt + 1) + OPA, kt + 1, w);
      } else if (more) {
        // the next tile's k-tile 0, into the stage this last k-tile leaves idle (stage pointers
        // formed here: held across the loop they would take registers)
        GfStage<GF_BM> na;
        GfStage<BN> nb;
        na.init(A, lda, tmn * GF_BM, 0, tid);
        nb.init(B, ldb, tnn * BN, 0, tid);
        na.issue(stage(kt + 1), 0, w);
        nb.issue(stage(kt + 1) + OPA, 0, w);
      }
      rd(As, Bs, 0, a0, b0);
#pragma unroll
      for (int g = 0; g < NG; g += 2) {
        rd(As, Bs, g + 1, a1, b1);
        mm(a0, b0);
        if (g + 2 < NG) rd(As, Bs, g + 2, a0, b0);
        mm(a1, b1);
      }
      // the next k-tile landed (this wave's DMA) and every wave is done with this one
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    GfBias<BN, MF> bias;
    bias.load(bias0, bias1, tn, wc, fh);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const long row = (long)tm * GF_BM + wr * 128 + MF * i + fr;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < NR / 4; ++q) {
          const int col = tn * BN + wc * WN + MF * j + (MF == 32 ? 8 * q + 4 * fh : 4 * fh);
          const f32x4 val =
              bias.add(f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]}, j, q);
          *reinterpret_cast<f32x4*>(C + row * ldc + col) = val;
        }
    }
    if (!more) break;
    v = vn;
    tm = tmn;
    tn = tnn;
    sa.init(A, lda, tm * GF_BM, 0, tid);
    sb.init(B, ldb, tn * BN, 0, tid);
    base = (base + nk) & 1;
  }
}
