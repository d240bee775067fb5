// 256 x 256 x 64 bf16 GEMM tile for the big NT GEMMs of the bf16 path (K1 input projection,
// dx, dW): C[M,N] fp32 = A[M,K] . B[N,K]^T (+ bias / beta, or split-K slabs).
//
// 8 waves as 2 (M) x 4 (N), each 128 x 64 of the output: 4 x 2 accumulators of
// v_mfma_f32_32x32x16_bf16, so a k-step of 16 reads 6 fragments (ds_read_b128) for 8 MFMAs
// (the 128 x 128 / 4-wave kernel reads 4 for 4).  Operands are staged global -> LDS with
// global_load_lds (16 B per lane, no VGPR round trip) into two stages of [256][64] bf16 per
// operand (128 KB, one workgroup per CU).  The LDS image is lane-linear per wave instruction,
// so the bank-conflict swizzle is applied to the per-lane global source: LDS row `row` holds
// logical 16-B slot `s` at physical slot s ^ ((row >> 1) & 7).  A 32x32x16 fragment read
// (lane -> row, one slot) then puts each ds_read_b128 lane group (MI355X_MICROARCH.md §LDS:
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) on 16 distinct 16-B bank slots: conflict-free.
// One barrier per k-tile: the next tile's DMA is issued before the current tile's MFMAs and
// retired (vmcnt(0)) before the barrier that ends them.
#pragma once
#include "sv_bf16.h"

#define G256_BM 256
#define G256_BK 64
#define G256_LDS (2 * 2 * G256_BM * G256_BK * 2)  // 2 stages x (A, B) x 256 x 64 bf16 = 128 KB

typedef __attribute__((address_space(3))) void* lds_vptr_t;
typedef __attribute__((address_space(1))) void* glb_vptr_t;

__device__ __forceinline__ int g256_phys_slot(int row, int slot) { return slot ^ ((row >> 1) & 7); }

// one operand's 256 x 64 k-tile: thread chunk q = tid + 512 i (i < 4) -> LDS byte q * 16, i.e.
// row q >> 3, physical slot q & 7, holding logical slot (q & 7) ^ ((row >> 1) & 7) of that row
struct G256Stage {
  const bf16_t* src[4];
  // rmax > 0: source rows clamped to rmax - 1 (a partial last tile: its padding rows' products
  // land only in C columns the epilogue does not store)
  __device__ __forceinline__ void init(const bf16_t* base, long ld, int row0, int k0, int tid, int rmax = 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 512 * i, row = q >> 3, ls = g256_phys_slot(row, q & 7);
      const int r = rmax > 0 ? min(row0 + row, rmax - 1) : row0 + row;
      src[i] = base + (long)r * ld + k0 + ls * 8;
    }
  }
  // DMA k-tile kt into `lds` (this operand's 32 KB of one stage); wave-uniform destination
  __device__ __forceinline__ void issue(char* lds, int kt, int wave) const {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((glb_vptr_t)(src[i] + kt * G256_BK),
                                       (lds_vptr_t)(lds + (wave * 64 + 512 * i) * 16), 16, 0, 0);
  }
};

enum { G256_STORE = 0, G256_SLAB = 1 };

// A operand in the persistent backward's fragment-order hand-off layout (sv_persist.hip, dgf):
// row m = t * bsl + b of A is (time slot t, batch row b); its 32-row group and 16-wide k-step s
// of gate g form one contiguous KB [lane][8] at slot t, block ((b / bm) * 4 + g) * (bm / 32) +
// (b / 32) % (bm / 32), k-step s.  A k-tile of 64 never crosses a gate (kg % 64 == 0), so a
// 256 x 64 A tile is 8 row groups x 4 k-steps = 32 whole KB: one per wave instruction, copied
// to LDS as is, and each lane's MFMA fragment is its own 16 B of one KB (conflict-free reads).
// second B operand of a fused pair of GEMMs sharing A (C = A . [B ; B2]^T): N-tiles at and past
// n1 read B2 (the backward's dW_hh and dW_ih of one layer: one pass over dG^T for both)
struct G256Dual {
  const bf16_t* B2;
  long ldb2;
  int n1;
  int rows2;  // rows of B2 (0: whole tiles); the rows past it read its last row (results unused)
};
struct G256AFrag {
  const bf16_t* base;  // dgf
  long fs;             // slot size (elements)
  int bsl, bm, kg;     // batch rows per slot, row-block size of the layout, gate K (= H)
  // k-tile kk (64 k) of A lies in gate g = kk / ktg at k-tile s = kk - g ktg of that gate; g is
  // (kk kdiv) >> 20 with kdiv = ceil(2^20 / ktg), exact for kk < 4096 (the host checks): a runtime
  // division per fill was ~30 instructions inside the 8-phase loop's phases (dx 17 % slower than on
  // a row-major A)
  int ktg;
  unsigned kdiv;
  long gstride;  // elements per gate of one row block's layout: (bm / 32) (kg / 16) 512
  // the row -> (slot, row block) split without division: x / d = umulhi(x, ceil(2^32 / d)),
  // exact for x d < 2^32 (the host checks T B x B < 2^32)
  unsigned bsl_div, bm_div;
  int kr, frag;  // bm / 32 row groups per row block; elements per (row group, gate): kg / 16 x 512
};
__host__ inline unsigned g256_magic(unsigned d) { return (unsigned)((((unsigned long long)1 << 32) + d - 1) / d); }
__host__ inline G256AFrag g256_afrag(const bf16_t* base, long fs, int bsl, int bm, int kg) {
  const int ktg = kg / 64;
  return G256AFrag{base, fs, bsl, bm, kg, ktg, (unsigned)(((1u << 20) + ktg - 1) / ktg),
                   (long)(bm / 32) * (kg / 16 * 512), g256_magic((unsigned)bsl), g256_magic((unsigned)bm),
                   bm / 32, kg / 16 * 512};
}
// element offset of row `row` (= t bsl + b) of the fragment-order A at gate 0, k-step 0
__device__ __forceinline__ long g256_af_rowoff(const G256AFrag& af, int row) {
  const unsigned t = __umulhi((unsigned)row, af.bsl_div), b = (unsigned)row - t * (unsigned)af.bsl;
  const unsigned rb = __umulhi(b, af.bm_div), q = (b >> 5) - rb * (unsigned)af.kr;
  return (long)t * af.fs + (long)(rb * 4u * (unsigned)af.kr + q) * af.frag;
}
// element offset of k-tile kk (64 k) of the fragment-order A, relative to a row group's gate 0
__device__ __forceinline__ long g256_af_koff(const G256AFrag& af, int kk) {
  const int g = (int)(((unsigned)kk * af.kdiv) >> 20), s = kk - g * af.ktg;
  return (long)g * af.gstride + (long)s * 2048;
}

// C tile store of a wave's 4 x 2 accumulators (bias / beta for G256_STORE, slab per k-split for
// G256_SLAB)
template <int EPI>
__device__ __forceinline__ void g256_epilogue_impl(f32x16 (&acc)[4][2], float* C, long ldc, long slab, int tm, int tn,
                                                   int wr, int wc, int lane, const float* bias0, const float* bias1,
                                                   float beta) {
  const int r = lane & 31;
  float* Cz = C + (EPI == G256_SLAB ? (long)blockIdx.y * slab : 0);
  float bsum[2];  // loaded before any store (see g8_bias)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = tn * G256_BM + wc * 64 + 32 * j + r;
    float badd = 0.f;
    if (EPI == G256_STORE) {
      if (bias0) badd += bias0[col];
      if (bias1) badd += bias1[col];
    }
    bsum[j] = badd;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = tn * G256_BM + wc * 64 + 32 * j + r;
    const float badd = bsum[j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = tm * G256_BM + wr * 128 + 32 * i + acc_row(e, lane);
        float* dst = Cz + (long)row * ldc + col;
        float v = acc[i][j][e];
        if (EPI == G256_STORE) {
          v += badd;
          if (beta != 0.f) v += beta * *dst;
        }
        *dst = v;
      }
  }
}

template <int EPI, int AF = 0>
__global__ __launch_bounds__(512, 1) void gemm_bf16_256_kernel(const bf16_t* __restrict__ A, long lda,
                                                              const bf16_t* __restrict__ B, long ldb,
                                                              float* __restrict__ C, long ldc, long slab, int M, int N,
                                                              int K, int kchunk, const float* __restrict__ bias0,
                                                              const float* __restrict__ bias1, float beta,
                                                              G256AFrag af = G256AFrag{}) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int tiles_n = N / G256_BM;
  const int nwg = tiles_n * (M / G256_BM);
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int kbeg = blockIdx.y * kchunk;
  const int nk = (min(K, kbeg + kchunk) - kbeg) / G256_BK;
  const int wr = w >> 2, wc = w & 3;  // wave's 128 x 64 output block: rows wr*128, cols wc*64
  G256Stage sa, sb;
  if constexpr (!AF) sa.init(A, lda, tm * G256_BM, kbeg, tid);
  sb.init(B, ldb, tn * G256_BM, kbeg, tid);
  constexpr int OPB = G256_BM * G256_BK * 2;  // bytes per operand per stage
  // fragment-order A (AF): wave w's instruction i copies KB c = 4 w + i = (row group c / 4,
  // k-step c % 4) of the tile
  long af_row[4];  // element offset of this lane's 16 B in row group c / 4 at gate 0, k-step 0
  if constexpr (AF) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * w + i, row = tm * G256_BM + 32 * (c >> 2);
      af_row[i] = g256_af_rowoff(af, row) + (c & 3) * 512 + lane * 8;
    }
  }
  auto issue_a = [&](char* lds, int kt) {
    if constexpr (AF) {
      const long goff = g256_af_koff(af, kbeg / G256_BK + kt);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((glb_vptr_t)(af.base + af_row[i] + goff),
                                         (lds_vptr_t)(lds + (4 * w + i) * 1024), 16, 0, 0);
    } else {
      sa.issue(lds, kt, w);
    }
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  if (nk > 0) {
    issue_a(smem, 0);
    sb.issue(smem + OPB, 0, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * 2 * OPB;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * 2 * OPB;
      issue_a(nxt, kt + 1);
      sb.issue(nxt + OPB, kt + 1, w);
    }
    const char* As = cur;
    const char* Bs = cur + OPB;
#pragma unroll
    for (int s = 0; s < G256_BK / 16; ++s) {
      bf16x8_t a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (AF) {
          a[i] = *reinterpret_cast<const bf16x8_t*>(As + ((wr * 4 + i) * 4 + s) * 1024 + lane * 16);
        } else {
          const int row = wr * 128 + 32 * i + r;
          a[i] = *reinterpret_cast<const bf16x8_t*>(As + row * 128 + g256_phys_slot(row, 2 * s + hh) * 16);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 64 + 32 * j + r;
        b[j] = *reinterpret_cast<const bf16x8_t*>(Bs + row * 128 + g256_phys_slot(row, 2 * s + hh) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(a[i], b[j], acc[i][j]);
    }
    // the next tile's DMA retired by every wave, and every wave done reading `cur`
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  g256_epilogue_impl<EPI>(acc, C, ldc, slab, tm, tn, wr, wc, lane, bias0, bias1, beta);
}
// ---- 8-phase schedule (gemm_bf16_256_kernel is kept for C rows that are not 16-B aligned) ----
// Same 256 x 256 x 64 tile, LDS images and DMA map as gemm_bf16_256_kernel, computed with
// v_mfma_f32_16x16x32_bf16 in the phase schedule of cdna_hip_programming.md §5 ("The 256² 8-phase
// template"): a k-tile is four phases, each one C quadrant (64 rows x 32 columns of the wave's
// 128 x 64) over K = 64 = 16 MFMAs, bracketed by raw s_barriers.  The two wave groups (wr = 0 / 1,
// one wave of each per SIMD) run one barrier apart, so one group's fragment reads and DMA issue
// overlap the other group's MFMAs (s_setprio 1 around the MFMA cluster).
//   phase 0: quadrant (0,0): read B nh0 (4 ds_read_b128) + A mh0 (8); issue A of k-tile kt + 1
//   phase 1: quadrant (0,1): read B nh1 (4);                          issue B of k-tile kt + 1
//   phase 2: quadrant (1,1): read A mh1 (8)
//   phase 3: quadrant (1,0): read B nh0 (4);  s_waitcnt vmcnt(0) (k-tile kt + 1 landed)
// Slot accounting (a slot = the span between two barriers; a group reads in every other slot and
// computes in the next): a stage is re-filled >= 2 slots after its last read (A: last read in
// phase 2, re-issued in the next k-tile's phase 0; B: phase 3 -> phase 1), so every read of it
// has retired (the reader's lgkmcnt(0) precedes the barrier that ends its MFMA slot); the fill
// of k-tile kt + 1 is waited for by every issuing wave before the barrier that ends its phase-3
// read slot, which both groups pass before reading kt + 1.
// The MFMA takes the B tile as its first operand, so each lane's 4 accumulator elements are 4
// consecutive C columns of one row (16-B stores): acc[mt][nt][v] = C[16 mt + fr][16 nt + 4 fq + v].
// The fragment reads are conflict-free on the swizzled image (slot ^ ((row >> 1) & 7)).
typedef float g8_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ g8_f32x4 mfma16_bf16(bf16x8_t a, bf16x8_t b, g8_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

enum { G8_STORE = 0, G8_SLAB = 1, G8_STORE_BF16 = 2 };

// 0 + bias0 + bias1 of a lane's 4 column groups (column tn 256 + wc 64 + 16 nt + 4 fq), every load
// issued before any store: a null test around each load interleaved with the stores made the
// compiler wait for each load on its own, and each such wait also for every store before it
__device__ __forceinline__ void g8_bias(const float* bias0, const float* bias1, int tn, int wc, int fq,
                                        g8_f32x4 (&bsum)[4]) {
  g8_f32x4 b0[4], b1[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) b0[nt] = b1[nt] = g8_f32x4{0.f, 0.f, 0.f, 0.f};
  const int col = tn * G256_BM + wc * 64 + 4 * fq;
  if (bias0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b0[nt] = *reinterpret_cast<const g8_f32x4*>(bias0 + col + 16 * nt);
  }
  if (bias1) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b1[nt] = *reinterpret_cast<const g8_f32x4*>(bias1 + col + 16 * nt);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    g8_f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (bias0) v += b0[nt];
    if (bias1) v += b1[nt];
    bsum[nt] = v;
  }
}

// ncol: C columns stored (the rest of a partial last tile dropped; a multiple of 4)
template <int EPI>
__device__ __forceinline__ void g8_epilogue(g8_f32x4 (&acc)[8][4], void* Cv, long ldc, long slab, int tm, int tn,
                                            int wr, int wc, int lane, const float* bias0, const float* bias1,
                                            float beta, int ncol = 1 << 30) {
  const int fr = lane & 15, fq = lane >> 4;
  g8_f32x4 bsum[4];
  if (EPI != G8_SLAB) g8_bias(bias0, bias1, tn, wc, fq, bsum);
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = tn * G256_BM + wc * 64 + 16 * nt + 4 * fq;
    if (col >= ncol) continue;
    const g8_f32x4 badd = EPI != G8_SLAB ? bsum[nt] : g8_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const long row = (long)tm * G256_BM + wr * 128 + 16 * mt + fr;
      g8_f32x4 v = acc[mt][nt];
      if constexpr (EPI == G8_STORE_BF16) {
        v += badd;
        bf16_t* dst = reinterpret_cast<bf16_t*>(Cv) + row * ldc + col;
        const unsigned lo = pack_bf2(v[0], v[1]);
        const unsigned hi = pack_bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(dst) = uint2{lo, hi};
      } else {
        float* dst = reinterpret_cast<float*>(Cv) + (EPI == G8_SLAB ? slab : 0) + row * ldc + col;  // slab: offset
        if (EPI == G8_STORE) {
          v += badd;
          if (beta != 0.f) v += beta * *reinterpret_cast<const g8_f32x4*>(dst);
        }
        *reinterpret_cast<g8_f32x4*>(dst) = v;
      }
    }
  }
}

// ---- 8-phase schedule with the fills spread two per phase ----
// Issuing a k-tile's 8 fills per wave in one or two phases measured slower: an
// LDS-DMA issue inside a phase that also reads fragments costs 100-185 cycles
// (MI355X_MICROARCH.md, "LDS-DMA piece"), so those read slots outlast the other group's 16 MFMAs.
// Here every phase issues exactly two 64-row chunks (chunk i = operand rows 64 i .. 64 i + 63;
// for A that is wave group i / 2's m-half i % 2, for B the column block of waves wc = i), and
// B nh0 stays in registers (B read in phases 0-1 only).  Per wave, in the phases of k-tile kt:
//   p0: B2(kt+1) B3(kt+1)   p1: A1(kt+1) A0(kt+2)   p2: A3(kt+1) A2(kt+2)   p3: B0(kt+2) B1(kt+2)
// Each chunk is re-filled >= 2 slots after its last read of the tile two back (A0 / A2: phase 0,
// A1 / A3: phase 2, B: phase 1).  Waits (counted, before the phase's issue): p3 vmcnt(4) -- every
// B chunk and A0 / A2 of kt+1 landed (the 4 younger ops are A1 / A0 / A3 / A2 of p1-p2); p1
// vmcnt(5) -- A1 / A3 of kt landed (younger: A2(kt+1) and the four B fills of kt+1), so the
// m-half-1 fragments read in p2 are ordered by the barrier that ends the p1 read slot.  Near the
// end of K, where fewer younger ops exist, the waits fall back to vmcnt(0).
// bf16 C through LDS: each wave's 128 x 64 tile (16 KB; the 128 KB of stages are free after the
// k-loop) is written as 8-B fragments, then stored as whole 128-B row pieces with one 16-B store
// per lane (16 store instructions per wave instead of 32 scattered 8-B ones: the store tail of a
// 256 x 256 tile is issue-bound, MI355X_MICROARCH.md "attention epilogue store tail")
__device__ __forceinline__ void g8_epilogue_bf16_lds(g8_f32x4 (&acc)[8][4], bf16_t* C, long ldc, int tm, int tn,
                                                     int wr, int wc, int w, int lane, const float* bias0,
                                                     const float* bias1, char* smem) {
  const int fr = lane & 15, fq = lane >> 4;
  char* tile = smem + w * 16384;  // [128 rows][128 B]
  g8_f32x4 bsum[4];
  g8_bias(bias0, bias1, tn, wc, fq, bsum);
  __syncthreads();                // every wave's last stage reads retired
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const g8_f32x4 v = acc[mt][nt] + bsum[nt];
      const unsigned lo = pack_bf2(v[0], v[1]);
      const unsigned hi = pack_bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(tile + (16 * mt + fr) * 128 + (16 * nt + 4 * fq) * 2) = uint2{lo, hi};
    }
  }
  // same wave reads back: LDS is ordered within a wave (the compiler waits lgkmcnt)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = 8 * i + (lane >> 3), c = lane & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + row * 128 + c * 16);
    *reinterpret_cast<uint4*>(C + ((long)tm * G256_BM + wr * 128 + row) * ldc + tn * G256_BM + wc * 64 + 8 * c) = v;
  }
}

// one 256 x 256 tile (tm, tn) of C = A . B^T (B2 past dual.n1) over the k-tiles [kbeg, kbeg + 64 nk)
// into acc: gemm_bf16_8q_kernel's prologue and 8-phase k-loop, shared by the queue-driven form.
// AUXA: cache-policy bits of the A fills (16 = sc1: A written in the same launch window by another
// kernel, read past the L1)
template <int AF, int AUXA = 0, int AUXB = 0>
__device__ __forceinline__ void g8_tile(const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B, long ldb,
                                        const G256AFrag& af, const G256Dual& dual, int tm, int tn, int kbeg, int nk,
                                        char* smem, g8_f32x4 (&acc)[8][4]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int wr = w >> 2, wc = w & 3;
  G256Stage sa, sb;
  if constexpr (!AF) sa.init(A, lda, tm * G256_BM, kbeg, tid);
  if (dual.B2 && tn * G256_BM >= dual.n1)
    sb.init(dual.B2, dual.ldb2, tn * G256_BM - dual.n1, kbeg, tid, dual.rows2);
  else
    sb.init(B, ldb, tn * G256_BM, kbeg, tid);
  constexpr int OPB = G256_BM * G256_BK * 2;
  // fragment-order A: chunk i of wave w is KB c = (2 i + w / 4) * 4 + w % 4 (row group 2 i + w / 4,
  // k-step w % 4), so a chunk is the 64 rows 64 i .. 64 i + 63 as for the row-major operand
  long af_row[4];
  if constexpr (AF) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rg = 2 * i + (w >> 2), row = tm * G256_BM + 32 * rg;
      af_row[i] = g256_af_rowoff(af, row) + (w & 3) * 512 + lane * 8;
    }
  }
  auto stage = [&](int kt) { return smem + (kt & 1) * 2 * OPB; };
  auto fill_a = [&](int kt, int i) {
    char* lds = stage(kt);
    if constexpr (AF) {
      const long goff = g256_af_koff(af, kbeg / G256_BK + kt);
      __builtin_amdgcn_global_load_lds((glb_vptr_t)(af.base + af_row[i] + goff),
                                       (lds_vptr_t)(lds + ((2 * i + (w >> 2)) * 4 + (w & 3)) * 1024), 16, 0, 0);
    } else {
      __builtin_amdgcn_global_load_lds((glb_vptr_t)(sa.src[i] + kt * G256_BK), (lds_vptr_t)(lds + (w * 64 + 512 * i) * 16),
                                       16, 0, AUXA);
    }
  };
  auto fill_b = [&](int kt, int i) {
    __builtin_amdgcn_global_load_lds((glb_vptr_t)(sb.src[i] + kt * G256_BK),
                                     (lds_vptr_t)(stage(kt) + OPB + (w * 64 + 512 * i) * 16), 16, 0, AUXB);
  };
  auto read_a = [&](const char* As, int mt, int ks) -> bf16x8_t {
    const int row = wr * 128 + 16 * mt + fr;
    if constexpr (AF) {
      return *reinterpret_cast<const bf16x8_t*>(As + ((row >> 5) * 4 + 2 * ks + (fq >> 1)) * 1024 +
                                                ((row & 31) + 32 * (fq & 1)) * 16);
    } else {
      return *reinterpret_cast<const bf16x8_t*>(As + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
    }
  };
  auto read_b = [&](const char* Bs, int nt, int ks) -> bf16x8_t {
    const int row = wc * 64 + 16 * nt + fr;
    return *reinterpret_cast<const bf16x8_t*>(Bs + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
  };
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = g8_f32x4{0.f, 0.f, 0.f, 0.f};
  // prologue: k-tile 0 whole, then k-tile 1's fills that the steady state issues in the phases of
  // k-tile -1 (A0 / A2 / B0 / B1); k-tile 0 landed
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fill_b(0, i);
#pragma unroll
    for (int i = 0; i < 4; ++i) fill_a(0, i);
  }
  if (nk > 1) {
    fill_a(1, 0);
    fill_a(1, 2);
    fill_b(1, 0);
    fill_b(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (wr == 1) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  bf16x8_t a[4][2], b0[2][2], b1[2][2];
  auto mma = [&](int mh, int nh, const bf16x8_t (&bq)[2][2]) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 * mh + i][2 * nh + j] = mfma16_bf16(bq[j][ks], a[i][ks], acc[4 * mh + i][2 * nh + j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int kt = 0; kt < nk; ++kt) {
    const char* As = stage(kt);
    const char* Bs = As + OPB;
    const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
    // phase 0: quadrant (0, 0)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b0[j][ks] = read_b(Bs, j, ks);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, i, ks);
    if (m1) {
      fill_b(kt + 1, 2);
      fill_b(kt + 1, 3);
    }
    mma(0, 0, b0);
    // phase 1: quadrant (0, 1); A1 / A3 of kt landed
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b1[j][ks] = read_b(Bs, 2 + j, ks);
    if (m1)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (m1) fill_a(kt + 1, 1);
    if (m2) fill_a(kt + 2, 0);
    mma(0, 1, b1);
    // phase 2: quadrant (1, 1)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, 4 + i, ks);
    if (m1) fill_a(kt + 1, 3);
    if (m2) fill_a(kt + 2, 2);
    mma(1, 1, b1);
    // phase 3: quadrant (1, 0); every B chunk and A0 / A2 of kt + 1 landed
    if (m2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (m1)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (m2) {
      fill_b(kt + 2, 0);
      fill_b(kt + 2, 1);
    }
    mma(1, 0, b0);
  }
  if (wr == 0) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int EPI, int AF = 0>
__global__ __launch_bounds__(512, 1) void gemm_bf16_8q_kernel(const bf16_t* __restrict__ A, long lda,
                                                             const bf16_t* __restrict__ B, long ldb, void* __restrict__ C,
                                                             long ldc, long slab, int M, int N, int K, int kchunk,
                                                             const float* __restrict__ bias0,
                                                             const float* __restrict__ bias1, float beta,
                                                             G256AFrag af = G256AFrag{}, G256Dual dual = G256Dual{},
                                                             DbFin fin = DbFin{}) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_n = N / G256_BM;
  const int nwg = tiles_n * (M / G256_BM);
  if (fin.n > 0 && (int)blockIdx.x >= nwg) {  // a deferred bias finalize (one-shot grids only)
    dbfin_run(fin, blockIdx.x - nwg);
    return;
  }
  int id = xcd_remap(blockIdx.x, nwg), sl = 0;
  if (gridDim.y > 1) splitk_tile(nwg, id, sl);
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int kbeg = sl * kchunk;
  const int nk = (min(K, kbeg + kchunk) - kbeg) / G256_BK;
  const int wr = w >> 2, wc = w & 3;
  g8_f32x4 acc[8][4];
  g8_tile<AF>(A, lda, B, ldb, af, dual, tm, tn, kbeg, nk, smem, acc);
  if constexpr (EPI == G8_STORE_BF16)
    g8_epilogue_bf16_lds(acc, reinterpret_cast<bf16_t*>(C), ldc, tm, tn, wr, wc, w, lane, bias0, bias1, smem);
  else
    g8_epilogue<EPI>(acc, C, ldc, (long)sl * slab, tm, tn, wr, wc, lane, bias0, bias1, beta);
}

// ---- persistent form of the 8-phase kernel (G8_STORE_BF16 / G8_STORE, no split-K) ----
// The K1 shape (K = 768: 12 k-tiles per 256 x 256 tile, 4800 tiles) spent ~40 % of each tile in
// its prologue (k-tile 0's fill latency) and its store tail.  Here a grid of one workgroup per CU
// walks the tiles (virtual block v = blockIdx.x + i * gridDim.x, the same xcd_remap as the
// one-shot kernel), and the next tile's k-tile 0 is filled while this tile's C is stored: its
// fills go to the stage the last k-tile did not use, and the bf16 C tile goes through the other
// stage in two 64-row halves (8 KB per wave), after which k-tile 1's first fills go there.  The
// stage of k-tile kt is (kt + base) & 1, base advancing by nk per tile.  Same MFMA order per tile
// as gemm_bf16_8q_kernel (bit-identical results).
// The bf16 C tile goes out with non-temporal stores: with plain stores the
// 128 KB per tile pushed the B panels out of the XCD's L2 (K1 at c3: 571 -> 550 us, A/B in
// profiles/r04_v6_bf16_k1_order_ab.txt; non-temporal A fills measured slower, 569 us)
__device__ __forceinline__ void g8_epilogue_bf16_half(g8_f32x4 (&acc)[8][4], int hlf, bf16_t* C, long ldc, int tm,
                                                      int tn, int wr, int wc, int lane, const float* bl, char* tile) {
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int col = tn * G256_BM + wc * 64 + 16 * nt + 4 * fq;
    const g8_f32x4 badd = bl ? *reinterpret_cast<const g8_f32x4*>(bl + col) : g8_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const g8_f32x4 v = acc[4 * hlf + m][nt] + badd;
      const unsigned lo = pack_bf2(v[0], v[1]);
      const unsigned hi = pack_bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(tile + (16 * m + fr) * 128 + (16 * nt + 4 * fq) * 2) = uint2{lo, hi};
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * i + (lane >> 3), c = lane & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + row * 128 + c * 16);
    uint4* dst = reinterpret_cast<uint4*>(C + ((long)tm * G256_BM + wr * 128 + 64 * hlf + row) * ldc + tn * G256_BM +
                                          wc * 64 + 8 * c);
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(dst));
  }
}

#define G8P_BIAS_LDS (32 * 1024)  // LDS bytes for the persistent kernel's bias sums (N <= 8192)
// Tile order: column groups of 4 tiles (grouped_tile).  K1 at c3 (12
// column tiles): groups of 4 with non-temporal C stores 540-545 us and 0.66 GB of corrected FETCH
// per launch against row-major 548-553 us / 0.89 GB (groups of 6: 538-551 us / 0.64 GB; 3: no
// faster).  Without the non-temporal stores the grouping alone gained nothing (547 -> 574 us in r03)

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_bf16_8qp_kernel(const bf16_t* __restrict__ A, long lda,
                                                              const bf16_t* __restrict__ B, long ldb, void* __restrict__ C,
                                                              long ldc, int M, int N, int K,
                                                              const float* __restrict__ bias0,
                                                              const float* __restrict__ bias1, float beta) {
  static_assert(EPI == G8_STORE_BF16 || EPI == G8_STORE, "persistent form: plain stores");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int tiles_n = N / G256_BM;
  const int nwg = tiles_n * (M / G256_BM);
  const int nk = K / G256_BK;
  const int wr = w >> 2, wc = w & 3;
  constexpr int OPB = G256_BM * G256_BK * 2;
  int v = blockIdx.x;
  if (v >= nwg) return;
  // bf16 out: 0 + bias0 + bias1 of every column staged in LDS behind the two stages (G8P_BIAS_LDS;
  // the host checks N fits), so the store tail reads it without a global load (a load there waits
  // for the next tile's fills issued before it, and for the stores)
  const float* bl = nullptr;
  if (EPI == G8_STORE_BF16 && (bias0 || bias1)) {
    float* b = reinterpret_cast<float*>(smem + 2 * 2 * G256_BM * G256_BK * 2);
    for (int c = tid; c < N; c += 512) {
      float x = 0.f;
      if (bias0) x += bias0[c];
      if (bias1) x += bias1[c];
      b[c] = x;
    }
    __syncthreads();
    bl = b;
  }
  int base = 0;
  auto tile_of = [&](int vv, int& tm_, int& tn_) {
    const int id = xcd_remap(vv, nwg);
    grouped_tile(id, M / G256_BM, tiles_n, 4, tm_, tn_);
  };
  int tm, tn;
  tile_of(v, tm, tn);
  G256Stage sa, sb;
  sa.init(A, lda, tm * G256_BM, 0, tid);
  sb.init(B, ldb, tn * G256_BM, 0, tid);
  auto stage = [&](int kt) { return smem + ((kt + base) & 1) * 2 * OPB; };
  auto fill_a = [&](int kt, int i) {
    __builtin_amdgcn_global_load_lds((glb_vptr_t)(sa.src[i] + kt * G256_BK), (lds_vptr_t)(stage(kt) + (w * 64 + 512 * i) * 16),
                                     16, 0, 0);
  };
  auto fill_b = [&](int kt, int i) {
    __builtin_amdgcn_global_load_lds((glb_vptr_t)(sb.src[i] + kt * G256_BK),
                                     (lds_vptr_t)(stage(kt) + OPB + (w * 64 + 512 * i) * 16), 16, 0, 0);
  };
  auto read_a = [&](const char* As, int mt, int ks) -> bf16x8_t {
    const int row = wr * 128 + 16 * mt + fr;
    return *reinterpret_cast<const bf16x8_t*>(As + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
  };
  auto read_b = [&](const char* Bs, int nt, int ks) -> bf16x8_t {
    const int row = wc * 64 + 16 * nt + fr;
    return *reinterpret_cast<const bf16x8_t*>(Bs + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
  };
  // first tile: k-tile 0 whole (the later tiles get it during the previous tile's store tail)
#pragma unroll
  for (int i = 0; i < 4; ++i) fill_b(0, i);
#pragma unroll
  for (int i = 0; i < 4; ++i) fill_a(0, i);
  g8_f32x4 acc[8][4];
  bf16x8_t a[4][2], b0[2][2], b1[2][2];
  auto mma = [&](int mh, int nh, const bf16x8_t (&bq)[2][2]) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 * mh + i][2 * nh + j] = mfma16_bf16(bq[j][ks], a[i][ks], acc[4 * mh + i][2 * nh + j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  while (true) {
    // prologue remainder: k-tile 1's fills that the steady state issues in the phases of k-tile -1
    if (nk > 1) {
      fill_a(1, 0);
      fill_a(1, 2);
      fill_b(1, 0);
      fill_b(1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 1) {
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = g8_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      const char* As = stage(kt);
      const char* Bs = As + OPB;
      const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) b0[j][ks] = read_b(Bs, j, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, i, ks);
      if (m1) {
        fill_b(kt + 1, 2);
        fill_b(kt + 1, 3);
      }
      mma(0, 0, b0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) b1[j][ks] = read_b(Bs, 2 + j, ks);
      if (m1)
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (m1) fill_a(kt + 1, 1);
      if (m2) fill_a(kt + 2, 0);
      mma(0, 1, b1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, 4 + i, ks);
      if (m1) fill_a(kt + 1, 3);
      if (m2) fill_a(kt + 2, 2);
      mma(1, 1, b1);
      if (m2)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (m1)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (m2) {
        fill_b(kt + 2, 0);
        fill_b(kt + 2, 1);
      }
      mma(1, 0, b0);
    }
    if (wr == 0) {
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave is past its last read of both stages.  The next tile's k-tile 0 goes to the
    // stage k-tile nk - 1 did not use, behind this tile's stores
    const int tm0 = tm, tn0 = tn;
    char* tail = stage(nk - 1);  // the C staging area (bf16 output)
    const int vn = v + gridDim.x;
    const bool more = vn < nwg;
    if (more) {
      tile_of(vn, tm, tn);
      sa.init(A, lda, tm * G256_BM, 0, tid);
      sb.init(B, ldb, tn * G256_BM, 0, tid);
      base = (base + nk) & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) fill_b(0, i);
#pragma unroll
      for (int i = 0; i < 4; ++i) fill_a(0, i);
    }
    if constexpr (EPI == G8_STORE_BF16) {
      char* wt = tail + w * 8192;  // [64 rows][128 B] per wave
      g8_epilogue_bf16_half(acc, 0, reinterpret_cast<bf16_t*>(C), ldc, tm0, tn0, wr, wc, lane, bl, wt);
      g8_epilogue_bf16_half(acc, 1, reinterpret_cast<bf16_t*>(C), ldc, tm0, tn0, wr, wc, lane, bl, wt);
      __syncthreads();  // every wave's reads of the C staging area done before k-tile 1 refills it
    } else {
      g8_epilogue<EPI>(acc, C, ldc, 0L, tm0, tn0, wr, wc, lane, bias0, bias1, beta);
    }
    if (!more) break;
    v = vn;
  }
}
