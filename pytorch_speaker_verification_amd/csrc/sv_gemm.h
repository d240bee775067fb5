// fp32 MFMA (v_mfma_f32_32x32x2_f32, exact f32) tile machinery for gfx950.
//
// A tile of R output rows x SV_BK reduction steps is staged global -> registers ->
// LDS as [SV_BK][LD] (the output-row index contiguous), which is exactly what the
// 32x32x2 f32 MFMA operand map wants: lane l reads T[k0 + (l>>5)][r0 + (l&31)]
// (two conflict-free 32-lane ds_read_b32 groups).  Sources may be "k-contiguous"
// (element (r,k) at base[row(r)*ld + k], loaded as float4 along k and scattered as
// 4 ds_write_b32) or "r-contiguous" (element (r,k) at base[k*ld + col(r)], loaded as
// float4 along r and stored as one ds_write_b128).  Row maps let the LSTM step
// kernels gather the four gate row-blocks of W_hh into one tile.
#pragma once
#include "sv_common.h"

#define SV_BK 16

// ---------------------------------------------------------------------------
// row maps: tile-local row r -> global row (k-contig) or column (r-contig) index,
// and its validity
struct RowMapLinear {
  int base, limit;
  __device__ __forceinline__ int operator()(int r) const { return base + r; }
  __device__ __forceinline__ bool valid(int r) const { return base + r < limit; }
};
// 4 gates x U units: tile row r -> gate (r / U) * H + j0 + (r % U)   (PyTorch [i,f,g,o])
template <int U>
struct RowMapGates {
  int j0, H;
  __device__ __forceinline__ int operator()(int r) const { return (r / U) * H + j0 + (r % U); }
  __device__ __forceinline__ bool valid(int r) const { return j0 + (r % U) < H; }
};

template <bool KCONTIG, int R>
struct TileLd {
  static constexpr int value = KCONTIG ? R + 2 : R + 4;
};

// Register stage for one R x SV_BK tile, NT threads cooperating.
template <int R, int NT, bool KCONTIG>
struct TileStage {
  static constexpr int NV = (R * SV_BK / 4) / NT;  // float4 per thread
  static_assert(NV >= 1 && NV * NT * 4 == R * SV_BK, "tile/thread mismatch");
  static constexpr int LD = TileLd<KCONTIG, R>::value;
  f32x4 v[NV];

  template <class Map>
  __device__ __forceinline__ void load(const float* __restrict__ base, long ld, const Map& map, int k0, int K,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (KCONTIG) {
        const int r = q >> 2, kq = (q & 3) * 4;
        if (map.valid(r) && k0 + kq < K) x = *reinterpret_cast<const f32x4*>(base + (long)map(r) * ld + k0 + kq);
      } else {
        const int k = q / (R / 4), r4 = (q % (R / 4)) * 4;
        if (map.valid(r4) && k0 + k < K) x = *reinterpret_cast<const f32x4*>(base + (long)(k0 + k) * ld + map(r4));
      }
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(float* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      if (KCONTIG) {
        const int r = q >> 2, kq = (q & 3) * 4;
        lds[(kq + 0) * LD + r] = v[i].x;
        lds[(kq + 1) * LD + r] = v[i].y;
        lds[(kq + 2) * LD + r] = v[i].z;
        lds[(kq + 3) * LD + r] = v[i].w;
      } else {
        const int k = q / (R / 4), r4 = (q % (R / 4)) * 4;
        *reinterpret_cast<f32x4*>(lds + k * LD + r4) = v[i];
      }
    }
  }
};

// One wave's MFMA work on one staged k-tile: acc[TM][TN] 32x32 tiles at wave offsets
// (wm0, wn0) inside the LDS tiles As[SV_BK][LDA], Bs[SV_BK][LDB].
template <int TM, int TN, int LDA, int LDB>
__device__ __forceinline__ void mfma_ktile(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                           f32x16 (&acc)[TM][TN]) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < SV_BK; kk += 2) {
    float a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = As[(kk + h) * LDA + wm0 + 32 * i + r];
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = Bs[(kk + h) * LDB + wn0 + 32 * j + r];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x2(a[i], b[j], acc[i][j]);
  }
}

// Block-cooperative double-buffered main loop: NT threads stage BM x BK (A) and
// BN x BK (B) tiles; every wave computes its (TM x TN) x 32x32 sub-tile at (wm0, wn0).
// lds must hold 2 * SV_BK * (LDA + LDB) floats.
template <int BM, int BN, int NT, bool AK, bool BKC, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop(const float* __restrict__ A, long lda, const MapA& mapA,
                                              const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                              int kend, float* lds, int tid, int wm0, int wn0,
                                              f32x16 (&acc)[TM][TN]) {
  using SA = TileStage<BM, NT, AK>;
  using SB = TileStage<BN, NT, BKC>;
  constexpr int LDA = SA::LD, LDB = SB::LD;
  constexpr int BUF = SV_BK * (LDA + LDB);
  const int lane = tid & 63;
  SA sa;
  SB sb;
  const int nk = (kend - kbeg + SV_BK - 1) / SV_BK;
  if (nk <= 0) return;
  sa.load(A, lda, mapA, kbeg, kend, tid);
  sb.load(B, ldb, mapB, kbeg, kend, tid);
  sa.store(lds, tid);
  sb.store(lds + SV_BK * LDA, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* cur = lds + (kt & 1) * BUF;
    float* nxt = lds + ((kt + 1) & 1) * BUF;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, lda, mapA, kbeg + (kt + 1) * SV_BK, kend, tid);
      sb.load(B, ldb, mapB, kbeg + (kt + 1) * SV_BK, kend, tid);
    }
    mfma_ktile<TM, TN, LDA, LDB>(cur, cur + SV_BK * LDA, wm0, wn0, lane, acc);
    if (more) {
      sa.store(nxt, tid);
      sb.store(nxt + SV_BK * LDA, tid);
    }
    __syncthreads();
  }
}

template <int TM, int TN>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[TM][TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
}

// bijective XCD-aware block remap (cdna_hip_programming.md §5, T1): blocks that the
// dispatcher deals to one XCD (b % 8 equal) get a contiguous range of tile ids.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  if (q == 0) return orig;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
}

// ===========================================================================
// k-major tiles: both operands k-contiguous in HBM (element (r,k) at base[row(r)*ld + k])
// and in LDS as [R][BK+4] (16-B aligned rows; the +4-float pad makes a 16-lane group's
// ds_read_b128 of 16 distinct rows hit 16 distinct 16-B bank slots).  For the 32x32x2 f32
// MFMA, lane (r = l&31, h = l>>5) reads 4 consecutive k at 8g + 4h with one ds_read_b128
// and feeds MFMAs c = 0..3 with k_phys = 8g + 4h + c: the two lane halves together cover
// k = 8g .. 8g+7 (a fixed permutation of the reduction order, identical for A and B).
// ===========================================================================
template <int R, int NT, int BK>
struct KTileStage {
  static constexpr int LD = BK + 4;
  static constexpr int C4 = BK / 4;  // float4 per row
  static constexpr int NV = (R * C4) / NT;
  static_assert(NV >= 1 && NV * NT == R * C4, "tile/thread mismatch");
  f32x4 v[NV];

  template <class Map>
  __device__ __forceinline__ void load(const float* __restrict__ base, long ld, const Map& map, int k0, int K,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      const int r = q / C4, c = (q % C4) * 4;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (map.valid(r) && k0 + c < K) x = *reinterpret_cast<const f32x4*>(base + (long)map(r) * ld + k0 + c);
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(float* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      *reinterpret_cast<f32x4*>(lds + (q / C4) * LD + (q % C4) * 4) = v[i];
    }
  }
};

template <int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_km(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                              f32x16 (&acc)[TM][TN]) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int g = 0; g < BK / 8; ++g) {
    f32x4 a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const f32x4*>(As + (wm0 + 32 * i + r) * LD + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const f32x4*>(Bs + (wn0 + 32 * j + r) * LD + 8 * g + 4 * h);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x2(a[i][c], b[j][c], acc[i][j]);
  }
}

// lds must hold 2 * (BM + BN) * (BK + 4) floats
template <int BM, int BN, int NT, int BK, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_km(const float* __restrict__ A, long lda, const MapA& mapA,
                                                 const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                 int kend, float* lds, int tid, int wm0, int wn0,
                                                 f32x16 (&acc)[TM][TN]) {
  using SA = KTileStage<BM, NT, BK>;
  using SB = KTileStage<BN, NT, BK>;
  constexpr int LD = BK + 4;
  constexpr int BUF = (BM + BN) * LD;
  const int lane = tid & 63;
  SA sa;
  SB sb;
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  sa.load(A, lda, mapA, kbeg, kend, tid);
  sb.load(B, ldb, mapB, kbeg, kend, tid);
  sa.store(lds, tid);
  sb.store(lds + BM * LD, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    float* cur = lds + (kt & 1) * BUF;
    float* nxt = lds + ((kt + 1) & 1) * BUF;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, lda, mapA, kbeg + (kt + 1) * BK, kend, tid);
      sb.load(B, ldb, mapB, kbeg + (kt + 1) * BK, kend, tid);
    }
    mfma_ktile_km<TM, TN, BK, LD>(cur, cur + BM * LD, wm0, wn0, lane, acc);
    if (more) {
      sa.store(nxt, tid);
      sb.store(nxt + BM * LD, tid);
    }
    __syncthreads();
  }
}

// Rolling-prefetch variant of gemm_mainloop_km (software pipeline of depth D k-tiles): the
// loads of tile kt + D go into the registers tile kt has just left for LDS, so D tiles are in
// flight while one is multiplied.  For the per-step kernels, whose every launch starts from a
// cold L2 and pulls its operands from the Infinity Cache.  lds as gemm_mainloop_km.
template <int BM, int BN, int NT, int BK, int D, int TM, int TN, class MapA, class MapB, bool DIAG = false>
__device__ __forceinline__ void gemm_mainloop_km_pipe(const float* __restrict__ A, long lda, const MapA& mapA,
                                                      const float* __restrict__ B, long ldb, const MapB& mapB,
                                                      int kbeg, int kend, float* lds, int tid, int wm0, int wn0,
                                                      f32x16 (&acc)[TM][TN], int rot = 0) {
  using SA = KTileStage<BM, NT, BK>;
  using SB = KTileStage<BN, NT, BK>;
  constexpr int LD = BK + 4;
  constexpr int BUF = (BM + BN) * LD;
  const int lane = tid & 63;
  const int nk = (kend - kbeg + BK - 1) / BK;
  // k-tile visiting order rotated by `rot` (workgroups sharing an operand panel start on
  // different tiles instead of all hitting the same lines at once)
  auto kof = [&](int kt) { return kbeg + ((kt + rot) % nk) * BK; };
  SA sa[D];
  SB sb[D];
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nk) {
      sa[j].load(A, lda, mapA, kof(j), kend, tid);
      sb[j].load(B, ldb, mapB, kof(j), kend, tid);
    }
  for (int k0 = 0; k0 < nk; k0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int kt = k0 + j;
      if (kt < nk) {
        // DIAG (profiling only): every k-tile re-uses tile 0 from LDS, no further global loads
        float* buf = lds + (DIAG ? 0 : (kt & 1) * BUF);
        if (!DIAG || kt == 0) {
          sa[j].store(buf, tid);
          sb[j].store(buf + BM * LD, tid);
        }
        if (!DIAG && kt + D < nk) {
          sa[j].load(A, lda, mapA, kof(kt + D), kend, tid);
          sb[j].load(B, ldb, mapB, kof(kt + D), kend, tid);
        }
        __syncthreads();
        mfma_ktile_km<TM, TN, BK, LD>(buf, buf + BM * LD, wm0, wn0, lane, acc);
      }
    }
  }
  __syncthreads();
}

// D == 1: the plain double-buffered loop; D > 1: the rolling pipeline
template <int BM, int BN, int NT, int BK, int D, int TM, int TN, bool DIAG = false, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_km_d(const float* __restrict__ A, long lda, const MapA& mapA,
                                                   const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                   int kend, float* lds, int tid, int wm0, int wn0,
                                                   f32x16 (&acc)[TM][TN], int rot = 0) {
  if constexpr (D > 1)
    gemm_mainloop_km_pipe<BM, BN, NT, BK, D, TM, TN, MapA, MapB, DIAG>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds,
                                                                       tid, wm0, wn0, acc, rot);
  else
    gemm_mainloop_km<BM, BN, NT, BK, TM, TN>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds, tid, wm0, wn0, acc);
}
