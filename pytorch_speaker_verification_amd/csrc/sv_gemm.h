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

template <int TM, int TN, class AccT>
__device__ __forceinline__ void zero_acc(AccT (&acc)[TM][TN]) {
  constexpr int NR = sizeof(AccT) / sizeof(float);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;
}

// bijective XCD-aware block remap (cdna_hip_programming.md §5, T1): blocks that the
// dispatcher deals to one XCD (b % 8 equal) get a contiguous range of tile ids.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  if (q == 0) return orig;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
}

// Column-grouped tile order for the one-shot (no split-K) GEMM tiles: position id (after
// xcd_remap, so each XCD owns a contiguous run of positions) walks the tile grid column group by
// column group -- G column tiles (the largest divisor of tiles_n <= gmax), every row, then the next
// group.  An XCD's concurrent tiles then share G panels of B (resident in its L2 for the whole
// run) and each row panel of A is fetched once per group instead of the B panels once per few
// rows: at the K1 shape (12 column tiles) B panels were re-fetched by every XCD for every 32 tiles.
__device__ __forceinline__ void grouped_tile(int id, int tiles_m, int tiles_n, int gmax, int& tm, int& tn) {
  int G = gmax < tiles_n ? gmax : tiles_n;
  while (tiles_n % G) --G;
  const int per = tiles_m * G;
  const int cg = id / per, rem = id - cg * per;
  tm = rem / G;
  tn = cg * G + rem % G;
}

// Split-K launches (grid tiles x slabs): slab-major positions dealt to the XCDs in contiguous runs,
// so each XCD works on (mostly) one K slab and its tiles share that slab's A / B panels through its
// L2; the plain map gave every XCD pieces of every slab (dW at c2: 2.8x the algorithmic bytes).
// Every (tile, slab) computes what it did before: the results are bit-identical.
__device__ __forceinline__ void splitk_tile(int nwg, int& id, int& slab) {
  const int L = blockIdx.x + blockIdx.y * gridDim.x;
  const int pos = xcd_remap(L, gridDim.x * gridDim.y);
  slab = pos / nwg;
  id = pos - slab * nwg;
}

// XCD-aware 2-D tile map for the per-step kernels (grid nbx unit-blocks x nby row-blocks):
// the dispatcher deals linear block L to XCD L % 8; give each XCD a compact rectangle of
// (nby/2) x (nbx/4) tiles so the operand panels it reads (row-blocks of the left operand,
// unit-blocks of W) are shared through its own L2 instead of every XCD pulling every row-block
// from the Infinity Cache.  Falls back to the identity map when the grid does not split.
// Enabled by `on` (runtime switch, so one binary can A/B it).
__device__ __forceinline__ void xcd_tile_map(int on, int& bx, int& by) {
  const int nbx = gridDim.x, nby = gridDim.y;
  bx = blockIdx.x;
  by = blockIdx.y;
  if (!on || (nbx & 3) || (nby & 1)) return;
  const int L = blockIdx.x + nbx * blockIdx.y;
  const int xcd = L & 7, slot = L >> 3;
  const int ru = nbx >> 2, rr = nby >> 1;  // rectangle: rr row-blocks x ru unit-blocks
  bx = (xcd & 3) * ru + slot % ru;
  by = (xcd >> 2) * rr + slot / ru;
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

  // Buffer loads relative to the tile's first row (a uniform base, so the resource lives in
  // SGPRs): an element outside the tile (row past the map's limit, or k >= K) gets an offset
  // past num_records and reads 0 -- branch-free, unlike guarded global loads, which the
  // compiler wraps in one exec-mask branch per load.  Needs the tile's row span x ld x 4 bytes
  // below 2^31 (checked in launch_gemm_t; the step kernels' spans are a few MB).
  template <class Map>
  __device__ __forceinline__ void load(const float* __restrict__ base, long ld, const Map& map, int k0, int K,
                                       int tid) {
    const int m0 = map(0);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + (long)m0 * ld), 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      const int r = q / C4, c = (q % C4) * 4;
      const bool ok = map.valid(r) && k0 + c < K;
      const int off = ok ? (int)(((long)(map(r) - m0) * ld + k0 + c) * 4) : 0x7FFFFFF0;
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
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

// ---------------------------------------------------------------------------
// fp32 products on the bf16 MFMA pipe ("bf16x6" split): every fp32 operand x is split in
// registers into three bf16 terms x = x0 + x1 + x2 (round-to-nearest at each level, so
// |x1| <= 2^-9 |x|, |x2| <= 2^-18 |x|, residual <= 2^-27 |x|), and a*b is accumulated as
//   a1 b1 + a2 b0 + a0 b2 + a1 b0 + a0 b1 + a0 b0
// dropping a1 b2 + a2 b1 + a2 b2 (<= 2^-26 |ab|): each product is carried to ~2^-25
// relative, below fp32's own rounding (2^-24), with fp32 accumulation in the MFMA -- an fp32
// GEMM whose multiplies run on v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA rate, 6 MFMAs per
// product: 2.67x the native fp32 MFMA throughput).  Reads the same k-major fp32 LDS tiles as
// mfma_ktile_km: lane (r, h) takes k = 16 s + 8 h .. + 7 of its row (two ds_read_b128).
typedef __bf16 sv_bf16x8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void sv_split3(const f32x4 lo, const f32x4 hi, sv_bf16x8v& p0, sv_bf16x8v& p1,
                                          sv_bf16x8v& p2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = j < 4 ? lo[j] : hi[j - 4];
    const __bf16 b0 = (__bf16)x;
    const float r1 = x - (float)b0;
    const __bf16 b1 = (__bf16)r1;
    const float r2 = r1 - (float)b1;
    p0[j] = b0;
    p1[j] = b1;
    p2[j] = (__bf16)r2;
  }
}
__device__ __forceinline__ f32x16 mfma_bf16x8(sv_bf16x8v a, sv_bf16x8v b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_km_x6(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                                 f32x16 (&acc)[TM][TN]) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < BK / 16; ++s) {
    sv_bf16x8v a0[TM], a1[TM], a2[TM], b0[TN], b1[TN], b2[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* p = As + (wm0 + 32 * i + r) * LD + 16 * s + 8 * h;
      sv_split3(*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 4), a0[i], a1[i], a2[i]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* p = Bs + (wn0 + 32 * j + r) * LD + 16 * s + 8 * h;
      sv_split3(*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 4), b0[j], b1[j], b2[j]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = mfma_bf16x8(a1[i], b1[j], c);
        c = mfma_bf16x8(a2[i], b0[j], c);
        c = mfma_bf16x8(a0[i], b2[j], c);
        c = mfma_bf16x8(a1[i], b0[j], c);
        c = mfma_bf16x8(a0[i], b1[j], c);
        acc[i][j] = mfma_bf16x8(a0[i], b0[j], c);
      }
  }
}
// The same k-major tiles on v_mfma_f32_16x16x4_f32 (exact f32, 32-cycle issue; per the
// microarch guide the 16x16 shapes hold a higher clock than the 32x32 ones under sustained
// load).  Operand map: lane (r = l&15, q = l>>4) reads 4 consecutive k at 16g + 4q with one
// ds_read_b128 and feeds MFMAs c = 0..3 with k_phys = 16g + 4q + c (a fixed permutation of the
// reduction order, identical for A and B).  Here TM/TN count 16-row blocks; accumulator reg r
// of lane l holds C[row 4(l>>4) + r][col l&15].
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_km16(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                                f32x4 (&acc)[TM][TN]) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int g = 0; g < BK / 16; ++g) {
    f32x4 a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const f32x4*>(As + (wm0 + 16 * i + r) * LD + 16 * g + 4 * q);
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const f32x4*>(Bs + (wn0 + 16 * j + r) * LD + 16 * g + 4 * q);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x4(a[i][c], b[j][c], acc[i][j]);
  }
}

// dispatch between the exact fp32 MFMA k-tile and the bf16x6 one; the 16x16 accumulator type
// selects the 16x16x4 k-tile
template <bool X6, int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_f32(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                               f32x16 (&acc)[TM][TN]) {
  if constexpr (X6)
    mfma_ktile_km_x6<TM, TN, BK, LD>(As, Bs, wm0, wn0, lane, acc);
  else
    mfma_ktile_km<TM, TN, BK, LD>(As, Bs, wm0, wn0, lane, acc);
}
template <bool X6, int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_f32(const float* As, const float* Bs, int wm0, int wn0, int lane,
                                               f32x4 (&acc)[TM][TN]) {
  static_assert(!X6, "bf16x6 runs on the 32x32 tiles");
  mfma_ktile_km16<TM, TN, BK, LD>(As, Bs, wm0, wn0, lane, acc);
}

// lds must hold 2 * (BM + BN) * (BK + 4) floats
template <int BM, int BN, int NT, int BK, int TM, int TN, class MapA, class MapB, bool X6 = false, class AccT>
__device__ __forceinline__ void gemm_mainloop_km(const float* __restrict__ A, long lda, const MapA& mapA,
                                                 const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                 int kend, float* lds, int tid, int wm0, int wn0,
                                                 AccT (&acc)[TM][TN]) {
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
    mfma_ktile_f32<X6, TM, TN, BK, LD>(cur, cur + BM * LD, wm0, wn0, lane, acc);
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
template <int BM, int BN, int NT, int BK, int D, int TM, int TN, class MapA, class MapB, bool DIAG = false,
          bool X6 = false, class AccT>
__device__ __forceinline__ void gemm_mainloop_km_pipe(const float* __restrict__ A, long lda, const MapA& mapA,
                                                      const float* __restrict__ B, long ldb, const MapB& mapB,
                                                      int kbeg, int kend, float* lds, int tid, int wm0, int wn0,
                                                      AccT (&acc)[TM][TN], int rot = 0) {
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
        mfma_ktile_f32<X6, TM, TN, BK, LD>(buf, buf + BM * LD, wm0, wn0, lane, acc);
      }
    }
  }
  __syncthreads();
}

// Software-pipelined variant with one barrier per k-tile and a prefetched local read
// (32x32x2 exact fp32 only).  Tile kt+1 waits in a register stage and is written to the
// other LDS buffer during tile kt, after the first k-group's MFMAs are issued; with S stages
// its global loads were issued S tiles earlier.  The MFMA fragments of k-group g+1 are read
// while group g multiplies, and the barrier sits before the last k-group's MFMAs, which then
// cover the LDS latency of the next tile's first fragments.  Safety: the barrier in tile kt
// orders (a) every read of tile kt (issued before it, completed by the waitcnt a barrier
// implies) before the writes of tile kt+2 into the same buffer, and (b) the writes of tile
// kt+1 before its reads.  Template D = SV_PLR + S.
constexpr int SV_PLR = 100;
template <int BM, int BN, int NT, int BK, int S, int TM, int TN, class MapA, class MapB, bool NOLOAD = false>
__device__ __forceinline__ void gemm_mainloop_km_plr(const float* __restrict__ A, long lda, const MapA& mapA,
                                                     const float* __restrict__ B, long ldb, const MapB& mapB,
                                                     int kbeg, int kend, float* lds, int tid, int wm0, int wn0,
                                                     f32x16 (&acc)[TM][TN]) {
  using SA = KTileStage<BM, NT, BK>;
  using SB = KTileStage<BN, NT, BK>;
  constexpr int LD = BK + 4;
  constexpr int BUF = (BM + BN) * LD;
  constexpr int G = BK / 8;
  static_assert(G % 2 == 0 && S >= 1, "k-groups are consumed in pairs");
  const int lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  SA sa[S];
  SB sb[S];
  // tile 0 straight to LDS buffer 0; tile k >= 1 lives in stage (k - 1) % S
  sa[0].load(A, lda, mapA, kbeg, kend, tid);
  sb[0].load(B, ldb, mapB, kbeg, kend, tid);
  sa[0].store(lds, tid);
  sb[0].store(lds + BM * LD, tid);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    sa[j].load(A, lda, mapA, kbeg + (j + 1) * BK, kend, tid);
    sb[j].load(B, ldb, mapB, kbeg + (j + 1) * BK, kend, tid);
  }
  __syncthreads();
  auto rd = [&](const float* buf, int g, f32x4 (&a)[TM], f32x4 (&b)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const f32x4*>(buf + (wm0 + 32 * i + r) * LD + 8 * g + 4 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      b[j] = *reinterpret_cast<const f32x4*>(buf + BM * LD + (wn0 + 32 * j + r) * LD + 8 * g + 4 * h);
  };
  auto mm = [&](const f32x4 (&a)[TM], const f32x4 (&b)[TN]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x2(a[i][c], b[j][c], acc[i][j]);
  };
  f32x4 a0[TM], b0[TN], a1[TM], b1[TN];
  rd(lds, 0, a0, b0);
  for (int k0 = 0; k0 < nk; k0 += S) {
#pragma unroll
    for (int js = 0; js < S; ++js) {
      const int kt = k0 + js;
      if (kt < nk) {
        const float* cur = lds + (kt & 1) * BUF;
        float* nxt = lds + ((kt + 1) & 1) * BUF;
#pragma unroll
        for (int g = 0; g < G; g += 2) {
          // even group in (a0, b0), odd group in (a1, b1)
          rd(cur, g + 1, a1, b1);
          mm(a0, b0);
          if (g == 0) {
            // after the first group's MFMAs are issued, so the LDS counter the next fragment
            // reads wait on does not include these writes.  Unconditional: past the last
            // tile the stage re-stores data nobody reads and the loads are guarded off
            // (k0 >= kend).
            sa[js].store(nxt, tid);
            sb[js].store(nxt + BM * LD, tid);
            if constexpr (!NOLOAD) {  // NOLOAD (profiling only): LDS traffic without global loads
              sa[js].load(A, lda, mapA, kbeg + (kt + 1 + S) * BK, kend, tid);
              sb[js].load(B, ldb, mapB, kbeg + (kt + 1 + S) * BK, kend, tid);
            }
          }
          if (g + 2 < G) {
            rd(cur, g + 2, a0, b0);
          } else {
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            rd(nxt, 0, a0, b0);
            __builtin_amdgcn_sched_barrier(0);
          }
          mm(a1, b1);
        }
      }
    }
  }
  __syncthreads();
}

// D == 1: the plain double-buffered loop; D > 1: the rolling pipeline; D == SV_PLR + S: the
// pipelined-local-read loop above with S register stages
template <int BM, int BN, int NT, int BK, int D, int TM, int TN, bool DIAG = false, bool X6 = false, class MapA,
          class MapB, class AccT>
__device__ __forceinline__ void gemm_mainloop_km_d(const float* __restrict__ A, long lda, const MapA& mapA,
                                                   const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                   int kend, float* lds, int tid, int wm0, int wn0,
                                                   AccT (&acc)[TM][TN], int rot = 0) {
  if constexpr (D >= SV_PLR)
    gemm_mainloop_km_plr<BM, BN, NT, BK, (D > SV_PLR ? D - SV_PLR : 1), TM, TN, MapA, MapB, DIAG>(
        A, lda, mapA, B, ldb, mapB, kbeg, kend, lds, tid, wm0, wn0, acc);
  else if constexpr (D > 1)
    gemm_mainloop_km_pipe<BM, BN, NT, BK, D, TM, TN, MapA, MapB, DIAG, X6>(A, lda, mapA, B, ldb, mapB, kbeg, kend,
                                                                           lds, tid, wm0, wn0, acc, rot);
  else
    gemm_mainloop_km<BM, BN, NT, BK, TM, TN, MapA, MapB, X6>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds, tid, wm0,
                                                             wn0, acc);
}

// ---------------------------------------------------------------------------
// bf16x6 with the split done once per element, at LDS-store time ("X3" tiles): the fp32 tile
// loaded from HBM is written to LDS as three bf16 planes [3][R][BK+8] (x = x0 + x1 + x2, each
// level round-to-nearest), so each element is split by one thread instead of by every wave that
// reads it, and the MFMA k-tile reads bf16 fragments straight from the planes.  Same products,
// same accuracy as mfma_ktile_km_x6.
typedef unsigned short sv_u16;
__device__ __forceinline__ unsigned sv_pack_bf16(float lo, float hi) {
  const __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (unsigned)*reinterpret_cast<const sv_u16*>(&a) | ((unsigned)*reinterpret_cast<const sv_u16*>(&b) << 16);
}
__device__ __forceinline__ float sv_bf16_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float sv_bf16_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

template <int R, int NT, int BK>
struct KTileStageX3 {
  static constexpr int LD = BK + 8;  // bf16 elements per plane row (16-B aligned, conflict-free b128)
  static constexpr int C4 = BK / 4;
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
  // planes: [3][R][LD] bf16
  __device__ __forceinline__ void store(sv_u16* planes, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      const int off = (q / C4) * LD + (q % C4) * 4;
      unsigned p0[2], p1[2], p2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float xa = v[i][2 * h], xb = v[i][2 * h + 1];
        p0[h] = sv_pack_bf16(xa, xb);
        const float ra = xa - sv_bf16_lo(p0[h]), rb = xb - sv_bf16_hi(p0[h]);
        p1[h] = sv_pack_bf16(ra, rb);
        p2[h] = sv_pack_bf16(ra - sv_bf16_lo(p1[h]), rb - sv_bf16_hi(p1[h]));
      }
      *reinterpret_cast<uint2*>(planes + off) = uint2{p0[0], p0[1]};
      *reinterpret_cast<uint2*>(planes + R * LD + off) = uint2{p1[0], p1[1]};
      *reinterpret_cast<uint2*>(planes + 2 * R * LD + off) = uint2{p2[0], p2[1]};
    }
  }
};

template <int TM, int TN, int BK, int RA, int RB>
__device__ __forceinline__ void mfma_ktile_x3(const sv_u16* Ap, const sv_u16* Bp, int wm0, int wn0, int lane,
                                              f32x16 (&acc)[TM][TN]) {
  constexpr int LD = BK + 8;
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < BK / 16; ++s) {
    sv_bf16x8v a0[TM], a1[TM], a2[TM], b0[TN], b1[TN], b2[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int o = (wm0 + 32 * i + r) * LD + 16 * s + 8 * h;
      a0[i] = *reinterpret_cast<const sv_bf16x8v*>(Ap + o);
      a1[i] = *reinterpret_cast<const sv_bf16x8v*>(Ap + RA * LD + o);
      a2[i] = *reinterpret_cast<const sv_bf16x8v*>(Ap + 2 * RA * LD + o);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = (wn0 + 32 * j + r) * LD + 16 * s + 8 * h;
      b0[j] = *reinterpret_cast<const sv_bf16x8v*>(Bp + o);
      b1[j] = *reinterpret_cast<const sv_bf16x8v*>(Bp + RB * LD + o);
      b2[j] = *reinterpret_cast<const sv_bf16x8v*>(Bp + 2 * RB * LD + o);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = mfma_bf16x8(a1[i], b1[j], c);
        c = mfma_bf16x8(a2[i], b0[j], c);
        c = mfma_bf16x8(a0[i], b2[j], c);
        c = mfma_bf16x8(a1[i], b0[j], c);
        c = mfma_bf16x8(a0[i], b1[j], c);
        acc[i][j] = mfma_bf16x8(a0[i], b0[j], c);
      }
  }
}

// rolling-prefetch (depth D) main loop over X3 tiles.  lds (bytes): 2 stages x 3 planes x
// (BM + BN) x (BK + 8) bf16 = 12 (BM + BN)(BK + 8) bytes.
template <int BM, int BN, int NT, int BK, int D, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_x3(const float* __restrict__ A, long lda, const MapA& mapA,
                                                 const float* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                 int kend, void* lds_raw, int tid, int wm0, int wn0,
                                                 f32x16 (&acc)[TM][TN]) {
  using SA = KTileStageX3<BM, NT, BK>;
  using SB = KTileStageX3<BN, NT, BK>;
  constexpr int LD = BK + 8;
  constexpr int PA = 3 * BM * LD, STAGE = 3 * (BM + BN) * LD;
  sv_u16* lds = reinterpret_cast<sv_u16*>(lds_raw);
  const int lane = tid & 63;
  const int nk = (kend - kbeg + BK - 1) / BK;
  SA sa[D];
  SB sb[D];
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nk) {
      sa[j].load(A, lda, mapA, kbeg + j * BK, kend, tid);
      sb[j].load(B, ldb, mapB, kbeg + j * BK, kend, tid);
    }
  for (int k0 = 0; k0 < nk; k0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int kt = k0 + j;
      if (kt < nk) {
        sv_u16* buf = lds + (kt & 1) * STAGE;
        sa[j].store(buf, tid);
        sb[j].store(buf + PA, tid);
        if (kt + D < nk) {
          sa[j].load(A, lda, mapA, kbeg + (kt + D) * BK, kend, tid);
          sb[j].load(B, ldb, mapB, kbeg + (kt + D) * BK, kend, tid);
        }
        __syncthreads();
        mfma_ktile_x3<TM, TN, BK, BM, BN>(buf, buf + PA, wm0, wn0, lane, acc);
      }
    }
  }
  __syncthreads();
}
