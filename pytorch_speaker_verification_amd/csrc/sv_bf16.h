// bf16 GEMM building blocks shared by the step kernels (sv_bf16.hip) and the persistent
// recurrences (sv_persist.hip): bf16 storage type, k-major LDS tile staging, the
// v_mfma_f32_32x32x16_bf16 k-tile, and the main loops over them.
#pragma once
#include "sv_common.h"
#include "sv_gemm.h"

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;  // storage type across the C ABI

#define BBK 64  // k-tile (bf16 elements)

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// k-major bf16 tile: element (r,k) at base[row(r)*ld + k]; LDS [R][BK+8] (144-B rows: a 16-lane
// group's ds_read_b128 of 16 distinct rows is conflict-free).  One 16-B chunk = 8 k per load.
template <int R, int NT, int BK>
struct BTileStage {
  static constexpr int LD = BK + 8;
  static constexpr int C8 = BK / 8;
  static constexpr int NV = (R * C8) / NT;
  static_assert(NV >= 1 && NV * NT == R * C8, "tile/thread mismatch");
  uint4 v[NV];
  template <class Map>
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, const Map& map, int k0, int K,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int q = tid + NT * i;
      const int r = q / C8, c = (q % C8) * 8;
      uint4 x = {0u, 0u, 0u, 0u};
      if (map.valid(r) && k0 + c < K) x = *reinterpret_cast<const uint4*>(base + (long)map(r) * ld + k0 + c);
      v[i] = x;
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

// lane (r = l&31, h = l>>5) supplies A[r][16s + 8h + j] / B[16s + 8h + j][r], j = 0..7
template <int TM, int TN, int BK, int LD>
__device__ __forceinline__ void mfma_ktile_bf(const bf16_t* As, const bf16_t* Bs, int wm0, int wn0, int lane,
                                              f32x16 (&acc)[TM][TN]) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int s = 0; s < BK / 16; ++s) {
    bf16x8_t a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const bf16x8_t*>(As + (wm0 + 32 * i + r) * LD + 16 * s + 8 * h);
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (wn0 + 32 * j + r) * LD + 16 * s + 8 * h);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma_bf16(a[i], b[j], acc[i][j]);
  }
}

// lds must hold 2 * (BM + BN) * (BK + 8) bf16
template <int BM, int BN, int NT, int BK, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_bf(const bf16_t* __restrict__ A, long lda, const MapA& mapA,
                                                 const bf16_t* __restrict__ B, long ldb, const MapB& mapB, int kbeg,
                                                 int kend, bf16_t* lds, int tid, int wm0, int wn0,
                                                 f32x16 (&acc)[TM][TN]) {
  using SA = BTileStage<BM, NT, BK>;
  using SB = BTileStage<BN, NT, BK>;
  constexpr int LD = BK + 8;
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
    bf16_t* cur = lds + (kt & 1) * BUF;
    bf16_t* nxt = lds + ((kt + 1) & 1) * BUF;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, lda, mapA, kbeg + (kt + 1) * BK, kend, tid);
      sb.load(B, ldb, mapB, kbeg + (kt + 1) * BK, kend, tid);
    }
    mfma_ktile_bf<TM, TN, BK, LD>(cur, cur + BM * LD, wm0, wn0, lane, acc);
    if (more) {
      sa.store(nxt, tid);
      sb.store(nxt + BM * LD, tid);
    }
    __syncthreads();
  }
}

// Register-prefetch main loop for the latency-bound recurrent steps: every global load of a
// super-chunk of SC k-tiles is issued up front (one HBM/L2 round trip per super-chunk instead
// of one per k-tile), then the tiles are staged through two LDS buffers, one barrier each.
template <int BM, int BN, int NT, int SC, int TM, int TN, class MapA, class MapB, bool DIAG = false>
__device__ __forceinline__ void gemm_mainloop_bf_rp(const bf16_t* __restrict__ A, long lda, const MapA& mapA,
                                                    const bf16_t* __restrict__ B, long ldb, const MapB& mapB,
                                                    int kbeg, int kend, bf16_t* lds, int tid, int wm0, int wn0,
                                                    f32x16 (&acc)[TM][TN]) {
  using SA = BTileStage<BM, NT, BBK>;
  using SB = BTileStage<BN, NT, BBK>;
  constexpr int LD = BBK + 8;
  constexpr int BUF = (BM + BN) * LD;
  const int lane = tid & 63;
  const int nk = (kend - kbeg + BBK - 1) / BBK;
  int it = 0;
  for (int c0 = 0; c0 < nk; c0 += SC) {
    SA sa[SC];
    SB sb[SC];
    // DIAG (profiling only): only the first super-chunk is fetched; later k-tiles re-use LDS
    if (!DIAG || c0 == 0) {
#pragma unroll
      for (int j = 0; j < SC; ++j) {
        if (c0 + j < nk) {
          sa[j].load(A, lda, mapA, kbeg + (c0 + j) * BBK, kend, tid);
          sb[j].load(B, ldb, mapB, kbeg + (c0 + j) * BBK, kend, tid);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < SC; ++j) {
      if (c0 + j < nk) {
        bf16_t* buf = lds + (DIAG ? 0 : (it & 1) * BUF);
        if (!DIAG || c0 == 0) {
          sa[j].store(buf, tid);
          sb[j].store(buf + BM * LD, tid);
        }
        __syncthreads();
        mfma_ktile_bf<TM, TN, BBK, LD>(buf, buf + BM * LD, wm0, wn0, lane, acc);
        ++it;
      }
    }
  }
  __syncthreads();
}

// Rolling-prefetch main loop (software pipeline of depth D k-tiles): the loads of tile
// kt + D are issued into the registers tile kt has just left for LDS, so D tiles are always in
// flight and only the first round trip is exposed (the super-chunk loop above exposes one per
// super-chunk).  One LDS double buffer, one barrier per k-tile.
template <int BM, int BN, int NT, int D, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_bf_pipe(const bf16_t* __restrict__ A, long lda, const MapA& mapA,
                                                      const bf16_t* __restrict__ B, long ldb, const MapB& mapB,
                                                      int kbeg, int kend, bf16_t* lds, int tid, int wm0, int wn0,
                                                      f32x16 (&acc)[TM][TN]) {
  using SA = BTileStage<BM, NT, BBK>;
  using SB = BTileStage<BN, NT, BBK>;
  constexpr int LD = BBK + 8;
  constexpr int BUF = (BM + BN) * LD;
  const int lane = tid & 63;
  const int nk = (kend - kbeg + BBK - 1) / BBK;
  SA sa[D];
  SB sb[D];
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nk) {
      sa[j].load(A, lda, mapA, kbeg + j * BBK, kend, tid);
      sb[j].load(B, ldb, mapB, kbeg + j * BBK, kend, tid);
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
          sa[j].load(A, lda, mapA, kbeg + (kt + D) * BBK, kend, tid);
          sb[j].load(B, ldb, mapB, kbeg + (kt + D) * BBK, kend, tid);
        }
        __syncthreads();
        mfma_ktile_bf<TM, TN, BBK, LD>(buf, buf + BM * LD, wm0, wn0, lane, acc);
      }
    }
  }
  __syncthreads();
}

// SC <= 12: super-chunk loop of SC tiles; SC = 100 + D: rolling pipeline of depth D;
// SC = 200 + x: diagnostic super-chunk loop that fetches only its first super-chunk
template <int BM, int BN, int NT, int SC, int TM, int TN, class MapA, class MapB>
__device__ __forceinline__ void gemm_mainloop_step(const bf16_t* __restrict__ A, long lda, const MapA& mapA,
                                                   const bf16_t* __restrict__ B, long ldb, const MapB& mapB,
                                                   int kbeg, int kend, bf16_t* lds, int tid, int wm0, int wn0,
                                                   f32x16 (&acc)[TM][TN]) {
  if constexpr (SC > 200)
    gemm_mainloop_bf_rp<BM, BN, NT, SC - 200, TM, TN, MapA, MapB, true>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds,
                                                                        tid, wm0, wn0, acc);
  else if constexpr (SC > 100)
    gemm_mainloop_bf_pipe<BM, BN, NT, SC - 100, TM, TN>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds, tid, wm0, wn0,
                                                        acc);
  else
    gemm_mainloop_bf_rp<BM, BN, NT, SC, TM, TN>(A, lda, mapA, B, ldb, mapB, kbeg, kend, lds, tid, wm0, wn0, acc);
}

// acc[m] += A_m . W over NS k-steps of 16, A_m = LDS rows (A0 + m * mstride; this lane's row and
// k-offset folded in), W = this wave's B fragments in registers.  The A fragments run P k-steps
// ahead of the MFMAs in a register ring: a scheduling barrier per step keeps each step's NACC
// MFMAs in front of the ds_read_b128s of step s + P, so every read is waited for P steps later
// (lgkmcnt(P-1 ...)) and the LDS latency hides behind the MFMAs instead of being paid per MFMA.
template <int NS, int NACC, int P>
__device__ __forceinline__ void mfma_lds_pipe(const bf16_t* A0, int mstride, const bf16x8_t (&W)[NS],
                                              f32x16 (&acc)[NACC]) {
  bf16x8_t f[P][NACC];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int m = 0; m < NACC; ++m) f[p][m] = *reinterpret_cast<const bf16x8_t*>(A0 + m * mstride + 16 * p);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int m = 0; m < NACC; ++m) acc[m] = mfma_bf16(f[s % P][m], W[s], acc[m]);
    if (s + P < NS) {
#pragma unroll
      for (int m = 0; m < NACC; ++m) f[s % P][m] = *reinterpret_cast<const bf16x8_t*>(A0 + m * mstride + 16 * (s + P));
    }
    // a full scheduling barrier per k-step (group barriers let the scheduler satisfy "NACC DS
    // reads here" with the reads the next MFMAs need, i.e. prefetch distance 0)
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ bf16_t to_bf(float x) {
  const __bf16 b = (__bf16)x;
  return *reinterpret_cast<const bf16_t*>(&b);
}
__device__ __forceinline__ float from_bf(bf16_t x) { return __uint_as_float((unsigned)x << 16); }
// x rounded to bf16 (nearest even) and back: the stored x-projection of the bf16 path
__device__ __forceinline__ float round_bf(float x) { return from_bf(to_bf(x)); }
// 4 consecutive bf16 <-> 4 floats (8-B loads / stores of activations and x-projections)
// a (low half) and b (high half) rounded to bf16 in one v_cvt_pk_bf16_f32 (to_bf's rounding, bit for bit)
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  typedef float fl2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector(fl2_t{a, b}, bf2_t));
}
__device__ __forceinline__ uint2 pack_bf4(float a, float b, float c, float d) {
  return uint2{pack_bf2(a, b), pack_bf2(c, d)};
}
__device__ __forceinline__ float4 unpack_bf4(uint2 p) {
  return float4{__uint_as_float(p.x << 16), __uint_as_float(p.x & 0xffff0000u), __uint_as_float(p.y << 16),
                __uint_as_float(p.y & 0xffff0000u)};
}

// Activations of the mixed-precision (bf16) path: v_exp_f32 + v_rcp_f32 forms (about 5 VALU
// instructions each instead of the accurate library tanh / division sequences, which made the
// cell update of the persistent recurrences VALU-bound: 144 -> ~40 instructions per element).
// Absolute error a few fp32 ulps of 1 (tanh near 0 included: 2 s(2x) - 1 cancels to an absolute,
// not relative, error), far below the bf16 rounding of the stored activations; the fp32 path
// keeps the accurate functions.
__device__ __forceinline__ float bf_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float bf_tanh(float x) {
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// LSTM cell forward of one element, shared by the bf16 step, wavefront and persistent kernels
// (contraction off, so every schedule rounds identically): pre-activations (recurrent part p +
// input part x) -> activated gates a[4] = i f g o, returns c_t, sets h_t
__device__ __forceinline__ float lstm_cell_fwd(const float (&p)[4], const float (&x)[4], float c_prev, float (&a)[4],
                                               float& h) {
#pragma clang fp contract(off)
  a[0] = bf_sigmoid(p[0] + x[0]);
  a[1] = bf_sigmoid(p[1] + x[1]);
  a[2] = bf_tanh(p[2] + x[2]);
  a[3] = bf_sigmoid(p[3] + x[3]);
  const float c = a[1] * c_prev + a[0] * a[2];
  h = a[3] * bf_tanh(c);
  return c;
}

// LSTM cell backward of one element, shared by the per-step and the persistent bf16 backward
// kernels so both round identically (contraction off: every product and sum rounded as written)
//   in: dh (recurrent + upstream), activated gates i f g o, c_t, c_{t-1}, dcf_in = dc_{t+1} f_{t+1}
//   out: d[4] = gate pre-activation gradients (i f g o), return dc_t f_t
__device__ __forceinline__ float lstm_cell_bwd(float dh, float i, float f, float g, float o, float c, float cp,
                                               float dcf_in, float (&d)[4]) {
#pragma clang fp contract(off)
  const float tc = bf_tanh(c);
  const float dc = dh * o * (1.f - tc * tc) + dcf_in;
  d[0] = dc * g * i * (1.f - i);
  d[1] = dc * cp * f * (1.f - f);
  d[2] = dc * i * (1.f - g * g);
  d[3] = dh * tc * o * (1.f - o);
  return dc * f;
}

// Two elements at once in packed fp32 (v_pk_mul_f32 / v_pk_add_f32: one VALU issue for both):
// the same per-element operations in the same order as lstm_cell_bwd (contraction off, the
// transcendentals per element), so results are bit-identical to it.
// the persistent bf16 kernels' diagnostic bits (dbg, profiling only, results invalid) are honoured
// only in A/B builds with -DSV_PDBG=-1; product builds fold every such branch away (the runtime
// value in per-element code cost scheduling: DESIGN §4)
#ifndef SV_PDBG
#define SV_PDBG 0
#endif
typedef float f2_t __attribute__((ext_vector_type(2)));
// a pair rounded to bf16 (nearest even) and back: one v_cvt_pk_bf16_f32 (round_bf, bit for bit)
__device__ __forceinline__ f2_t round_bf2(f2_t x) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2_t));
  return f2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// x + b for a pair, each rounded to bf16 (nearest even) and back: one v_pk_add_f32 and one
// v_cvt_pk_bf16_f32 for both (round_bf(x.x + b), round_bf(x.y + b), bit for bit)
__device__ __forceinline__ f2_t round_bf2(f2_t x, float b) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(x + b, bf2_t));
  return f2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// the cell backward's dG of 4 units x 4 gates (ddv[unit][gate]) as bf16 pairs, pr[gate][p] = units
// 2p (low half) and 2p + 1 (high half), one v_cvt_pk_bf16_f32 per pair; dbs[gate][unit] (the bias
// partials) += the rounded values, two per v_pk_add_f32 (the per-element form's sums, bit for bit)
__device__ __forceinline__ void pack_dg4(const float (&ddv)[4][4], unsigned (&pr)[4][2], float (&dbs)[4][4]) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{ddv[2 * p][q], ddv[2 * p + 1][q]}, bf2_t));
      pr[q][p] = u;
      const f2_t d = f2_t{dbs[q][2 * p], dbs[q][2 * p + 1]} + f2_t{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
      dbs[q][2 * p] = d.x;
      dbs[q][2 * p + 1] = d.y;
    }
}
// acc[i] += round_bf(x[i] + b) over 16 accumulator elements, in pairs
template <typename V>
__device__ __forceinline__ void add_round_bf16x(V& acc, const V& x, float b) {
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const f2_t s = f2_t{acc[i], acc[i + 1]} + round_bf2(f2_t{x[i], x[i + 1]}, b);
    acc[i] = s.x;
    acc[i + 1] = s.y;
  }
}
__device__ __forceinline__ f2_t bf_tanh2(f2_t x) {
#pragma clang fp contract(off)
  const f2_t y = -2.0f * x;
  const f2_t e = f2_t{__expf(y.x), __expf(y.y)};
  const f2_t d = 1.0f + e;
  const f2_t r = f2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return 2.0f * r - 1.0f;
}
__device__ __forceinline__ f2_t bf_sigmoid2(f2_t x) {
#pragma clang fp contract(off)
  const f2_t y = -x;
  const f2_t d = 1.0f + f2_t{__expf(y.x), __expf(y.y)};
  return f2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
// lstm_cell_fwd on two elements (same operations, same order: bit-identical)
__device__ __forceinline__ f2_t lstm_cell_fwd2(const f2_t (&p)[4], const f2_t (&x)[4], f2_t c_prev, f2_t (&a)[4],
                                               f2_t& h) {
#pragma clang fp contract(off)
  a[0] = bf_sigmoid2(p[0] + x[0]);
  a[1] = bf_sigmoid2(p[1] + x[1]);
  a[2] = bf_tanh2(p[2] + x[2]);
  a[3] = bf_sigmoid2(p[3] + x[3]);
  const f2_t c = a[1] * c_prev + a[0] * a[2];
  h = a[3] * bf_tanh2(c);
  return c;
}
__device__ __forceinline__ f2_t lstm_cell_bwd2(f2_t dh, f2_t i, f2_t f, f2_t g, f2_t o, f2_t c, f2_t cp, f2_t dcf_in,
                                               f2_t (&d)[4]) {
#pragma clang fp contract(off)
  const f2_t tc = bf_tanh2(c);
  const f2_t dc = dh * o * (1.f - tc * tc) + dcf_in;
  d[0] = dc * g * i * (1.f - i);
  d[1] = dc * cp * f * (1.f - f);
  d[2] = dc * i * (1.f - g * g);
  d[3] = dh * tc * o * (1.f - o);
  return dc * f;
}
// the cell backward of 4 consecutive units as two packed pairs (lstm_cell_bwd2; per element the
// operations of lstm_cell_bwd, so bit-identical to it): dh (recurrent + upstream), gates i f g o,
// c_t, c_{t-1}, dcf in / out; dd[v][q] the gate pre-activation gradients of unit v
template <class V4, class A4>
__device__ __forceinline__ void lstm_cell_bwd_x4(const V4& dh, const A4& i, const A4& f, const A4& g, const A4& o,
                                                 const V4& c, const V4& cp, float (&dcf)[4], float (&dd)[4][4]) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int v0 = 2 * p, v1 = 2 * p + 1;
    f2_t d2[4];
    const f2_t r = lstm_cell_bwd2(f2_t{dh[v0], dh[v1]}, f2_t{i[v0], i[v1]}, f2_t{f[v0], f[v1]}, f2_t{g[v0], g[v1]},
                                  f2_t{o[v0], o[v1]}, f2_t{c[v0], c[v1]}, f2_t{cp[v0], cp[v1]},
                                  f2_t{dcf[v0], dcf[v1]}, d2);
    dcf[v0] = r.x;
    dcf[v1] = r.y;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      dd[v0][q] = d2[q].x;
      dd[v1][q] = d2[q].y;
    }
  }
}

// recurrent-step tile: 64 batch rows x 32 hidden units (x 4 gates = 128 gate columns)
#define BF_BM 64
#define BF_U 32

// Caller-owned synchronisation block of the persistent recurrences (sv_sync_size() bytes,
// zeroed once by the caller; include/sv_ge2e.h).  u32 words:
//   [0]                       sticky status: 0 ok, bit 0 / bit 1 = a forward / backward hand-off
//                             wait timed out (every later wait on this block returns at once, so
//                             the launch drains; outputs since then are invalid)
//   [SV_SYNC_CNT ..)          arrival counters: SV_SYNC_CHANNELS channels x SV_PCNT_ROWS row
//                             blocks x SV_PCNT_STRIDE words (one 128-B line per counter); each
//                             launch zeroes the rows it uses of its channel, unless the stack
//                             forward zeroed them all (r06: the forward recurrences' channels
//                             0 .. L-1 and, from SV_BWD_CH0 on, the backward's, in its state-reset
//                             launch; a backward with SV_SCHED_CNT_READY then zeroes none)
//   [SV_SYNC_STAMP ..)        u64 phase stamps of the persistent backward (profiling)
#define SV_PCNT_ROWS 64
#define SV_PCNT_STRIDE 32
#define SV_SYNC_CHANNELS 8
#define SV_BWD_CH0 4  // the backward recurrences' channels: SV_BWD_CH0 + layer (wavefront: + its dW flags at + L)
#define SV_SYNC_CNT 32
#define SV_NSTAMP 8
#define SV_NSTAMP_WG 1024
#define SV_SYNC_STAMP (SV_SYNC_CNT + SV_SYNC_CHANNELS * SV_PCNT_ROWS * SV_PCNT_STRIDE)
#define SV_SYNC_WORDS (SV_SYNC_STAMP + 2 * SV_NSTAMP_WG * SV_NSTAMP)

// persistent forward recurrence of one layer (sv_persist.hip); sync: the caller's block, chan: its
// counter channel
extern "C" int sv_persist_fwd_ok(int B, int H);
int sv_persist_fwd_fusex_ok(int H, int F);
int sv_persist_fwd_bf16(int T, int B, int H, const bf16_t* whh_bf, bf16_t* gates, float* c_tm, float* h_tm,
                        bf16_t* h_bf, bf16_t* hT, hipStream_t stream, unsigned* sync, int chan = 0,
                        const bf16_t* x_bf = nullptr, int F = 0, const bf16_t* wih_bf = nullptr,
                        const float* b_ih = nullptr, const float* b_hh = nullptr, hipEvent_t pre = nullptr,
                        hipEvent_t post = nullptr, int counters_zeroed = 0);
// persistent backward recurrence of one layer (sv_persist.hip)
extern "C" int sv_persist_bwd_ok(int B, int H);
extern "C" size_t sv_persist_bwd_scratch(int T, int B, int H);
int sv_persist_bm(int B, int H, int cus);
struct DbFin;  // (below)
int sv_persist_bwd_bf16(int T, int B, int H, const bf16_t* whhT, const bf16_t* acts, const float* c_tm,
                        const float* dhup, int up_full, bf16_t* dg, bf16_t* dgT, bf16_t* dgf, hipStream_t stream,
                        unsigned* sync, float* db_ih = nullptr, float* db_hh = nullptr, hipEvent_t pre = nullptr,
                        hipEvent_t post = nullptr, int chan = 0, int counters_zeroed = 0,
                        DbFin* defer = nullptr);
// a persistent backward's bias-gradient finalize (db[c] = sum over the nrb row-block partials of
// column c, rows in order; db_hh gets the same sums), deferred into the launch that follows the
// recurrence (the dx GEMM, or the whole-K weight-gradient launch) as extra workgroups past its tiles:
// up to SV_DBF_MAX layers, G columns each
#define SV_DBF_MAX 3
struct DbFin {
  const float* dbp[SV_DBF_MAX];
  float* db_ih[SV_DBF_MAX];
  float* db_hh[SV_DBF_MAX];
  int n, nrb, G;
};
// workgroups of `threads` threads the finalize needs
__host__ __device__ inline int dbfin_blocks(const DbFin& f, int threads) {
  return f.n > 0 ? f.n * ((f.G + threads - 1) / threads) : 0;
}
// finalize workgroup `blk` (0 .. dbfin_blocks - 1) with blockDim.x threads
__device__ __forceinline__ void dbfin_run(const DbFin& f, int blk) {
  const int per = (f.G + (int)blockDim.x - 1) / (int)blockDim.x;
  const int l = blk / per, c = (blk % per) * (int)blockDim.x + (int)threadIdx.x;
  if (l >= f.n || c >= f.G) return;
  const float* p = l == 0 ? f.dbp[0] : l == 1 ? f.dbp[1] : f.dbp[2];
  float* o1 = l == 0 ? f.db_ih[0] : l == 1 ? f.db_ih[1] : f.db_ih[2];
  float* o2 = l == 0 ? f.db_hh[0] : l == 1 ? f.db_hh[1] : f.db_hh[2];
  float s = 0.f;
  for (int r = 0; r < f.nrb; ++r) s += p[(long)r * f.G + c];
  o1[c] = s;
  if (o2) o2[c] = s;
}
int sv_dbfin_launch(const DbFin& f, hipStream_t stream);  // as its own launch (sv_persist.hip)
// launcher of the wide-tile persistent backward (sv_persist3.hip; grid = nub x nrb workgroups)
int sv_persist3_bwd_launch(dim3 grid, int nub, hipStream_t stream, const bf16_t* whhT, const bf16_t* acts,
                           const float* c_tm, const float* dhup, int up_full, bf16_t* dg, bf16_t* dgT, long lddgT,
                           bf16_t* dgf, int T, int Bp, int B, int H, unsigned* cnt, int xcd, unsigned* sync,
                           unsigned limit, int fault, int dbg, float* dbp);
// launcher of the wide-tile persistent forward (sv_persist3.hip; no fused input projection)
int sv_persist3_fwd_launch(dim3 grid, int nub, hipStream_t stream, const bf16_t* whh_bf, bf16_t* gates, float* c_tm,
                           float* h_tm, bf16_t* h_bf, bf16_t* hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt,
                           int xcd, unsigned* status, unsigned limit, int fault, const bf16_t* x_bf = nullptr,
                           int F = 0, const bf16_t* wih_bf = nullptr, const float* b_ih = nullptr,
                           const float* b_hh = nullptr, int dbg = 0);
// launcher of the 16-row wide persistent forward (sv_persist3.hip; nrb x nub workgroups, H = 768,
// B % 16 == 0; x_bf: layer 0's input projection in the kernel, F = 40)
int sv_persist16_fwd_launch(int nrb, int nub, hipStream_t stream, const bf16_t* whh_bf, bf16_t* gates, float* c_tm,
                            float* h_tm, bf16_t* h_bf, bf16_t* hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt,
                            int xcd, unsigned* status, unsigned limit, int fault, const bf16_t* x_bf = nullptr,
                            int F = 0, const bf16_t* wih_bf = nullptr, const float* b_ih = nullptr,
                            const float* b_hh = nullptr);
// CUs of the device `stream` belongs to (cached per device); dims fit co-resident on `cus` CUs
int sv_stream_cus(hipStream_t stream);
int sv_persist_fwd_fits(int B, int H, int cus);
int sv_persist_bwd_fits(int B, int H, int cus);
// hand-off wait limit and the test-only fault switch (SV_PERSIST_FAULT) of the persistent kernels
unsigned sv_persist_limit();
int sv_persist_fault(int bwd);
// layer-wavefront forward (sv_wave.hip): all L layers in one launch for small B
int sv_wave_fwd_fits(int L, int T, int B, int F, int H, int cus);
int sv_wave_fwd_bf16(int L, int T, int B, int F, int H, const bf16_t* x_bf, const bf16_t* const* w_ih_bf,
                     const bf16_t* const* w_hh_bf, const float* const* b_ih, const float* const* b_hh,
                     bf16_t* const* gates, float* const* c_tm, float* const* h_tm, bf16_t* const* h_bf,
                     bf16_t* const* hT, unsigned* sync, hipStream_t stream, unsigned limit, int fault, hipEvent_t pre,
                     hipEvent_t post, int counters_zeroed = 0);
// layer-wavefront backward (sv_persist3.hip / sv_persist.hip): all L = 3 layers' recurrences and
// their upstream gradients dx in one launch, for the small per-GPU batches (B <= 80 at H = 768)
constexpr int WB_L = 3;
// Row stride (elements) of the library's own W_ih^T copies (bf16 [F][4H]) that the dx GEMMs read
// as their B operand: 4H + 64.  At 4H = 3072 a row is 6 KB, so the 256 rows of a k-tile
// fill all fell on one L2 channel; 64 more elements (128 B) spread them: the c3 dx GEMM 569 -> 478 us
// isolated (scripts/gemm_ld_ab.py).  Values only move: results are bit-identical.
inline long bf16_wiht_ld(int H) { return 4L * H + 64; }

struct WaveBwdArgs {
  const bf16_t* whhT[WB_L];  // [H][4H] bf16 (W_hh^T)
  const bf16_t* wihT[WB_L];  // [H][4H] bf16 (W_ih^T; layers >= 1)
  const bf16_t* acts[WB_L];  // [T][B][4H] bf16
  const float* c[WB_L];      // [T][B][H]
  float* dx[WB_L];           // [T][B][H] (layers >= 1): this layer's dx = layer l-1's dh_up
  bf16_t* dgf[WB_L];         // fragment-order dG hand-off, [T][nrb][4][32 rows][H] bf16
  bf16_t* dgT[WB_L];         // [4H][T Bp]
  float* dbp[WB_L];          // [nrb][4H] bias partials or NULL
  unsigned* cnt[WB_L];
  const float* dh_last;      // [B][H]: the top layer's dh_up at t = T-1
  unsigned* status;
  unsigned limit;
  long lddgT;
  int T, Bp, B, H, nub, nrb, fault;
  long ldwih;   // row stride of wihT (elements; bf16_wiht_ld)
};
int sv_wave_bwd_launch(const WaveBwdArgs& a, hipStream_t stream);
int sv_wave_bwd_fits(int L, int B, int H, int cus);
size_t sv_wave_bwd_scratch(int L, int T, int B, int H);
int sv_wave_bwd_bf16(int L, int T, int B, int H, const bf16_t* const* whhT, const bf16_t* const* wihT,
                     const bf16_t* const* acts, const float* const* c_tm, const float* dh_last, float* const* dx,
                     bf16_t* const* dgT, void* scratch, unsigned* sync, hipStream_t stream, float* const* db_ih,
                     float* const* db_hh, hipEvent_t pre, hipEvent_t post, long ldwih = 0,
                     int zero_next = 0, int ch0 = 0, int counters_zeroed = 0, DbFin* defer = nullptr);
