// Layer-wavefront persistent recurrences for small per-GPU batches (BASELINE c4: 8 speakers x
// 10 utterances = 80 rows per rank at 8 GPUs).
//
// Why: at B = 80 one layer's W-stationary recurrence (sv_persist.hip) is 3 row blocks x 24 unit
// blocks = 72 workgroups on 256 CUs, and the three layers run one after another, each behind its
// own input-projection GEMM.  Here ONE launch runs all layers: layer l's step t needs only layer
// l's h_{t-1} and layer l-1's h_t, so the layers advance as a wavefront (layer l one step behind
// layer l-1) on 3 x 72 = 216 co-resident workgroups, and the input projection x_t W_ih^T of the
// upper layers is computed in the recurrence itself (no K1 GEMM): T + L - 1 dependent steps
// instead of L x T.
//
// Workgroup (layer l, unit block ub, row block rb): 256 threads = 4 waves, one per SIMD (512
// registers each).  Wave g owns gate g of the tile's 32 units and holds BOTH its weight slices in
// registers for the whole launch: W_hh^l rows [g H + j0, +32) x K = H (48 bf16x8 MFMA B
// fragments) and W_ih^l's (48; layer 0: 3 over F = 40 features).  Per step it contracts
// h_{t-1}^l and x_t^l = h_t^{l-1} (layer 0: the frames, read straight from global) into ONE
// 32 x 32 accumulator with v_mfma_f32_32x32x16_bf16 (96 MFMAs), adds b_ih + b_hh, and the gate
// tiles meet in LDS for the cell update (the shared contraction-free lstm_cell_fwd; 4 units x 1
// row per thread).  Both A tiles (32 rows x H bf16) are staged into LDS with `sc1` loads.
// Hand-off of h_t^l: hand-off table row 1 of MI355X_MICROARCH.md, exactly as sv_persist.hip
// (16-B `sc1` stores of an LDS-staged bf16 tile, every storing wave drains vmcnt, workgroup
// barrier, one lane adds to its (layer, row block) counter in the caller's sync block; consumers
// poll with `sc1` loads, bounded, with the same sticky timeout status).
// Outputs are those of the per-layer schedule (activated gates, c, h fp32; h bf16 slots; hT), so
// the backward runs unchanged.
#include <algorithm>
#include "sv_bf16.h"
#include "sv_persist_dev.h"
#include "../../include/sv_ge2e.h"

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

namespace {
constexpr int WV_L = 3;       // layers of one wavefront launch (hp.model.num_layer)
constexpr int WV_BM = 32;     // rows per workgroup
constexpr int WV_NS = 48;     // k-steps of 16 over H = 768
constexpr int WV_XS = 3;      // k-steps of 16 over layer 0's F = 40 features (zero-padded to 48)
constexpr int WV_F = 40;
constexpr int WV_LDP = 4 * BF_U + 4;    // pre tile [32][LDP] fp32
constexpr int WV_LDB = BF_U + 8;        // hsb [32][LDB] bf16
constexpr int WV_LDT = WV_BM + 8;       // hts [32][LDT] bf16
constexpr int WV_NT = 256;              // threads per workgroup
}  // namespace

struct WaveFwd2Args {
  const bf16_t* whh[WV_L];   // [4H][H] bf16
  const bf16_t* wih[WV_L];   // [4H][F_l] bf16
  const float* bih[WV_L];
  const float* bhh[WV_L];
  bf16_t* gates[WV_L];       // [T][B][4H] activated, bf16
  float* c[WV_L];            // [T][B][H]
  float* h[WV_L];            // [T+1][B][H] (slot 0 = 0, written by the host)
  bf16_t* hb[WV_L];          // [T+1][B][H] bf16 (slot 0 = 0)
  bf16_t* hT[WV_L];          // [H][(T+1)Bp] or NULL
  const bf16_t* x_bf;        // [T][B][F]
  unsigned* cnt[WV_L];       // per-layer row-block counters (sync block channels)
  unsigned* status;
  unsigned limit;
  long ldhT;
  int T, Bp, B, H, nub, nrb, fault;
  int stamp;  // SV_WAVE3_STAMP=1 (profiling): per-phase s_memtime cycle sums into the sync block
  int dbg;    // SV_WAVE3_DEBUG (diagnostics)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wv_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

__device__ __forceinline__ void wv_wait(unsigned* c, unsigned target, unsigned* status, unsigned limit) {
  unsigned spins = 0;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    __builtin_amdgcn_s_sleep(2);
    if (++spins > limit) {
      __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}

// acc += A (the tile's LDS image) . W: fragments read 4 ahead (one full scheduling barrier per
// k-step keeps the reads that far ahead of their MFMAs)
__device__ __forceinline__ void w3_mfma_lds(const char* tile, int lane, const bf16x8_t (&W)[WV_NS], f32x16& acc) {
  const W3Frag frag(tile, lane);
  constexpr int P = 4;  // fragments in flight; one full scheduling barrier per k-step keeps them so
  bf16x8_t f[P];
#pragma unroll
  for (int j = 0; j < P; ++j) f[j] = frag(j);
#pragma unroll
  for (int s = 0; s < WV_NS; ++s) {
    acc = mfma_bf16(f[s % P], W[s], acc);
    if (s + P < WV_NS) f[s % P] = frag(s + P);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the same, with the 12 pieces of the next step's x-tile DMA (into `dtile`, slot ts of `rd`) issued
// one per 4 k-steps between the MFMAs (an LDS-DMA issue costs least among bare MFMAs:
// MI355X_MICROARCH.md, "LDS-DMA piece")
__device__ __forceinline__ void w3_mfma_lds_dma(const char* tile, int lane, const bf16x8_t (&W)[WV_NS], f32x16& acc,
                                                __amdgpu_buffer_rsrc_t rd, int ts, int B, int H, int b0, char* dtile,
                                                int g) {
  const W3Frag frag(tile, lane);
  constexpr int P = 4;
  bf16x8_t f[P];
#pragma unroll
  for (int j = 0; j < P; ++j) f[j] = frag(j);
#pragma unroll
  for (int s = 0; s < WV_NS; ++s) {
    acc = mfma_bf16(f[s % P], W[s], acc);
    if (s + P < WV_NS) f[s % P] = frag(s + P);
    if (s % 4 == 1) w3_dma_piece(rd, ts, B, H, b0, dtile, g, lane, s / 4);
    __builtin_amdgcn_sched_barrier(0);
  }
}


template <bool L0, bool STAMP>
__device__ __forceinline__ void w3_run(const WaveFwd2Args& a, int l, int ub, int rb, char* tile_x, char* tile_h,
                                       float* pre, bf16_t* hsb, bf16_t* hts) {
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int H = a.H, B = a.B, T = a.T, nub = a.nub;
  const int j0 = ub * BF_U, b0 = rb * WV_BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  unsigned* my_cnt = a.cnt[l] + rb * SV_PCNT_STRIDE;
  unsigned* below = L0 ? nullptr : a.cnt[l - 1] + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  const int dbg = a.dbg & SV_PDBG;  // (diagnostic bits: A/B builds with -DSV_PDBG=-1 only)
  const bool wok = j0 + r < H;
  bf16x8_t wh[WV_NS], wx[WV_NS];
  {
    const bf16_t* rh = a.whh[l] + ((long)g * H + j0 + r) * H + 8 * hh;
    const int K = L0 ? WV_F : H;
    const bf16_t* rx = a.wih[l] + ((long)g * H + j0 + r) * K + 8 * hh;
#pragma unroll
    for (int s = 0; s < WV_NS; ++s) {
      bf16x8_t z = {};
      wh[s] = wok ? *reinterpret_cast<const bf16x8_t*>(rh + 16 * s) : z;
      wx[s] = (wok && 16 * s + 8 * hh < K) ? *reinterpret_cast<const bf16x8_t*>(rx + 16 * s) : z;
    }
  }
  float xbias = 0.f;
  if (wok) {
    const int col = g * H + j0 + r;
    xbias = a.bih[l][col] + a.bhh[l][col];
  }
  const int u4 = (tid & 7) * 4, brow = tid >> 3;
  const long gb = b0 + brow;
  float cst[4] = {0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rxs = wv_rsrc(a.x_bf, (unsigned)((long)T * B * WV_F * 2));
  const unsigned hbytes = (unsigned)((long)(T + 1) * BH * 2);
  const __amdgpu_buffer_rsrc_t rown = wv_rsrc(a.hb[l], hbytes);
  const __amdgpu_buffer_rsrc_t rbel = wv_rsrc(L0 ? a.hb[l] : a.hb[l - 1], hbytes);
  if constexpr (!L0) {  // x_0 = h_0^{l-1}
    if (tid == 0) wv_wait(below, producers, a.status, a.limit);
    __syncthreads();
    w3_dma(rbel, 1, B, H, b0, tile_x, g, lane);
  }
  // raw barriers (no fence) where a DMA is in flight: __syncthreads' release fence would drain it
  auto raw_barrier = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // STAMP is a template parameter, not a runtime test: a branch between an MFMA and the reads of
  // its accumulators made the compiler's hazard padding too short (the first AGPR read returned a
  // stale a15: rows 27 and 31 of every tile wrong)
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = STAMP ? __builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int i) {
    if constexpr (STAMP) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      ph[i] += now - tlast;
      tlast = now;
    }
  };
  for (int t = 0; t < T; ++t) {
    // h_{t-1} (t = 0: slot 0, zeros -- the h-part then adds exact zeros, so every step has the
    // same DMA / wait shape and the compiler can count the waits)
    if (tid == 0 && t > 0) wv_wait(my_cnt, producers * (unsigned)t, a.status, a.limit);
    if (dbg & 1)
      __syncthreads();  // debug: drain everything (the x DMA too) here
    else
      raw_barrier();
    mark(0);
    w3_dma(rown, t, B, H, b0, tile_h, g, lane);
    mark(1);
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    unsigned xpoll = 0;
    if constexpr (!L0) {
      // this wave's x DMA and everything older (the 12 h DMAs are the newest), then all waves'
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      raw_barrier();
      // the layer below's counter for step t + 1's x tile, read now: its round trip runs under the
      // x-part, and the answer decides at the h-part whether that DMA goes there
      if (tid == 0 && t + 1 < T) xpoll = __hip_atomic_load(below, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      w3_mfma_lds(tile_x, lane, wx, acc);
    } else {
      u32x4_t xa[WV_XS];
#pragma unroll
      for (int s = 0; s < WV_XS; ++s) {  // rows past B: zeros (offset past the step's rows)
        const unsigned off = 16 * s + 8 * hh < WV_F
                                 ? ((unsigned)t * (unsigned)(B * WV_F) + (unsigned)min(b0 + r, B) * (unsigned)WV_F +
                                    (b0 + r < B ? 16 * s + 8 * hh : 0)) * 2u
                                 : 0xFFFFFFF0u;
        xa[s] = __builtin_amdgcn_raw_buffer_load_b128(rxs, b0 + r < B ? off : 0xFFFFFFF0u, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < WV_XS; ++s) acc = mfma_bf16(__builtin_bit_cast(bf16x8_t, xa[s]), wx[s], acc);
    }
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const f2_t v = round_bf2(f2_t{acc[i], acc[i + 1]}, xbias);
      acc[i] = v.x;
      acc[i + 1] = v.y;
    }
    mark(2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __shared__ int xflag;
    if (!L0 && tid == 0) xflag = (t + 1 < T && xpoll >= producers * (unsigned)(t + 2) && !(dbg & 2)) ? 1 : 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // every wave past the x-part: tile_x is free
    bool xe = false;
    if constexpr (!L0) xe = xflag != 0;
    if (xe)
      w3_mfma_lds_dma(tile_h, lane, wh, acc, rbel, t + 2, B, H, b0, tile_x, g);
    else
      w3_mfma_lds(tile_h, lane, wh, acc);
    mark(3);
#pragma unroll
    for (int i = 0; i < 16; ++i) pre[acc_row(i, lane) * WV_LDP + g * BF_U + r] = acc[i];
    __syncthreads();
    uint2 act[4];
    float4 cv, hv;
    {
      float4 pq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pq[q] = *reinterpret_cast<const float4*>(pre + brow * WV_LDP + q * BF_U + u4);
      float ao[4][4], co[4], ho[4];
      unsigned pk[2] = {0u, 0u};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float pv[4] = {pq[0][v], pq[1][v], pq[2][v], pq[3][v]};
        const float xv[4] = {0.f, 0.f, 0.f, 0.f};
        float a4[4], h;
        const float c = lstm_cell_fwd(pv, xv, cst[v], a4, h);
        cst[v] = c;
#pragma unroll
        for (int q = 0; q < 4; ++q) ao[q][v] = a4[q];
        co[v] = c;
        ho[v] = h;
      }
      pk[0] = pack_bf2(ho[0], ho[1]);
      pk[1] = pack_bf2(ho[2], ho[3]);
#pragma unroll
      for (int v = 0; v < 4; ++v) hts[(u4 + v) * WV_LDT + brow] = (bf16_t)(pk[v >> 1] >> (16 * (v & 1)));
      *reinterpret_cast<uint2*>(hsb + brow * WV_LDB + u4) = uint2{pk[0], pk[1]};
#pragma unroll
      for (int q = 0; q < 4; ++q) act[q] = pack_bf4(ao[q][0], ao[q][1], ao[q][2], ao[q][3]);
      cv = float4{co[0], co[1], co[2], co[3]};
      hv = float4{ho[0], ho[1], ho[2], ho[3]};
    }
    __syncthreads();
    mark(4);
    if (tid < WV_BM * 4) {
      const int row = tid >> 2, c = tid & 3, gr = b0 + row;
      const __amdgpu_buffer_rsrc_t rw = wv_rsrc(a.hb[l] + (long)(t + 1) * BH, (unsigned)(BH * 2));
      if (gr < B && j0 + 8 * c < H) {
        const uint4 v = *reinterpret_cast<const uint4*>(hsb + row * WV_LDB + 8 * c);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw,
                                               ((unsigned)gr * (unsigned)H + (unsigned)(j0 + 8 * c)) * 2u, 0,
                                               16 /* sc1 */);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && !(a.fault && t == 0 && blockIdx.x == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mark(5);
    // off the critical chain: activations, c, h and hT of step t (before the next x DMA, so the
    // counted wait above sees only DMAs behind it)
    if (gb < B && j0 + u4 < H) {
      bf16_t* gp = a.gates[l] + (long)t * BG + gb * G + j0 + u4;
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(gp + q * H) = act[q];
      *reinterpret_cast<float4*>(a.c[l] + (long)t * BH + gb * H + j0 + u4) = cv;
      if (t == T - 1) *reinterpret_cast<float4*>(a.h[l] + (long)(t + 1) * BH + gb * H + j0 + u4) = hv;  // h_{T-1} only
    }
    if (a.hT[l] && tid < BF_U * (WV_BM / 8)) {
      const int u = tid >> 2, c = tid & 3, gc = b0 + 8 * c;
      if (gc < a.Bp && j0 + u < H) {
        bf16_t* row = a.hT[l] + (long)(j0 + u) * a.ldhT;
        *reinterpret_cast<uint4*>(row + (long)(t + 1) * a.Bp + gc) = *reinterpret_cast<const uint4*>(hts + u * WV_LDT + 8 * c);
        if (t == 0) *reinterpret_cast<uint4*>(row + gc) = uint4{0u, 0u, 0u, 0u};
      }
    }
    if (!L0 && t + 1 < T && !xe) {  // x_{t+1}: tile_x is free (every wave is past this step's x-part)
      if (tid == 0) wv_wait(below, producers * (unsigned)(t + 2), a.status, a.limit);
      raw_barrier();
      w3_dma(rbel, t + 2, B, H, b0, tile_x, g, lane);
    }
    mark(6);
  }
  if (STAMP && tid == 0 && blockIdx.x < SV_NSTAMP_WG) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(a.status + SV_SYNC_STAMP) + blockIdx.x * SV_NSTAMP;
    for (int i = 0; i < 7; ++i) st[i] = ph[i];
    st[7] = (unsigned long long)l;
  }
}

template <bool STAMP>
__global__ __launch_bounds__(256, 1) void lstm_wave3_fwd_bf16_kernel(const WaveFwd2Args a) {
  __shared__ __attribute__((aligned(16))) char tile_x[W3_TILE];
  __shared__ __attribute__((aligned(16))) char tile_h[W3_TILE];
  __shared__ __attribute__((aligned(16))) float pre[WV_BM * WV_LDP];
  __shared__ __attribute__((aligned(16))) bf16_t hsb[WV_BM * WV_LDB];
  __shared__ __attribute__((aligned(16))) bf16_t hts[BF_U * WV_LDT];
  const int nub = a.nub;
  int ub, rb, l;
  {
    const int i = blockIdx.x, n = gridDim.x;
    const int x = i & 7, q = n >> 3, rr = n & 7;
    const int L = x * q + min(x, rr) + (i >> 3);
    ub = L % nub;
    rb = (L / nub) % a.nrb;
    l = L / (nub * a.nrb);
  }
  if (l == 0)
    w3_run<true, STAMP>(a, l, ub, rb, tile_x, tile_h, pre, hsb, hts);
  else
    w3_run<false, STAMP>(a, l, ub, rb, tile_x, tile_h, pre, hsb, hts);
}

// ---- host ----
// can the layer-wavefront forward run these dims co-resident on a device of `cus` CUs?
// (the DMA addresses of the h slots are 32-bit buffer offsets: (T + 1) B H bf16 < 4 GiB)
int sv_wave_fwd_fits(int L, int T, int B, int F, int H, int cus) {
  const int nub = (H + BF_U - 1) / BF_U, nrb = (B + WV_BM - 1) / WV_BM;
  return L == WV_L && H == WV_NS * 16 && F == WV_F && nrb <= SV_PCNT_ROWS && (long)L * nub * nrb <= cus &&
         (long)B * H * 2 < (1L << 31) && (long)(T + 1) * B * H * 2 < (1L << 32) - (1L << 20);
}

// all L layers' recurrences of the bf16 stack forward in one launch (no K1 GEMMs): writes what the
// per-layer schedule writes.  h_tm / h_bf slot 0 and padded hT columns must be zero (the caller's
// memsets).  Counter channels 0..L-1 of `sync` (zeroed here unless counters_zeroed).
int sv_wave_fwd_bf16(int L, int T, int B, int F, int H, const bf16_t* x_bf, const bf16_t* const* w_ih_bf,
                     const bf16_t* const* w_hh_bf, const float* const* b_ih, const float* const* b_hh,
                     bf16_t* const* gates, float* const* c_tm, float* const* h_tm, bf16_t* const* h_bf,
                     bf16_t* const* hT, unsigned* sync, hipStream_t stream, unsigned limit, int fault, hipEvent_t pre,
                     hipEvent_t post, int counters_zeroed) {
  if (!sv_wave_fwd_fits(L, T, B, F, H, sv_stream_cus(stream))) return SV_ESHAPE;
  if (!sync || !x_bf) return SV_EARG;
  WaveFwd2Args a{};
  a.nub = (H + BF_U - 1) / BF_U;
  a.nrb = (B + WV_BM - 1) / WV_BM;
  for (int l = 0; l < L; ++l) {
    a.whh[l] = w_hh_bf[l];
    a.wih[l] = w_ih_bf[l];
    a.bih[l] = b_ih[l];
    a.bhh[l] = b_hh[l];
    a.gates[l] = gates[l];
    a.c[l] = c_tm[l];
    a.h[l] = h_tm[l];
    a.hb[l] = h_bf[l];
    a.hT[l] = hT[l];
    a.cnt[l] = sync + SV_SYNC_CNT + (size_t)l * SV_PCNT_ROWS * SV_PCNT_STRIDE;
  }
  // counters_zeroed: the caller zeroed channels 0..L-1 in its state-reset launch
  if (!counters_zeroed)
    if (int rc = sv_zero_counters(a.cnt[0], L, (long)SV_PCNT_ROWS * SV_PCNT_STRIDE, a.nrb * SV_PCNT_STRIDE, stream))
      return rc;
  a.x_bf = x_bf;
  a.status = sync;
  a.limit = limit;
  a.fault = fault;
  a.T = T;
  a.B = B;
  a.H = H;
  a.Bp = (B + 7) & ~7;
  a.ldhT = (long)(T + 1) * a.Bp;
  hipError_t e;
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;
  // LDS-DMA staging of both A tiles (wave3).  The register-staged form (wave2: eight dependent
  // global round trips per step, same products in the same order) measured 1.20 vs 0.85 ms for
  // the c4 rank-shape forward.
  a.dbg = 0;
#ifdef SV_WAVE3_STAMP  // A/B stamp builds only: per-phase cycle sums of wave 0, workgroups < 512
  a.stamp = 1;
  hipLaunchKernelGGL(lstm_wave3_fwd_bf16_kernel<true>, dim3(L * a.nub * a.nrb), dim3(WV_NT), 0, stream, a);
#else
  a.stamp = 0;
  hipLaunchKernelGGL(lstm_wave3_fwd_bf16_kernel<false>, dim3(L * a.nub * a.nrb), dim3(WV_NT), 0, stream, a);
#endif
  SV_LAUNCH_CHECK();
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  return SV_OK;
}
