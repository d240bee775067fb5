// W-stationary persistent recurrences of the fp32 path (config c2: exact fp32 MFMA products).
//
// Why: the per-step fp32 kernels (K2 lstm_step_fwd_v2_kernel / K3 lstm_step_bwd_v2_kernel) stream
// their W_hh tile (393 KB per workgroup) from L2 every timestep and run at 53 % / 45 % of the fp32
// MFMA rate alone, less beside the layer pipeline's GEMMs.  Here ONE launch per layer runs all T
// steps with each workgroup's W_hh slice held in registers for the whole sequence, so a step is
// bound by its MFMAs (v_mfma_f32_32x32x2_f32, 64 cycles each) plus one hand-off.
//
// Tile (H = 768): 64 batch rows x 32 hidden units x 4 gates; grid (H / 32) x ceil(B / 64) = 240
// workgroups at B = 640, one per CU (4 waves, 512 registers each).  Wave g holds gate g's weights
// for its 32 units over K = H: 96 k-groups of 8 = 384 fp32 registers per lane (256 AGPRs + 128
// VGPRs).  A k-group's 4 MFMAs take k = 8 kg + 4 h + c (c = 0..3) from lane half h: a fixed
// permutation of the summation order applied to both operands, so every operand fetch is 16 B.
//
// Forward: h_{t-1} of the 64 rows (196 KB) is staged through a 4-slot LDS ring of 64-k chunks by
// LDS-DMA (global_load_lds, sc1), two chunks ahead, one barrier per chunk; the four waves share each
// chunk.  The x-projection of step t (K1 output incl. biases, in `gates`) arrives by the same DMA.
// Hand-off: h_t through h_tm[t + 1] (16-B sc1 stores, vmcnt(0), one arrival per workgroup on the row
// block's counter; MI355X_MICROARCH.md hand-off table row 1), read back with sc1 DMA.
// Backward: dh_rec = dG_{t+1} W_hh: wave g streams gate g's K = H slice of dG_{t+1} from a
// fragment-order hand-off buffer straight into registers (1 KB per load instruction), 12 k-groups
// ahead, as two 32-row half chains (below); the per-gate partials meet in LDS and are summed in
// gate order (K3's order).
// Outputs are the per-step kernels' buffers (activations, c, h, h^T / dG, dG^T), so either direction
// composes with the other schedule; results agree with the per-step kernels to fp32 rounding.
#include <algorithm>

#include "sv_persist_dev.h"
#include "../../include/sv_ge2e.h"

namespace {
constexpr int PF_BM = 64, PF_U = 32;
constexpr int PF_KC = 64;                  // k per forward A chunk
constexpr int PF_CH = PF_BM * PF_KC * 4;   // 16 KB
constexpr int PF_NB = 4;                   // ring slots (chunk c + 2 is issued while c is consumed)
constexpr int PF_NA = 64;                  // weight k-groups in AGPRs (4 x 64 = 256 registers)
constexpr int PF_XCD = 1;                  // XCD-grouped tile order (persist_tile)
typedef __attribute__((address_space(3))) void* pf_lds_t;
typedef __attribute__((address_space(1))) void* pf_glb_t;

// LDS slot of 16-B chunk s of row `row` in a [64][64 k] fp32 ring chunk (an involution)
__device__ __forceinline__ int pf_slot(int row, int s) { return s ^ (row & 15); }

// a lane's weight k-groups (16 B each, k-group kg at w + stride kg): the first PF_NA into AGPRs
// (pinned element by element), NV into VGPRs, NL into the wave's LDS slots (lane-strided 1 KB)
template <int NV, int NL>
__device__ __forceinline__ void pf_load_w(const float* w, int stride, float (&wa)[4 * PF_NA], float (&wv)[4 * NV],
                                          char* wl) {
#pragma unroll
  for (int s = 0; s < PF_NA; ++s) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(w + stride * s);
#pragma unroll
    for (int c = 0; c < 4; ++c) wa[4 * s + c] = x[c];
  }
#pragma unroll
  for (int s = 0; s < NV; ++s) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(w + stride * (PF_NA + s));
#pragma unroll
    for (int c = 0; c < 4; ++c) wv[4 * s + c] = x[c];
  }
#pragma unroll
  for (int s = 0; s < NL; ++s)
    *reinterpret_cast<f32x4*>(wl + s * 1024) = *reinterpret_cast<const f32x4*>(w + stride * (PF_NA + NV + s));
#pragma unroll
  for (int i = 0; i < 4 * PF_NA; ++i) asm volatile("" : "+a"(wa[i]));
}

template <int N>
__device__ __forceinline__ void pf_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
}  // namespace

// ============================================================================
// forward
// ============================================================================
// NV / NL: weight k-groups kept in VGPRs / in LDS (after the PF_NA in AGPRs)
// XKG > 0 (layer 0, F = 8 XKG input features): the input projection x_t W_ih^T is formed in the
// kernel (no K1 GEMM, no x-projection round trip through HBM): W_ih fragments, the x_t tile and
// b_ih + b_hh live in the x-projection's LDS region; the x-part's MFMAs run at the top of each step,
// before the hand-off wait (they need no h_{t-1}), and start the accumulators the h-part adds to.
template <int NKG, int NV, int NL, int XKG = 0>
__global__ __launch_bounds__(256, 1) void lstm_persist_fwd_f32_kernel(
    const float* __restrict__ whh, float* gates, float* __restrict__ c_tm, float* h_tm, float* __restrict__ hT,
    long ldhT, int T, int Bp, int B, unsigned* cnt, int nub, int xcd, unsigned* status, unsigned limit, int fault,
    const float* __restrict__ x_tm = nullptr, const float* __restrict__ wih = nullptr,
    const float* __restrict__ b_ih = nullptr, const float* __restrict__ b_hh = nullptr) {
  constexpr int H = 8 * NKG, NCH = H / PF_KC, KGC = PF_KC / 8;
  constexpr int XF = 8 * XKG, XLD = XF + 4;  // x tile [64][XLD] fp32 (an odd 16-B row stride: conflict-free)
  constexpr int XSL = XLD / 4;               // 16-B slots per x-tile row
  constexpr int GXN = XKG ? 0 : 8;           // x-projection DMA ops per wave in the k-loop's counted waits
  static_assert(XKG == 0 || (4 * XKG * 1024 + 4 * PF_U * 4 + PF_BM * PF_U * 4 <= PF_BM * 4 * PF_U * 4 &&
                             PF_BM * XLD * 4 <= PF_CH && XSL % 2 == 1 &&
                             (PF_BM * (4 * PF_U + 4) + PF_U * (PF_BM + 4)) * 4 <= 3 * PF_CH),
                "W_ih + biases + c fit the x-projection region; the x tile ring slot 3, above pre + hts");
  static_assert(NCH >= 4 && H % PF_KC == 0 && PF_NA + NV + NL == NKG, "chunk schedule / weight split");
  constexpr int LDP = 4 * PF_U + 4;  // pre [64][LDP] fp32
  constexpr int LDH = PF_BM + 4;     // hts [32][LDH] fp32
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem;                                            // [NB][64 rows][256 B]
  float* gxs = reinterpret_cast<float*>(smem + PF_NB * PF_CH);  // [64][4 * 32] x-projection of step t
  char* wl = smem + PF_NB * PF_CH + PF_BM * 4 * PF_U * 4;       // [4 waves][NL][64 lanes][16 B]
  float* pre = reinterpret_cast<float*>(smem);                  // after the k-loop: aliases the ring
  float* hts = pre + PF_BM * LDP;                               // (aliases the ring too)
  // XKG: x tile, W_ih fragments and biases in the x-projection region; c staged in the ring
  // (the x tile lives in ring slot 3, free from the end of one k-loop to the next step's chunk-3 DMA,
  // above pre + hts; W_ih, the biases and the step's c in the x-projection region)
  float* xs = reinterpret_cast<float*>(ring + 3 * PF_CH);           // [64][XLD]
  char* wil = reinterpret_cast<char*>(gxs);                         // [4 waves][XKG][64 lanes][16 B]
  float* bsl = reinterpret_cast<float*>(wil + 4 * XKG * 1024);      // [4 gates][32 units] b_ih + b_hh
  float* cst = XKG ? bsl + 4 * PF_U : gxs;                          // c_t of the step (row stride CLD)
  constexpr int CLD = XKG ? PF_U : 4 * PF_U;
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * PF_U, b0 = rb * PF_BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  // x_t's tile by LDS-DMA: 64 rows x XSL slots lane-linear, wave g issuing instructions g, g + 4, ...;
  // the pad slot of a row re-reads its last data slot (never read back)
  auto dma_x = [&](int tt) {
    if constexpr (XKG > 0) {
      constexpr int NI = (PF_BM * XSL + 63) / 64;
      int z = 0;  // (an opaque zero: no per-lane offset hoisted out of the time loop into registers)
      asm volatile("" : "+v"(z));
      const __amdgpu_buffer_rsrc_t rx = sv_rsrc(x_tm + (long)tt * B * XF, (unsigned)((long)B * XF * 4));
#pragma unroll
      for (int jj = 0; jj < (NI + 3) / 4; ++jj) {
        const int j = 4 * jj + g;
        if (j < NI) {  // (wave-uniform)
          const int q = 64 * j + lane + z, row = min(q / XSL, PF_BM - 1), sl = min(q % XSL, XSL - 2);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(reinterpret_cast<char*>(xs) + j * 1024), 16,
                                                   (unsigned)((min(b0 + row, B - 1) * XF + 4 * sl) * 4), 0, 0, 0);
        }
      }
    }
  };
  if constexpr (XKG > 0) {
    // W_ih of gate g, units j0 + r: lane (r, hh) of k-group kg holds W_ih[g H + j0 + r][8 kg + 4 hh .. + 3]
#pragma unroll
    for (int kg = 0; kg < XKG; ++kg)
      *reinterpret_cast<f32x4*>(wil + ((g * XKG + kg) * 64 + lane) * 16) =
          *reinterpret_cast<const f32x4*>(wih + ((long)g * H + j0 + r) * XF + 8 * kg + 4 * hh);
    if (tid < 4 * PF_U) {
      const long col = (long)(tid >> 5) * H + j0 + (tid & 31);
      bsl[tid] = (b_ih ? b_ih[col] : 0.f) + (b_hh ? b_hh[col] : 0.f);
    }
    dma_x(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // W_hh of gate g, units j0 + r: lane (r, hh) of k-group kg holds W[g H + j0 + r][8 kg + 4 hh .. + 3]
  // (one scalar per register: pinned element by element to AGPRs, the MFMAs read them in place)
  float wa[4 * PF_NA], wv[4 * NV];
  {
    const float* wr = whh + ((long)g * H + j0 + r) * H + 4 * hh;
    pf_load_w<NV, NL>(wr, 8, wa, wv, wl + (g * NL * 64 + lane) * 16);
  }
  auto wfrag = [&](int kg) -> f32x4 {  // (kg a compile-time constant after unrolling)
    if (kg < PF_NA) {
      const int b = 4 * (kg < PF_NA ? kg : 0);
      return f32x4{wa[b], wa[b + 1], wa[b + 2], wa[b + 3]};
    }
    if (kg < PF_NA + NV) {
      const int b = 4 * (kg < PF_NA + NV && kg >= PF_NA ? kg - PF_NA : 0);
      return f32x4{wv[b], wv[b + 1], wv[b + 2], wv[b + 3]};
    }
    return *reinterpret_cast<const f32x4*>(wl + ((g * NL + (kg - PF_NA - NV)) * 64 + lane) * 16);
  };
  // elementwise map: thread -> units 4 quad .. + 3 of rows 2 rp, 2 rp + 1
  const int quad = tid & 7, rp = tid >> 3;
  float cs[2][4];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v) cs[k][v] = 0.f;
#ifdef SV_PF32_STAMP  // A/B stamp builds only: wave 0's cycles per phase, summed over steps 1 .. T-1
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tl = 0;
  auto stamp = [&](int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (i >= 0) ph[i] += n - tl;
    tl = n;
  };
#define PF_STAMP(i) if (t > 0) stamp(i)
#else
#define PF_STAMP(i)
#endif
  for (int t = 0; t < T; ++t) {
    PF_STAMP(-1);
    // the wave index through an opaque SGPR copy: the DMA address arithmetic stays inside the step
    // (hoisted out of the time loop, the per-lane addresses would hold registers the weights need)
    // and scalar where it is uniform -- the step's base in a buffer descriptor, a row group's LDS
    // address (M0) and the chunk offset in SALU, 32-bit per-lane offsets -- where an opaque VGPR
    // zero made every address a 64-bit VALU chain with a v_readfirstlane for M0
    int gs = __builtin_amdgcn_readfirstlane(g);
    asm volatile("" : "+s"(gs));
    const __amdgpu_buffer_rsrc_t rh = sv_rsrc(h_tm + (long)t * B * H, (unsigned)((long)B * H * 4));
    const __amdgpu_buffer_rsrc_t rg = sv_rsrc(gates + (long)t * BG, (unsigned)(BG * 4));
    auto dma_chunk = [&](int ch, int slot) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rowu = 16 * gs + 4 * j, rl = lane >> 4, row = rowu + rl;
        const unsigned vo = (__umul24((unsigned)min(b0 + row, B - 1), (unsigned)H) + 4u * ((lane & 15) ^ (4 * j + rl))) * 4u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, (pf_lds_t)(ring + slot * PF_CH + rowu * 256), 16, vo,
                                                 (unsigned)(ch * PF_KC * 4), 0, 16 /* sc1 */);
      }
    };
    auto dma_gx = [&]() {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rowu = 2 * (8 * gs + j), row = rowu + (lane >> 5), s = lane & 31;
        const unsigned vo =
            (__umul24((unsigned)min(b0 + row, B - 1), (unsigned)G) + (unsigned)((s >> 3) * H + j0 + 4 * (s & 7))) * 4u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (pf_lds_t)(gxs + (8 * gs + j) * 256), 16, vo, 0, 0, 0);
      }
    };
    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
    if constexpr (XKG > 0) {  // x_t W_ih^T (x_t landed and visible: the previous step's drain + barrier)
#pragma unroll
      for (int kg = 0; kg < XKG; ++kg) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + r * XLD + 8 * kg + 4 * hh);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + (32 + r) * XLD + 8 * kg + 4 * hh);
        const f32x4 wx = *reinterpret_cast<const f32x4*>(wil + ((g * XKG + kg) * 64 + lane) * 16);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[c], wx[c], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[c], wx[c], acc1, 0, 0, 0);
        }
      }
    }
    if (t > 0) {
      if (tid == 0) {
        persist_wait(my_cnt, (unsigned)nub * (unsigned)t, status, limit, 1u);
      }
      __syncthreads();
      PF_STAMP(0);  // 0: hand-off wait
      dma_chunk(0, 0);
      dma_chunk(1, 1);
      // fragments two k-groups ahead, across chunk boundaries: chunk ch + 1's wait and barrier come
      // before the last two k-groups of chunk ch, so its first fragments are read while those run.
      // Waits (this wave's ops younger than chunk c + 1's four): chunk c + 2's and, for c <= 1, the
      // x-projection's eight (issued at chunk 0, behind chunk 2's) -- c = 0, 1: 12; then 4; last: 0.
      pf_vmwait<4>();  // chunk 0 (chunk 1 in flight)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      PF_STAMP(1);  // 1: first chunk's DMA latency
      auto afrag = [&](int kg, f32x4& x0, f32x4& x1) {
        const char* cb = ring + ((kg / KGC) % PF_NB) * PF_CH;
        const int kk = kg % KGC;
        x0 = *reinterpret_cast<const f32x4*>(cb + r * 256 + 16 * pf_slot(r, 2 * kk + hh));
        x1 = *reinterpret_cast<const f32x4*>(cb + (32 + r) * 256 + 16 * pf_slot(32 + r, 2 * kk + hh));
      };
      f32x4 a0, a1, b0_, b1_, w = wfrag(0), wn = wfrag(1);
      afrag(0, a0, a1);
      afrag(1, b0_, b1_);
#pragma unroll
      for (int kg = 0; kg < NKG; ++kg) {
        const int ch = kg / KGC, kk = kg % KGC;
        if (kk == 0 && ch + 2 < NCH) dma_chunk(ch + 2, (ch + 2) % PF_NB);
        if (XKG == 0 && kg == 0) dma_gx();
        if (kk == KGC - 2 && ch + 1 < NCH) {  // chunk ch + 1 landed, every wave's part
          if (ch <= 1)
            pf_vmwait<4 + GXN>();
          else if (ch + 2 < NCH)
            pf_vmwait<4>();
          else
            pf_vmwait<0>();
          __builtin_amdgcn_s_barrier();  // (slot (ch + 3) % 4's last reads, chunk ch - 1's, are done)
          asm volatile("" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
        // the first MFMA pair, then k-group kg + 2's reads, then the rest: hipcc waits lgkmcnt(0)
        // before a k-group's first MFMA (every outstanding LDS read), so reads issued after it have
        // the group's other six MFMAs before the next such wait
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[0], w[0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[0], w[0], acc1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        f32x4 n0 = a0, n1 = a1, nw = w;
        if (kg + 2 < NKG) {
          afrag(kg + 2, n0, n1);
          nw = wfrag(kg + 2);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 1; c < 4; ++c) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[c], w[c], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[c], w[c], acc1, 0, 0, 0);
        }
        a0 = b0_;
        a1 = b1_;
        w = wn;
        b0_ = n0;
        b1_ = n1;
        wn = nw;
        __builtin_amdgcn_sched_barrier(0);
      }
      pf_vmwait<0>();  // the x-projection (already waited for by the chunk waits; kept explicit)
    } else {
      if constexpr (XKG == 0) {
        dma_gx();
        pf_vmwait<0>();
      }
    }
    PF_STAMP(2);  // 2: k-loop after the first chunk
    __syncthreads();  // every wave done with the ring (pre aliases it) and its gxs part landed
    // XKG: x_{t+1} into ring slot 3 now (this step's x-part read x_t there before the poll barrier;
    // the hand-off drain below waits for it, the cell's 2-3k cycles after its issue)
    if (XKG > 0 && t + 1 < T) dma_x(t + 1);
    // pre-activation exchange: wave g's row halves -> pre[row][g 32 + unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pre[acc_row(i, lane) * LDP + g * PF_U + r] = acc0[i];
      pre[(32 + acc_row(i, lane)) * LDP + g * PF_U + r] = acc1[i];
    }
    __syncthreads();
    // cell update; the activations go back into pre and c into gxs's gate-0 slot, in place (each
    // thread rewrites only the positions it read), for the stores after the arrival
    f32x4 hv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = 2 * rp + k;
      f32x4 p[4], x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        p[q] = *reinterpret_cast<const f32x4*>(pre + row * LDP + q * PF_U + 4 * quad);
        x[q] = *reinterpret_cast<const f32x4*>(XKG ? bsl + q * PF_U + 4 * quad
                                                   : gxs + row * (4 * PF_U) + q * PF_U + 4 * quad);
      }
      f32x4 cv;
#pragma unroll
      for (int v = 0; v < 4; ++v) {  // the per-step kernel's cell (lstm_step_fwd_v2_kernel)
        const float i_ = sv_sigmoid(p[0][v] + x[0][v]);
        const float f_ = sv_sigmoid(p[1][v] + x[1][v]);
        const float g_ = sv_tanh(p[2][v] + x[2][v]);
        const float o_ = sv_sigmoid(p[3][v] + x[3][v]);
        const float c = f_ * cs[k][v] + i_ * g_;
        cs[k][v] = c;
        cv[v] = c;
        hv[k][v] = o_ * sv_tanh(c);
        p[0][v] = i_;
        p[1][v] = f_;
        p[2][v] = g_;
        p[3][v] = o_;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(pre + row * LDP + q * PF_U + 4 * quad) = p[q];
      *reinterpret_cast<f32x4*>(cst + row * CLD + 4 * quad) = cv;
    }
    PF_STAMP(3);  // 3: exchange + cell
    // the hand-off: h_t into h_tm[t + 1], 16-B sc1 stores, drained before the arrival
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int gb = b0 + 2 * rp + k;
      if (gb < B) {
        const __amdgpu_buffer_rsrc_t rw = sv_rsrc(h_tm + (long)(t + 1) * BH, (unsigned)(BH * 4));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, hv[k]), rw,
                                               ((unsigned)gb * (unsigned)H + (unsigned)(j0 + 4 * quad)) * 4u, 0,
                                               16 /* sc1 */);
      }
    }
    // off the chain, after the arrival: activations, c, h^T of step t (issuing them behind the
    // hand-off stores, before their drain, measured slower: DESIGN §4)
    auto offchain = [&]() {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int row = 2 * rp + k;
        const long gb = b0 + row;
#pragma unroll
        for (int v = 0; v < 4; ++v) hts[(4 * quad + v) * LDH + row] = gb < B ? hv[k][v] : 0.f;
        if (gb < B) {
          float* gp = gates + (long)t * BG + gb * G + j0 + 4 * quad;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<f32x4*>(gp + q * H) = *reinterpret_cast<const f32x4*>(pre + row * LDP + q * PF_U + 4 * quad);
          *reinterpret_cast<f32x4*>(c_tm + (long)t * BH + gb * H + j0 + 4 * quad) =
              *reinterpret_cast<const f32x4*>(cst + row * CLD + 4 * quad);
        }
      }
    };
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && persist_arrive_ok(fault, t == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PF_STAMP(4);  // 4: hand-off stores + drain + arrival
    offchain();
    if (hT) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // 32 unit rows x 16 pieces of 4 batch columns
        const int p = tid + 256 * i, u = p >> 4, c = p & 15, gb = b0 + 4 * c;
        if (gb < Bp) {
          float* row = hT + (long)(j0 + u) * ldhT;
          *reinterpret_cast<f32x4*>(row + (long)(t + 1) * Bp + gb) = *reinterpret_cast<const f32x4*>(hts + u * LDH + 4 * c);
          if (t == 0) *reinterpret_cast<f32x4*>(row + gb) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    PF_STAMP(5);  // 5: off-chain stores
  }
#ifdef SV_PF32_STAMP
  if (tid == 0 && blockIdx.x < SV_NSTAMP_WG / 2) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(status + SV_SYNC_STAMP) + blockIdx.x * SV_NSTAMP;
    for (int i = 0; i < 6; ++i) st[i] = ph[i];
  }
#endif
#undef PF_STAMP
}

// ============================================================================
// backward, half-step form: the two 32-row halves of a workgroup's row block run as two
// independent recurrence chains, each with its own arrival counter ((row block, half) pair).  A
// workgroup does half 0's step t, then half 1's: while it runs half 1's k-loop, half 0's hand-off
// reaches the other workgroups, so one chain's epilogue + hand-off latency hides behind the other
// chain's MFMAs (c2: 4.89 -> 4.79 ms per layer; the same form of the forward measured slower,
// 4.33 -> 4.46 ms, so the forward keeps the 64-row tile).  Its smaller tiles leave LDS for 24
// weight k-groups, so the A fragments (the half's dG_{t+1}, from the fragment-order hand-off) can
// run 12 k-groups ahead.  Each half's k-group products are summed in two accumulators (c even /
// odd), added at the end; per half the partials meet in LDS and are summed in gate order.
// ============================================================================
constexpr int PH_BM = 32;                      // rows of a half

// the helper (prefetch) workgroups of the backward: step s's operands (activations, c_{s-1}, dh_up)
// of the XCD group's tiles, half a step ahead of the compute waves' own LDS-DMA of them (below)
__device__ void pf32_bwd_prefetch(const float* acts, const float* c_tm, const float* dhup, int up_full, int T, int B,
                                  int H, const unsigned* cnt, int nub, int ncomp, int npf, const unsigned* status,
                                  unsigned limit, char* scratch) {
  const int tid = threadIdx.x, g = tid >> 6;
  const int p = blockIdx.x - ncomp, x = blockIdx.x & 7, k = p >> 3, nk = npf >> 3;
  int l0, l1;
  persist_xcd_tiles(x, ncomp, l0, l1);
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  char* dst = scratch + g * 1024;
  int* skip = reinterpret_cast<int*>(scratch + 4096);
  // The compute workgroups DMA half 0's operands of step s at the end of half 1 of step s + 1 and
  // half 1's at the end of half 0 of step s (load_ew).  Each half's 32 rows are prefetched half a
  // step before that: half 0's once the group's first row block has finished half 0 of step s + 1,
  // half 1's once it has finished half 1 of step s + 1 -- so about one half-step of operands per
  // XCD is in flight in L2 (r05: the whole-step trigger two steps ahead held 1-1.5 steps, and part
  // of it was evicted before its DMA and fetched twice).
  const unsigned* ch[2] = {cnt + ((l0 / nub) * 2 + 0) * SV_PCNT_STRIDE, cnt + ((l0 / nub) * 2 + 1) * SV_PCNT_STRIDE};
  for (int s = T - 1; s >= 0; --s) {
    for (int hf = 0; hf < 2; ++hf) {
      if (tid == 0) {
        if (s + 1 <= T - 1) {  // trigger: half hf of step s + 1 done (T - 1 - s steps counted)
          unsigned spins = 0;
          const unsigned target = (unsigned)nub * (unsigned)(T - 1 - s);
          while (__hip_atomic_load(ch[hf], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target &&
                 !__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) && ++spins < limit)
            __builtin_amdgcn_s_sleep(8);
        }
        // too late (the compute waves have issued their own DMA of these operands): half 0's once
        // half 1 of step s + 1 is done, half 1's once half 0 of step s is done -- skip, so a slow
        // helper never holds the launch open
        *skip = hf == 0 ? __hip_atomic_load(ch[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)nub * (unsigned)(T - 1 - s)
                        : __hip_atomic_load(ch[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)nub * (unsigned)(T - s);
      }
      __syncthreads();
      const bool sk = *skip;
      __syncthreads();
      if (sk) continue;
      const float* up = dhup ? (up_full ? dhup + (long)s * BH : (s == T - 1 ? dhup : nullptr)) : nullptr;
      // a tile half's pieces: 32 rows x (4 gates of activations + c_{s-1} + dh_up) x 8 pieces of 16 B
      for (int L = l0 + k; L < l1; L += nk) {
        const int ub = L % nub, rb = L / nub, j0 = ub * PF_U;
        for (int i = tid; i < 6 * PH_BM * 8; i += 256) {
          const int kind = i >> 8, r2 = min(rb * PF_BM + hf * PH_BM + ((i >> 3) & 31), B - 1), pc = i & 7;
          const float* src = nullptr;
          if (kind < 4)
            src = acts + (long)s * BG + (long)r2 * G + (long)kind * H + j0 + 4 * pc;
          else if (kind == 4 && s > 0)
            src = c_tm + (long)(s - 1) * BH + (long)r2 * H + j0 + 4 * pc;
          else if (kind == 5 && up)
            src = up + (long)r2 * H + j0 + 4 * pc;
          if (src) persist_prefetch16(src, dst);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

template <int NKG, int P, int NV, int NL>
__global__ __launch_bounds__(256, 1) void lstm_persist_bwd_f32_h2_kernel(
    const float* __restrict__ whhT, const float* __restrict__ acts, const float* __restrict__ c_tm,
    const float* __restrict__ dhup, int up_full, float* __restrict__ dg, float* __restrict__ dgT, long lddgT,
    float* dgf, int T, int Bp, int B, unsigned* cnt, int nub, int xcd, unsigned* status, unsigned limit, int fault,
    float* __restrict__ dbp, int ncomp, int npf) {
  constexpr int H = 8 * NKG;
  static_assert(PF_NA + NV + NL == NKG, "weight split");
  constexpr int LDR = PF_U + 4;      // red [4][32][LDR]
  constexpr int LDG = 4 * PF_U + 4;  // dgs [32][LDG] (over ea + ec)
  constexpr int LDT = PH_BM + 4;     // gts [128][LDT] (over red)
  constexpr int FBLK = NKG * 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // operand image: [32][128] activations of the half-step, [32][32] c_{t-1}, [32][32] dh_up (issuing
  // the next half-step's into a second image during this one's k-loop measured slower: DESIGN §4)
  constexpr int ESET = PH_BM * 6 * PF_U;       // floats per image
  float* red = reinterpret_cast<float*>(smem) + ESET;  // [4][32][LDR]
  float* gts = red;
  char* wl = reinterpret_cast<char*>(red + 4 * PH_BM * LDR);
  float* const eimg = reinterpret_cast<float*>(smem);
  if ((int)blockIdx.x >= ncomp) {  // a helper workgroup: operand prefetch only
    pf32_bwd_prefetch(acts, c_tm, dhup, up_full, T, B, 8 * NKG, cnt, nub, ncomp, npf, status, limit, smem);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb, ncomp);
  const int j0 = ub * PF_U;
  const int nrb = ncomp / nub;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  const long FS = (long)nrb * 4 * 2 * FBLK;
  float wa[4 * PF_NA], wv[4 * NV];
  {
    const float* wr = whhT + (long)(j0 + r) * G + (long)g * H + 4 * hh;
    pf_load_w<NV, NL>(wr, 8, wa, wv, wl + (g * NL * 64 + lane) * 16);
  }
  auto wfrag = [&](int kg) -> f32x4 {
    if (kg < PF_NA) {
      const int b = 4 * (kg < PF_NA ? kg : 0);
      return f32x4{wa[b], wa[b + 1], wa[b + 2], wa[b + 3]};
    }
    if (kg < PF_NA + NV) {
      const int b = 4 * (kg < PF_NA + NV && kg >= PF_NA ? kg - PF_NA : 0);
      return f32x4{wv[b], wv[b + 1], wv[b + 2], wv[b + 3]};
    }
    return *reinterpret_cast<const f32x4*>(wl + ((g * NL + (kg - PF_NA - NV)) * 64 + lane) * 16);
  };
  const int quad = tid & 7, erow = tid >> 3;
  // half-step (tt, hf)'s operands -> LDS: wave g: 4 activation pieces (rows 8 g ..), 1 of c_{t-1}, 1
  // of dh_up; absent operands written as zeros into the same slots
  // the dG^T buffer fits one 32-bit buffer descriptor with room for the dropped-store offset
  const bool dgt_fits = dgT && (long)4 * H * lddgT * 4 < (1L << 32) - 64;
  auto load_ew = [&](int tt, int hf) {
    float* ea = eimg;
    float* ec = ea + PH_BM * 4 * PF_U;
    float* eu = ec + PH_BM * PF_U;
    // (the forward's dma_chunk form: buffer loads, scalar bases, 32-bit per-lane offsets)
    int gs = __builtin_amdgcn_readfirstlane(g);
    asm volatile("" : "+s"(gs));
    const int b0 = rb * PF_BM + hf * PH_BM;
    const __amdgpu_buffer_rsrc_t ra_ = sv_rsrc(acts + (long)tt * BG, (unsigned)(BG * 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 2 * (4 * gs + j) + (lane >> 5), s = lane & 31;
      const unsigned vo =
          (__umul24((unsigned)min(b0 + row, B - 1), (unsigned)G) + (unsigned)((s >> 3) * H + j0 + 4 * (s & 7))) * 4u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (pf_lds_t)(ea + (4 * gs + j) * 256), 16, vo, 0, 0, 0);
    }
    const float* up = dhup ? (up_full ? dhup + (long)tt * BH : (tt == T - 1 ? dhup : nullptr)) : nullptr;
    const int q = g * 64 + lane, row = 8 * gs + (lane >> 3), c = lane & 7;
    const unsigned vo2 = (__umul24((unsigned)min(b0 + row, B - 1), (unsigned)H) + (unsigned)(j0 + 4 * c)) * 4u;
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    if (tt > 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(sv_rsrc(c_tm + (long)(tt - 1) * BH, (unsigned)(BH * 4)),
                                               (pf_lds_t)(ec + gs * 256), 16, vo2, 0, 0, 0);
    else
      *reinterpret_cast<f32x4*>(ec + 4 * q) = zero;
    if (up)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(sv_rsrc(up, (unsigned)(BH * 4)), (pf_lds_t)(eu + gs * 256), 16, vo2, 0,
                                               0, 0);
    else
      *reinterpret_cast<f32x4*>(eu + 4 * q) = zero;
  };
  f32x4 cv[2], dcf[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int gb = min(rb * PF_BM + hf * PH_BM + erow, B - 1);
    cv[hf] = *reinterpret_cast<const f32x4*>(c_tm + (long)(T - 1) * BH + (long)gb * H + j0 + 4 * quad);
    dcf[hf] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  load_ew(T - 1, 0);
  // threads < 128: bias-gradient partial of gate column tid over t and the row block, accumulated in
  // fp64 (320 fp32 half-step sums of a cancelling sum: in fp32 the c2 bias gradients were 8e-6 off)
  double dbs = 0.0;
#ifdef SV_PF32_STAMP  // A/B stamp builds only: wave 0's cycles per phase, summed over the half-steps of t < T-1
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tl = 0;
  auto stamp = [&](int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (i >= 0) ph[i] += n - tl;
    tl = n;
  };
#define PB_STAMP(i) if (t < T - 1) stamp(i)
#else
#define PB_STAMP(i)
#endif
  for (int t = T - 1; t >= 0; --t) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int b0 = rb * PF_BM + hf * PH_BM;
      unsigned* my_cnt = cnt + (rb * 2 + hf) * SV_PCNT_STRIDE;
      f32x16 acc0, acc1;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
      PB_STAMP(-1);
      if (t < T - 1) {
        if (tid == 0) {
          persist_wait(my_cnt, (unsigned)nub * (unsigned)(T - 1 - t), status, limit, 2u);
        }
        __syncthreads();
        PB_STAMP(0);  // 0: hand-off wait
#ifndef SV_PF32_STAMP
        // a scalar-memory op here keeps hipcc's wait for the first A fragment counted (vmcnt(P - 1));
        // without one it emitted vmcnt(0) before half 0's first MFMA, so every half-step waited for
        // all P fragments before its k-loop started (+0.35 ms per c2 step; the stamp builds, whose
        // s_memtime sits here, never had it)
        {
          const unsigned long long t_ = __builtin_amdgcn_s_memtime();
          asm volatile("" ::"s"(t_));
        }
#endif
        const __amdgpu_buffer_rsrc_t ra = sv_rsrc(dgf + (long)(t + 1) * FS, (unsigned)(FS * 4));
        const unsigned base = ((unsigned)(((rb * 4 + g) * 2 + hf) * FBLK) + (unsigned)lane * 4u) * 4u;
        u32x4_t fa[P];
#pragma unroll
        for (int p = 0; p < P; ++p) fa[p] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + 1024u * p, 0, 16 /* sc1 */);
        f32x4 w = wfrag(0);
        __builtin_amdgcn_sched_barrier(0);
        auto kstep = [&](int kg) {
          const f32x4 a = __builtin_bit_cast(f32x4, fa[kg % P]);
          const f32x4 nw = kg + 1 < NKG ? wfrag(kg + 1) : w;
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], w[0], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1], w[1], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2], w[2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[3], w[3], acc1, 0, 0, 0);
          if (kg + P < NKG) fa[kg % P] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + 1024u * (kg + P), 0, 16);
          w = nw;
          __builtin_amdgcn_sched_barrier(0);
        };
#pragma unroll
        for (int kg = 0; kg < NKG; ++kg) kstep(kg);
      }
      PB_STAMP(1);  // 1: k-loop (A fragments from the hand-off + MFMAs)
      float* ea = eimg;
      float* ec = ea + PH_BM * 4 * PF_U;
      float* eu = ec + PH_BM * PF_U;
      float* dgs = ea;
#pragma unroll
      for (int i = 0; i < 16; ++i) red[(g * PH_BM + acc_row(i, lane)) * LDR + r] = acc0[i] + acc1[i];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's operand DMA landed
      __syncthreads();
      PB_STAMP(2);  // 2: partial exchange + operand DMA wait
      f32x4 dh, cpv, a4[4];
      dh = *reinterpret_cast<const f32x4*>(red + (0 * PH_BM + erow) * LDR + 4 * quad);
      dh += *reinterpret_cast<const f32x4*>(red + (1 * PH_BM + erow) * LDR + 4 * quad);
      dh += *reinterpret_cast<const f32x4*>(red + (2 * PH_BM + erow) * LDR + 4 * quad);
      dh += *reinterpret_cast<const f32x4*>(red + (3 * PH_BM + erow) * LDR + 4 * quad);
      dh += *reinterpret_cast<const f32x4*>(eu + erow * PF_U + 4 * quad);
      cpv = *reinterpret_cast<const f32x4*>(ec + erow * PF_U + 4 * quad);
#pragma unroll
      for (int q = 0; q < 4; ++q) a4[q] = *reinterpret_cast<const f32x4*>(ea + erow * (4 * PF_U) + q * PF_U + 4 * quad);
      __syncthreads();  // the images and red are free: the dG tiles take their place
      f32x4 dq[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {  // the per-step kernel's cell backward (lstm_step_bwd_v2_kernel)
        const float d = dh[v];
        const float i_ = a4[0][v], f_ = a4[1][v], g_ = a4[2][v], o_ = a4[3][v];
        const float tc = sv_tanh(cv[hf][v]);
        const float dc = d * o_ * (1.f - tc * tc) + dcf[hf][v];
        dq[0][v] = dc * g_ * i_ * (1.f - i_);
        dq[1][v] = dc * cpv[v] * f_ * (1.f - f_);
        dq[2][v] = dc * i_ * (1.f - g_ * g_);
        dq[3][v] = d * tc * o_ * (1.f - o_);
        dcf[hf][v] = dc * f_;
      }
      cv[hf] = cpv;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *reinterpret_cast<f32x4*>(dgs + erow * LDG + q * PF_U + 4 * quad) = dq[q];
#pragma unroll
        for (int v = 0; v < 4; ++v) gts[(q * PF_U + 4 * quad + v) * LDT + erow] = dq[q][v];
      }
      __syncthreads();
      PB_STAMP(3);  // 3: cell + dG tiles into LDS
      // off-chain pieces of the half-step (the bias partials of gate column tid over this half's rows
      // in order, rows past B excluded; dG^T of the half-step).  The row bounds through an opaque
      // copy made here, so their predicates are formed here each half-step: hoisted out of the step
      // loop they were held across the k-loops in SGPRs and spilled to VGPR lanes
      int Bq = B, Bpq = Bp;
      asm volatile("" : "+s"(Bq), "+s"(Bpq));
      auto bias_part = [&]() {
        if (dbp && tid < 4 * PF_U) {
          // rows in order either way; the partial row block's runtime bound in its own branch (32
          // per-row predicates of both halves, hoisted out of the step loop, were 128 SGPRs spilled
          // to VGPR lanes and read back every step)
          const int nv = Bq - b0;
          float s = 0.f;
          if (nv >= PH_BM) {
#pragma unroll
            for (int e4 = 0; e4 < PH_BM / 4; ++e4) {
              const f32x4 v = *reinterpret_cast<const f32x4*>(gts + tid * LDT + 4 * e4);
#pragma unroll
              for (int e = 0; e < 4; ++e) s += v[e];
            }
          } else {
            for (int e = 0; e < nv; ++e) s += gts[tid * LDT + e];
          }
          dbs += s;
        }
      };
      // dG^T stores, 4 per thread (128 gate-unit rows x 8 pieces of 4 batch columns); `exact`: every
      // thread issues all 4 (pieces past Bp to an offset past the descriptor's range, dropped), so a
      // counted wait can name them
      auto dgt_stores = [&](bool exact) {
        // sc1 stores: written through and dropped from this XCD's L2 (MI355X_MICROARCH.md, stores of
        // each flavour), so the 48 KB per tile per step the dW GEMMs read back much later do not
        // evict the lines the helper workgroups prefetched
        const __amdgpu_buffer_rsrc_t rdt = sv_rsrc(dgT, (unsigned)((long)4 * H * lddgT * 4));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = tid + 256 * i, gu = p >> 3, c = p & 7, gbc = b0 + 4 * c;
          if (exact || gbc < Bpq) {
            f32x4 v = *reinterpret_cast<const f32x4*>(gts + gu * LDT + 4 * c);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (gbc + e >= Bq) v[e] = 0.f;
            const long eo = ((long)(gu >> 5) * H + j0 + (gu & 31)) * lddgT + (long)t * Bp + gbc;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rdt,
                                                   gbc < Bpq ? (unsigned)(eo * 4) : 0xFFFFFFF0u, 0, 16 /* sc1 */);
          }
        }
      };
      // the hand-off: 16 fragment blocks of 1 KB (gate q, this half, k-group 4 ub + kl); slot 0 (no
      // consumer step) only when the dx GEMM reads the fragment-order image (dg == nullptr)
      // with an arrival to make and dG^T written through one descriptor, the bias
      // partials and the dG^T stores go out behind the hand-off stores, before their drain, and the
      // drain counts them (vmcnt(4): this wave's hand-off stores, older, are done; a raw barrier, as
      // __syncthreads' release fence would drain the dG^T stores too)
      const bool ovl = t > 0 && !dg && dgt_fits;
      if (t > 0 || !dg) {
        const __amdgpu_buffer_rsrc_t rw = sv_rsrc(dgf + (long)t * FS, (unsigned)(FS * 4));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = tid + 256 * i, blk = p >> 6, L = p & 63;
          const int q = blk >> 2, kl = blk & 3;
          const f32x4 v = *reinterpret_cast<const f32x4*>(dgs + (L & 31) * LDG + q * PF_U + 8 * kl + 4 * (L >> 5));
          const unsigned off =
              ((unsigned)(((rb * 4 + q) * 2 + hf) * FBLK) + (unsigned)(4 * ub + kl) * 256u + (unsigned)L * 4u) * 4u;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rw, off, 0, 16 /* sc1 */);
        }
        if (ovl) {
          asm volatile("" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);  // (the dG^T stores stay younger than the hand-off's)
          bias_part();
          dgt_stores(true);
          asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          if (tid == 0 && persist_arrive_ok(fault, t == T - 1))
            __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (t > 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          if (tid == 0 && persist_arrive_ok(fault, t == T - 1))
            __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      PB_STAMP(4);  // 4: hand-off stores + drain + arrival
      if (!ovl) bias_part();
      const long gb = b0 + erow;
      if (dg && gb < Bq) {  // (dg == nullptr: the dx GEMM reads the fragment-order hand-off instead)
        float* dp = dg + (long)t * BG + gb * G + j0 + 4 * quad;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<f32x4*>(dp + q * H) = *reinterpret_cast<const f32x4*>(dgs + erow * LDG + q * PF_U + 4 * quad);
      }
      if (!ovl) dgt_stores(false);
      if (hf == 0 || t > 0) {
        __syncthreads();  // dgs / gts read by every wave before the next half-step's operands land
        if (hf == 0)
          load_ew(t, 1);
        else
          load_ew(t - 1, 0);
      }
      PB_STAMP(5);  // 5: off-chain (bias partials, dG / dG^T stores, next operand DMA issue)
    }
  }
  if (dbp && tid < 4 * PF_U) dbp[(long)rb * 4 * H + (long)(tid >> 5) * H + j0 + (tid & 31)] = (float)dbs;
#ifdef SV_PF32_STAMP
#ifdef SV_PF32_WAVE_STAMP  // every wave's phases, workgroups 0-127: slot 512 + 4 wg + wave
  if (lane == 0 && blockIdx.x < SV_NSTAMP_WG / 8) {
    unsigned long long* st = reinterpret_cast<unsigned long long*>(status + SV_SYNC_STAMP) +
                             (SV_NSTAMP_WG / 2 + 4 * blockIdx.x + g) * SV_NSTAMP;
    for (int i = 0; i < 6; ++i) st[i] = ph[i];
  }
#else
  if (tid == 0 && blockIdx.x < SV_NSTAMP_WG / 2) {  // second half of the stamp slots (the forward uses the first)
    unsigned long long* st =
        reinterpret_cast<unsigned long long*>(status + SV_SYNC_STAMP) + (SV_NSTAMP_WG / 2 + blockIdx.x) * SV_NSTAMP;
    for (int i = 0; i < 6; ++i) st[i] = ph[i];
  }
#endif
#endif
#undef PB_STAMP
}

// ============================================================================
// host side
// ============================================================================
namespace {
// weight k-groups (of 96 at H = 768) in VGPRs / LDS beside the 64 in AGPRs
// (measured: 20 / 24 forward k-groups in VGPRs and backward prefetch depths 8 / 16 no faster)
constexpr int PF_FWD_NV = 16, PF_FWD_NL = 32 - PF_FWD_NV, PH_BWD_NL = 24, PH_BWD_NV = 96 - PF_NA - PH_BWD_NL,
              PH_BWD_P = 12;
constexpr size_t pf_fwd_lds() {
  return (size_t)PF_NB * PF_CH + (size_t)PF_BM * 4 * PF_U * 4 + (size_t)4 * PF_FWD_NL * 1024;
}
constexpr size_t ph_bwd_lds() {
  return ((size_t)PH_BM * 4 * PF_U * 4 + 2 * (size_t)PH_BM * PF_U * 4) +
         (size_t)4 * PH_BM * (PF_U + 4) * 4 + (size_t)4 * PH_BWD_NL * 1024;
}
static_assert(pf_fwd_lds() <= 160 * 1024 && ph_bwd_lds() <= 160 * 1024, "LDS");
static_assert((size_t)4 * PF_U * (PH_BM + 4) <= (size_t)4 * PH_BM * (PF_U + 4), "gts fits in red");
static_assert((size_t)PH_BM * (4 * PF_U + 4) <= (size_t)PH_BM * 5 * PF_U, "dgs fits in ea + ec");
}  // namespace

// the fp32 persistent recurrences fit: H = 768, (H / 32) x ceil(B / 64) workgroups co-resident
int sv_persist_f32_fits(int B, int H, int cus) {
  const long nrb = (B + PF_BM - 1) / PF_BM;  // (two counters per row block: one per half)
  return H == 768 && B > 0 && 2 * nrb <= SV_PCNT_ROWS && (H / PF_U) * nrb <= cus && (long)B * 4 * H * 4 < (1L << 31);
}

// bytes of the backward's fragment-order hand-off: T slots of ceil(B / 64) x 64 rows x 4H fp32
size_t sv_persist_f32_bwd_scratch(int T, int B, int H) {  // hand-off slots + bias partials
  const size_t nrb = (size_t)((B + PF_BM - 1) / PF_BM);
  return ((size_t)T * nrb * PF_BM + nrb) * 4 * H * sizeof(float);
}

int sv_persist_fwd_f32(int T, int B, int H, const float* whh, float* gates, float* c_tm, float* h_tm, float* hT,
                       hipStream_t stream, unsigned* sync, int chan, hipEvent_t pre, hipEvent_t post,
                       const float* x_tm, int F, const float* wih, const float* b_ih, const float* b_hh) {
  if (!sv_persist_f32_fits(B, H, sv_stream_cus(stream))) return SV_ESHAPE;
  if (!sync || chan < 0 || chan >= SV_SYNC_CHANNELS || !whh || !gates || !c_tm || !h_tm) return SV_EARG;
  unsigned* cnt = sync + SV_SYNC_CNT + (size_t)chan * SV_PCNT_ROWS * SV_PCNT_STRIDE;
  const int nub = H / PF_U, nrb = (B + PF_BM - 1) / PF_BM;
  const int Bp = (B + 3) & ~3;
  hipError_t e = (hipError_t)sv_zero_counters(cnt, 1, 0, nrb * SV_PCNT_STRIDE, stream);
  if (e != hipSuccess) return (int)e;
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;
  if (x_tm) {  // layer 0: the input projection inside the recurrence (F = 40 only)
    if (F != 40 || !wih) return SV_EARG;
    hipLaunchKernelGGL((lstm_persist_fwd_f32_kernel<96, PF_FWD_NV, PF_FWD_NL, 5>), dim3(nub * nrb), dim3(256),
                       pf_fwd_lds(), stream, whh, gates, c_tm, h_tm, hT, (long)(T + 1) * Bp, T, Bp, B, cnt, nub,
                       PF_XCD, sync, sv_persist_limit(), sv_persist_fault(0), x_tm, wih, b_ih, b_hh);
  } else {
    hipLaunchKernelGGL((lstm_persist_fwd_f32_kernel<96, PF_FWD_NV, PF_FWD_NL>), dim3(nub * nrb), dim3(256),
                       pf_fwd_lds(), stream, whh, gates, c_tm, h_tm, hT, (long)(T + 1) * Bp, T, Bp, B, cnt, nub,
                       PF_XCD, sync, sv_persist_limit(), sv_persist_fault(0), nullptr, nullptr, nullptr, nullptr);
  }
  SV_LAUNCH_CHECK();
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  return SV_OK;
}

int sv_persist_bwd_f32(int T, int B, int H, const float* whhT, const float* acts, const float* c_tm,
                       const float* dhup, int up_full, float* dg, float* dgT, float* dgf, hipStream_t stream,
                       unsigned* sync, hipEvent_t pre, hipEvent_t post, float* db_ih, float* db_hh) {
  if (!sv_persist_f32_fits(B, H, sv_stream_cus(stream))) return SV_ESHAPE;
  // dg may be null: the row-major dG is then not written and slot 0 of dgf holds dG_0 as well
  if (!sync || !whhT || !acts || !c_tm || !dgT || !dgf || ((uintptr_t)dgf & 15)) return SV_EARG;
  unsigned* cnt = sync + SV_SYNC_CNT;  // channel 0
  const int nub = H / PF_U, nrb = (B + PF_BM - 1) / PF_BM;
  const int Bp = (B + 3) & ~3;
  // bias partials [nrb][4H] after the hand-off slots (db_ih NULL: not computed here)
  float* dbp = db_ih ? dgf + (size_t)T * nrb * PF_BM * 4 * H : nullptr;
  hipError_t e = (hipError_t)sv_zero_counters(cnt, 1, 0, 2 * nrb * SV_PCNT_STRIDE, stream);
  if (e != hipSuccess) return (int)e;
  if (pre && (e = hipEventRecord(pre, stream)) != hipSuccess) return (int)e;
  // helper workgroups on the CUs the grid leaves free, the same number per XCD (c2: 16)
  const int ncomp = nub * nrb, npf = std::min(16, (sv_stream_cus(stream) - ncomp) / 8 * 8);
  hipLaunchKernelGGL((lstm_persist_bwd_f32_h2_kernel<96, PH_BWD_P, PH_BWD_NV, PH_BWD_NL>), dim3(ncomp + npf),
                     dim3(256), ph_bwd_lds(), stream, whhT, acts, c_tm, dhup, up_full, dg, dgT, (long)T * Bp, dgf, T,
                     Bp, B, cnt, nub, PF_XCD, sync, sv_persist_limit(), sv_persist_fault(1), dbp, ncomp, npf);
  SV_LAUNCH_CHECK();
  if (post && (e = hipEventRecord(post, stream)) != hipSuccess) return (int)e;
  // bias gradients: the row blocks' partials summed in order (no row-sum pass over dG^T)
  return dbp ? sv_persist_db_finalize(dbp, nrb, 4 * H, db_ih, db_hh, stream) : SV_OK;
}
