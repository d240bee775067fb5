// Wide-tile persistent backward recurrence (see the kernel comment).  Its own translation unit:
// built with -mllvm -amdgpu-mfma-vgpr-form=1 (Makefile) so the two accumulators are VGPRs and
// all 256 AGPRs hold W_hh fragments.
#include "sv_persist_dev.h"
#include "../../include/sv_ge2e.h"

// ============================================================================
// Wide-tile W-stationary backward (H = 768, default; SV_PBWD3=0 keeps the 32-unit tile above).
// Tile: 32 batch rows x 64 hidden units, so the grid is (H / 64) x (B / 32) -- 240 workgroups at
// c3 as before -- but each workgroup streams HALF the hand-off bytes per step: wave g's A operand
// is 32 rows x H of dG_{t+1} (48 KB, one fragment per k-step) and every fragment feeds two MFMAs,
// one per 32-unit half of W_hh (2 x 48 B fragments = 384 registers: 256 AGPRs + 128 VGPRs).  The
// per-step operand stream of the 32-unit tile (393 KB per CU from the hand-off buffer, the
// kernel's dominant phase) becomes 196 KB.  Everything else is the 32-unit kernel's: the same
// per-gate k order and gate-order sum (bit-identical dG), fragment-order hand-off (row blocks of
// 32), operands staged by LDS-DMA after the arrival, bias partials per row block.
// ============================================================================
// NL: the last NL k-steps of the second W_hh half are read from LDS (staged once, 16 B per lane per
// fragment, prefetched two k-steps ahead) -- the registers cannot hold all 2 x NS fragments beside
// the step's working set
template <int NS, int P, int NL>
__global__ __launch_bounds__(256, 1) void lstm_persist3_bwd_bf16_kernel(
    const bf16_t* __restrict__ whhT, const bf16_t* __restrict__ acts, const float* __restrict__ c_tm,
    const float* __restrict__ dhup, int up_full, bf16_t* __restrict__ dg, bf16_t* __restrict__ dgT, long lddgT,
    bf16_t* dgf, int T, int Bp, int B, int H, unsigned* cnt, int nub, int xcd, unsigned* status, unsigned limit,
    int fault, int dbg, float* __restrict__ dbp, unsigned long long* __restrict__ stamps) {
  dbg &= SV_PDBG;
  constexpr int BM = 32, U = 64, KR = 2;  // rows, units, row passes of the epilogue (16 rows each)
  constexpr int LDR = U + 4;              // red [4][BM][LDR] fp32
  constexpr int LDG = 4 * U + 8;          // dgs [BM][LDG] bf16 (row-major dG tile)
  constexpr int LDT = BM + 8;             // gts [4U][LDT] bf16 (transposed dG tile)
  constexpr int FRAG = NS * 64 * 8;       // dgf elements of one (row block, gate)
  static_assert(P >= 1 && P <= NS, "prefetch depth");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);
  bf16_t* dgs = reinterpret_cast<bf16_t*>(smem + 4 * BM * LDR * 4);
  bf16_t* gts = dgs + BM * LDG;
  char* ewa = reinterpret_cast<char*>(gts + 4 * U * LDT);  // [BM][512 B]: gate q at ((q + row) & 3) * 128
  float* ewc = reinterpret_cast<float*>(ewa + BM * 512);    // [BM][U] c_{t-1}
  float* ewu = ewc + BM * U;                                // [BM][U] dh_up
  char* wl = reinterpret_cast<char*>(ewu + BM * U);         // [4 waves][NL][64 lanes][16 B]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * U, b0 = rb * BM;
  const int nrb = gridDim.x / nub;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  const long FS = (long)nrb * BM * G;
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  // W_hh fragments of gate g for units j0 + r (wa) and j0 + 32 + r (wb)
  constexpr int NR = NS - NL;  // second-half fragments kept in registers
  bf16x8_t wa[NS], wb[NR];
  {
    const bf16_t* ra = whhT + (long)(j0 + r) * G + (long)g * H + 8 * hh;
    const bf16_t* rbp = ra + 32 * G;
    const bool oka = j0 + r < H, okb = j0 + 32 + r < H;
    const bf16x8_t z = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) wa[s] = oka ? *reinterpret_cast<const bf16x8_t*>(ra + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NR; ++s) wb[s] = okb ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = NR; s < NS; ++s)
      *reinterpret_cast<bf16x8_t*>(wl + ((g * NL + s - NR) * 64 + lane) * 16) =
          okb ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+a"(wa[s]));
#pragma unroll
    for (int s = 0; s < 64 - NS; ++s) asm volatile("" : "+a"(wb[s]));  // the AGPRs left: 64 - NS fragments
  }
  auto wl_read = [&](int j) { return *reinterpret_cast<const bf16x8_t*>(wl + ((g * NL + j) * 64 + lane) * 16); };
  // elementwise map: thread -> 4 consecutive units (u4) x rows 2 brow, 2 brow + 1
  const int u4 = (tid & 15) * 4, brow = tid >> 4;
  float4 cv[KR];
  float dcf[KR][4];
  // bias-gradient partial sums of this thread's bf16 dG values over t and its two rows
  float dbs[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) dbs[q][v] = 0.f;
  const long Bv = B;
  // step tt's operands into LDS (buffer_load ... lds; rows past B and absent operands read zeros)
  // piece i (0..7) of step tt's operand DMA: 0-3 activations, 4-5 c_{t-1}, 6-7 dh_up
  auto ew_piece = [&](int tt, int i) {
    if (dbg & 512) tt = T - 1;  // (profiling only: every step reads step T-1's operands, cache-hot)
    if (i < 4) {
      const __amdgpu_buffer_rsrc_t ra_ = sv_rsrc(acts + (long)tt * BG, (unsigned)(BG * 2));
      const int p = (g * 4 + i) * 64 + lane, row = p >> 5, sl = p & 31;
      const int q = ((sl >> 3) - row) & 3, c = sl & 7;
      const long gb = b0 + row, gbv = gb < Bv ? gb : Bv + 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (lds_ptr_t)(ewa + (g * 4 + i) * 1024), 16,
                                               (unsigned)((gbv * G + q * H + j0 + 8 * c) * 2), 0, 0, 0);
    } else {
      const int j = i & 1;
      const int p = (g * 2 + j) * 64 + lane, row = p >> 4, c = p & 15;
      const long gb = b0 + row, gbv = gb < Bv ? gb : Bv + 64;
      const unsigned off = (unsigned)((gbv * H + j0 + 4 * c) * 4);
      if (i < 6) {
        const __amdgpu_buffer_rsrc_t rc_ =
            sv_rsrc(c_tm + (long)(tt > 0 ? tt - 1 : 0) * BH, tt > 0 ? (unsigned)(BH * 4) : 0u);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rc_, (lds_ptr_t)((char*)ewc + (g * 2 + j) * 1024), 16, off, 0, 0, 0);
      } else {
        const float* up = dhup ? (up_full ? dhup + (long)tt * BH : (tt == T - 1 ? dhup : nullptr)) : nullptr;
        const __amdgpu_buffer_rsrc_t ru_ = sv_rsrc(up ? up : c_tm, up ? (unsigned)(BH * 4) : 0u);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ru_, (lds_ptr_t)((char*)ewu + (g * 2 + j) * 1024), 16, off, 0, 0, 0);
      }
    }
  };
  auto load_ew = [&](int tt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) ew_piece(tt, i);
  };
  // store i (0..7) of step tt's dG tile from LDS: 0-3 row-major dG (when dg), 4-7 dG^T (when dgT)
  auto store_piece = [&](int tt, int i) {
    // buffer stores with 32-bit offsets (no 64-bit addresses kept live across the k-loop)
    if (i < 4) {
      if (!dg) return;
      const __amdgpu_buffer_rsrc_t rs = sv_rsrc(dg + (long)tt * BG, (unsigned)(BG * 2));
      const int q = tid + 256 * i, row = q >> 5, gq = (q >> 3) & 3, c = q & 7;
      const int gb = b0 + row, gj = j0 + 8 * c;
      const uint4 v = *reinterpret_cast<const uint4*>(dgs + row * LDG + gq * U + 8 * c);
      if (gb < B && gj < H)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rs,
                                               (unsigned)(((long)gb * G + (long)gq * H + gj) * 2), 0, 0);
    } else {
      if (!dgT) return;
      const __amdgpu_buffer_rsrc_t rs = sv_rsrc(dgT + (long)tt * Bp, (unsigned)(4L * H * lddgT * 2 - (long)tt * Bp * 2));
      const int q = tid + 256 * (i & 3), gu = q >> 2, c = q & 3;
      const int gq = gu / U, gj = j0 + gu % U, gb = b0 + 8 * c;
      const uint4 v = *reinterpret_cast<const uint4*>(gts + gu * LDT + 8 * (c ^ ((gu % U) >> 4 & 3)));
      if (i >= 8)  // (exact form, i = 8..11: always issued, an invalid piece to a dropped offset)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rs,
                                               gb < Bp && gj < H ? (unsigned)((((long)gq * H + gj) * lddgT + gb) * 2)
                                                                 : 0xFFFFFFF0u, 0, 0);
      else if (gb < Bp && gj < H)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rs,
                                               (unsigned)((((long)gq * H + gj) * lddgT + gb) * 2), 0, 0);
    }
  };
  {
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(c_tm + (long)(T - 1) * BH, (unsigned)(BH * 4));
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + 2 * brow + k;
      const u32x4_t x =
          __builtin_amdgcn_raw_buffer_load_b128(rc_, (unsigned)(((gb < Bv ? gb : Bv + 64) * H + j0 + u4) * 4), 0, 0);
      cv[k] = float4{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
#pragma unroll
      for (int v = 0; v < 4; ++v) dcf[k][v] = 0.f;
    }
  }
  load_ew(T - 1);
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
      // A fragments of dG_{t+1}: k-step s is the KB at (rb 4 + g) FRAG + s 512
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(dgf + (long)(t + 1) * FS, (unsigned)(FS * 2));
      constexpr unsigned kstep = 1024u;
      const unsigned base0 = ((unsigned)(rb * 4 + g) * (unsigned)FRAG + (unsigned)lane * 8u) * 2u;
      u32x4_t fa[P];
#pragma unroll
      for (int s = 0; s < P; ++s) fa[s] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * s, 0, 16 /* sc1 */);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8_t wq[2];  // LDS-resident fragments, two k-steps ahead
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8_t a = __builtin_bit_cast(bf16x8_t, fa[s % P]);
        acc0 = mfma_bf16(a, wa[s], acc0);
        acc1 = mfma_bf16(a, s < NR ? wb[s < NR ? s : 0] : wq[s & 1], acc1);
        if (s + 2 >= NR && s + 2 < NS) wq[s & 1] = wl_read(s + 2 - NR);  // k-step s + 2 (same parity)
        if (s + P < NS) fa[s % P] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * (s + P), 0, 16);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // per-gate partials -> red[g][row][unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      red[(g * BM + acc_row(i, lane)) * LDR + r] = acc0[i];
      red[(g * BM + acc_row(i, lane)) * LDR + 32 + r] = acc1[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's operand DMA landed
    __syncthreads();
    mark(1);
    {
      // thread: rows 2 brow and 2 brow + 1 (k = 0, 1) x units u4 .. u4 + 3; a unit's two rows land
      // in the transposed tile as one 4-B write (16 per thread instead of 32 2-B ones), at a chunk
      // swizzle that makes those writes conflict-free
      unsigned e0s[4][2] = {};  // row 2 brow's bf16 dG, (q, unit pair)
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        const int b = 2 * brow + k;
        const float4 r0 = *reinterpret_cast<const float4*>(red + (0 * BM + b) * LDR + u4);
        const float4 r1 = *reinterpret_cast<const float4*>(red + (1 * BM + b) * LDR + u4);
        const float4 r2 = *reinterpret_cast<const float4*>(red + (2 * BM + b) * LDR + u4);
        const float4 r3 = *reinterpret_cast<const float4*>(red + (3 * BM + b) * LDR + u4);
        const float4 cpv = *reinterpret_cast<const float4*>(ewc + b * U + u4);
        const float4 upv = *reinterpret_cast<const float4*>(ewu + b * U + u4);
        float4 f[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          f[q] = unpack_bf4(*reinterpret_cast<const uint2*>(ewa + b * 512 + ((q + b) & 3) * 128 + (u4 >> 3) * 16 +
                                                            (u4 & 7) * 2));
        unsigned pk[4][2];
        float4 dh4 = r0;  // (elementwise, the scalar order)
        dh4 += r1;
        dh4 += r2;
        dh4 += r3;
        dh4 += upv;
        float ddv[4][4];
        lstm_cell_bwd_x4(dh4, f[0], f[1], f[2], f[3], cv[k], cpv, dcf[k], ddv);
        pack_dg4(ddv, pk, dbs);
        const int sw = (2 * brow) ^ (((u4 >> 4) & 3) << 3);  // (the same for the 4 units)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            if (k == 0) {
              e0s[q][p] = pk[q][p];
            } else {
              const int u = u4 + 2 * p;
              *reinterpret_cast<unsigned*>(gts + (q * U + u) * LDT + sw) = (e0s[q][p] & 0xffffu) | (pk[q][p] << 16);
              *reinterpret_cast<unsigned*>(gts + (q * U + u + 1) * LDT + sw) = (e0s[q][p] >> 16) | (pk[q][p] & 0xffff0000u);
            }
          }
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(dgs + b * LDG + q * U + u4) = uint2{pk[q][0], pk[q][1]};
        cv[k] = cpv;  // c_{t-1} is the next step's c_t
      }
    }
    __syncthreads();
    mark(2);
    // the hand-off: 16 KB of dG_t per workgroup in fragment order (gate, k-step), 16-B sc1 stores
    if (!(dbg & 8)) {
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(dgf + (long)t * FS, (unsigned)(FS * 2));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = tid + 256 * i, c = p >> 6, l = p & 63;
        const int gq = c >> 2, sl = c & 3;
        const uint4 v = *reinterpret_cast<const uint4*>(dgs + (l & 31) * LDG + gq * U + 16 * sl + 8 * (l >> 5));
        const unsigned off =
            ((unsigned)(rb * 4 + gq) * (unsigned)FRAG + (unsigned)(j0 / 16 + sl) * 512u + (unsigned)l * 8u) * 2u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw, off, 0, 16 /* sc1 */);
      }
    }
    // with the dx GEMM on the hand-off (no row-major dG), the step's 4 dG^T stores per
    // thread go out behind the hand-off stores, before their drain, which counts them (vmcnt(4):
    // this wave's older hand-off stores done; a raw barrier: __syncthreads' fence would drain them)
    const bool ovl = !dbg && !dg && dgT;
    if (ovl) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // (the dG^T stores stay younger than the hand-off's)
#pragma unroll
      for (int i = 8; i < 12; ++i) store_piece(t, i);
      asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (tid == 0 && persist_arrive_ok(fault, t == T - 1))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mark(3);
    {
      // (dbg, profiling only: 64 skips the operand DMA, 128 the dG / dG^T stores).  The stores
      // first: their LDS reads issued behind an LDS-DMA would wait for it to land (the compiler
      // cannot tell the DMA's LDS range from the tiles', so it puts vmcnt(0) before every read)
      if (!ovl && !(dbg & 8) && !(dbg & 128))
#pragma unroll
        for (int i = 0; i < 8; ++i) store_piece(t, i);
      if (t > 0 && !(dbg & 64)) load_ew(t - 1);
    }
    mark(4);
  }
  if (stamp && tid == 0 && blockIdx.x < SV_NSTAMP_WG)
    for (int i = 0; i < 5; ++i) stamps[blockIdx.x * SV_NSTAMP + i] = ph[i];
  if (dbp) {
    __syncthreads();
    float* dsum = red;  // [16][4U] fp32: row pairs (2 brow, 2 brow + 1)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(dsum + brow * (4 * U) + q * U + u4) = float4{dbs[q][0], dbs[q][1], dbs[q][2], dbs[q][3]};
    __syncthreads();
    {
      const int q = tid / U, gj = j0 + tid % U;
      float sum = 0.f;
      for (int b = 0; b < 16; ++b) sum += dsum[b * (4 * U) + tid];
      if (gj < H) dbp[(long)rb * G + (long)q * H + gj] = sum;
    }
  }
}

int sv_persist3_bwd_launch(dim3 grid, int nub, hipStream_t stream, const bf16_t* whhT, const bf16_t* acts,
                           const float* c_tm, const float* dhup, int up_full, bf16_t* dg, bf16_t* dgT, long lddgT,
                           bf16_t* dgf, int T, int Bp, int B, int H, unsigned* cnt, int xcd, unsigned* sync,
                           unsigned limit, int fault, int dbg, float* dbp) {
  constexpr int NL = 12;
  constexpr size_t lds = (size_t)4 * 32 * 68 * 4 + (size_t)32 * 264 * 2 + (size_t)256 * 40 * 2 + (size_t)32 * 512 +
                         (size_t)2 * 32 * 64 * 4 + (size_t)4 * NL * 1024;
  unsigned long long* stamps = reinterpret_cast<unsigned long long*>(sync + SV_SYNC_STAMP);
  // (the operand DMA and the dG / dG^T stores deferred into the next step's k-loop measured slower
  // -- c3 bwd 1205 vs 1086 us per layer: the fragment waits count the older stores -- and deleted)
  // (operand-prefetch helper workgroups on the 16 free CUs, as the fp32 backward has them, measured
  // no gain here: DESIGN §4)
  hipLaunchKernelGGL((lstm_persist3_bwd_bf16_kernel<48, 8, NL>), grid, dim3(256), lds, stream, whhT, acts, c_tm,
                     dhup, up_full, dg, dgT, lddgT, dgf, T, Bp, B, H, cnt, nub, xcd, sync, limit, fault, dbg, dbp,
                     stamps);
  return (int)hipGetLastError();
}

// ============================================================================
// Wide-tile W-stationary forward (H = 768, layers without the fused input projection; the same
// conditions as the wide backward).  Tile: 32 batch rows x 64 hidden units x 4 gates; wave g
// holds gate g's W_hh rows for the 64 units (two halves of 48 MFMA B fragments: 256 AGPRs +
// VGPRs + NL LDS-resident fragments) for the whole sequence.  Per step only h_{t-1} of the 32
// rows (48 KB, half the 64 x 32 tile's staging) is staged into LDS with sc1 loads, and every A
// fragment read from LDS feeds two MFMAs.  Same per-gate k order, cell helper and hand-off as
// lstm_persist2_fwd_bf16_kernel (bit-identical outputs).
// ============================================================================
// XF > 0 (layer 0, F = 8 XF <= 48 features): the input projection formed in the kernel from x_bf
// [T,B,F] and W_ih [4H,F] (both halves' fragments in registers), rounded to bf16 with its biases as
// the K1 path stores it -- lstm_persist2_fwd_bf16_kernel's fused form.
// h_{t-1} is staged through registers in two halves (measured against LDS-DMA staging and the
// second half in flight during the first half's MFMAs: both slower, sv_persist3_fwd_launch)
template <int NS, int NL, int PA, int XF>
__global__ __launch_bounds__(256, 1) void lstm_persist3_fwd_bf16_kernel(
    const bf16_t* __restrict__ whh_bf, bf16_t* __restrict__ gates, float* __restrict__ c_tm, float* __restrict__ h_tm,
    bf16_t* h_bf, bf16_t* __restrict__ hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt, int nub, int xcd,
    unsigned* status, unsigned limit, int fault, const bf16_t* __restrict__ x_bf, const bf16_t* __restrict__ wih_bf,
    const float* __restrict__ b_ih, const float* __restrict__ b_hh, int dbg) {
  dbg &= SV_PDBG;
  // dbg (SV_PERSIST_DEBUG, profiling only, results invalid): 1 no hand-off waits, 2 no recurrent
  // MFMAs, 8 no post-arrival stores
  constexpr int BM = 32, U = 64, KR = 2;
  constexpr int K = NS * 16, LDA = K + 8;
  constexpr int LDP = 4 * U + 4;  // pre [BM][LDP] fp32
  constexpr int LDB = U + 8;      // hsb [BM][LDB] bf16
  constexpr int LDT = BM + 8;     // hts [U][LDT] bf16
  constexpr int NR = NS - NL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);                // [BM][LDA]
  float* pre = reinterpret_cast<float*>(smem + BM * LDA * 2);  // [BM][LDP]
  bf16_t* hsb = reinterpret_cast<bf16_t*>(pre + BM * LDP);     // [BM][LDB]
  bf16_t* hts = hsb + BM * LDB;                                // [U][LDT]
  char* wl = reinterpret_cast<char*>(hts + U * LDT);           // [4 waves][NL][64 lanes][16 B]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * U, b0 = rb * BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  // W_hh fragments of gate g: B[k][n] = W[g H + j0 + n][k], lane (n = r, k = 16 s + 8 hh .. +7)
  bf16x8_t wa[NS], wb[NR];
  {
    const bf16_t* ra = whh_bf + ((long)g * H + j0 + r) * K + 8 * hh;
    const bf16_t* rbp = ra + 32L * K;
    const bool oka = j0 + r < H, okb = j0 + 32 + r < H;
    const bf16x8_t z = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) wa[s] = oka ? *reinterpret_cast<const bf16x8_t*>(ra + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NR; ++s) wb[s] = okb ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = NR; s < NS; ++s)
      *reinterpret_cast<bf16x8_t*>(wl + ((g * NL + s - NR) * 64 + lane) * 16) =
          okb ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+a"(wa[s]));
#pragma unroll
    for (int s = 0; s < 64 - NS; ++s) asm volatile("" : "+a"(wb[s]));
  }
  auto wl_read = [&](int j) { return *reinterpret_cast<const bf16x8_t*>(wl + ((g * NL + j) * 64 + lane) * 16); };
  // fused input projection (XF > 0): W_ih fragments of both 32-column halves of gate g (zero past
  // F) and the columns' biases
  constexpr int XS = (XF + 1) / 2, F = 8 * XF;
  bf16x8_t wxa[XS > 0 ? XS : 1], wxb[XS > 0 ? XS : 1];
  float xba = 0.f, xbb = 0.f;
  if constexpr (XF > 0) {
    const int ca = g * H + j0 + r, cb = ca + 32;
    const bf16x8_t z = {};
#pragma unroll
    for (int s2 = 0; s2 < XS; ++s2) {
      const bool kok = 16 * s2 + 8 * hh < F;
      wxa[s2] = (kok && j0 + r < H) ? *reinterpret_cast<const bf16x8_t*>(wih_bf + (long)ca * F + 16 * s2 + 8 * hh) : z;
      wxb[s2] =
          (kok && j0 + 32 + r < H) ? *reinterpret_cast<const bf16x8_t*>(wih_bf + (long)cb * F + 16 * s2 + 8 * hh) : z;
    }
    if (j0 + r < H) xba = (b_ih ? b_ih[ca] : 0.f) + (b_hh ? b_hh[ca] : 0.f);
    if (j0 + 32 + r < H) xbb = (b_ih ? b_ih[cb] : 0.f) + (b_hh ? b_hh[cb] : 0.f);
  }
  // x_t A fragments (rows b0 + r, k = 16 s + 8 hh); rows past B and k past F read zeros
  u32x4_t xa[XS > 0 ? XS : 1];
  auto load_x = [&](int tt) {
    if constexpr (XF > 0) {
      const __amdgpu_buffer_rsrc_t rxs = sv_rsrc(x_bf + (long)tt * B * F, (unsigned)((long)B * F * 2));
#pragma unroll
      for (int s2 = 0; s2 < XS; ++s2) {
        const unsigned off =
            16 * s2 + 8 * hh < F ? ((unsigned)(b0 + r) * (unsigned)F + 16 * s2 + 8 * hh) * 2u : 0xFFFFFFF0u;
        xa[s2] = __builtin_amdgcn_raw_buffer_load_b128(rxs, off, 0, 0);
      }
    }
  };
  // elementwise map: thread -> 4 consecutive units (u4) x rows 2 brow, 2 brow + 1
  const int u4 = (tid & 15) * 4, brow = tid >> 4;
  const long Bv = B;
  float cst[KR][4];
#pragma unroll
  for (int k = 0; k < KR; ++k)
#pragma unroll
    for (int v = 0; v < 4; ++v) cst[k][v] = 0.f;
  // staging map: BM rows x K bf16 = 3072 16-B chunks, 12 per thread in two halves of 6
  constexpr int HALF = K / 2, CH = BM * HALF / 8 / 256;
  uint2 xg[KR][4];
  auto load_xg = [&](int tt) {
    if (dbg & 16) tt = 0;  // (profiling only: every step reads step 0's x-projection, cache-hot)
    if constexpr (XF > 0) {
      load_x(tt);
      return;
    }
    const __amdgpu_buffer_rsrc_t rx = sv_rsrc(gates + (long)tt * BG, (unsigned)(BG * 2));
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + 2 * brow + k;
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
      if (tid == 0 && !(dbg & 1)) persist_wait(my_cnt, producers * (unsigned)t, status, limit, 1u);
      __syncthreads();
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(h_bf + (long)t * BH, (unsigned)(BH * 2));
      auto stage_load = [&](int half, uint4 (&v)[CH]) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int q = tid + 256 * i, row = q / (HALF / 8), c = (q % (HALF / 8)) * 8 + half * HALF;
          const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(
              ra, ((unsigned)(b0 + row) * (unsigned)H + (unsigned)c) * 2u, 0, 16 /* sc1 */);
          v[i] = uint4{x.x, x.y, x.z, x.w};
        }
      };
      auto stage_store = [&](int half, const uint4 (&v)[CH]) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int q = tid + 256 * i, row = q / (HALF / 8), c = (q % (HALF / 8)) * 8 + half * HALF;
          *reinterpret_cast<uint4*>(As + row * LDA + c) = v[i];
        }
      };
      const bf16_t* A0 = As + r * LDA + 8 * hh;
      auto afrag = [&](int s) { return *reinterpret_cast<const bf16x8_t*>(A0 + 16 * s); };
      bf16x8_t wq[2];
      // k-steps [s0, s1) from the staged A tile: A fragments PA ahead (within the range), the
      // LDS-resident W fragments two ahead
      auto mma_range = [&](int s0, int s1) {
        bf16x8_t fa[PA];
#pragma unroll
        for (int p = 0; p < PA; ++p) fa[p] = afrag(s0 + p);
#pragma unroll
        for (int s = s0; s < s1; ++s) {
          acc0 = mfma_bf16(fa[(s - s0) % PA], wa[s], acc0);
          acc1 = mfma_bf16(fa[(s - s0) % PA], s < NR ? wb[s < NR ? s : 0] : wq[s & 1], acc1);
          if (s + PA < s1) fa[(s - s0) % PA] = afrag(s + PA);
          if (s + 2 >= NR && s + 2 < NS) wq[s & 1] = wl_read(s + 2 - NR);
          // a full scheduling barrier per k-step: with group barriers the scheduler satisfied
          // "one DS read here" with the read the next MFMA needs, sinking every fragment read to
          // just before its use (prefetch distance 0, one exposed LDS latency per k-step)
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          uint4 v[CH];
          stage_load(half, v);
          stage_store(half, v);
        }
        __syncthreads();
        load_xg(t);
        __builtin_amdgcn_sched_barrier(0);
        if (!(dbg & 2)) mma_range(0, NS);
      }
    } else {
      load_xg(0);
    }
    if constexpr (XF > 0) {  // pre-activation = recurrent part + bf16(x_t W_ih^T + b_ih + b_hh)
      f32x16 x0, x1;
#pragma unroll
      for (int i = 0; i < 16; ++i) x0[i] = x1[i] = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < XS; ++s2) {
        x0 = mfma_bf16(__builtin_bit_cast(bf16x8_t, xa[s2]), wxa[s2], x0);
        x1 = mfma_bf16(__builtin_bit_cast(bf16x8_t, xa[s2]), wxb[s2], x1);
      }
      add_round_bf16x(acc0, x0, xba);
      add_round_bf16x(acc1, x1, xbb);
    }
    // gate exchange: wave g's [32 rows][64 units] -> pre[row][g * 64 + unit]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      pre[acc_row(i, lane) * LDP + g * U + r] = acc0[i];
      pre[acc_row(i, lane) * LDP + g * U + 32 + r] = acc1[i];
    }
    __syncthreads();
    uint2 act[KR][4];
    float4 cv[KR], hv[KR];
    unsigned hk0[2] = {0u, 0u};  // row 2 brow's bf16 h (unit pairs), joined with row 2 brow + 1's
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = 2 * brow + k;
      float4 pq[4], xf[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pq[q] = *reinterpret_cast<const float4*>(pre + b * LDP + q * U + u4);
        xf[q] = XF > 0 ? float4{0.f, 0.f, 0.f, 0.f} : unpack_bf4(xg[k][q]);
      }
      float ao[4][4], co[4], ho[4];
      unsigned pk[2] = {0u, 0u};
#pragma unroll
      for (int vp = 0; vp < 2; ++vp) {  // unit pairs in packed fp32
        const int v0 = 2 * vp, v1 = v0 + 1;
        const f2_t pv[4] = {f2_t{pq[0][v0], pq[0][v1]}, f2_t{pq[1][v0], pq[1][v1]}, f2_t{pq[2][v0], pq[2][v1]},
                            f2_t{pq[3][v0], pq[3][v1]}};
        const f2_t xv[4] = {f2_t{xf[0][v0], xf[0][v1]}, f2_t{xf[1][v0], xf[1][v1]}, f2_t{xf[2][v0], xf[2][v1]},
                            f2_t{xf[3][v0], xf[3][v1]}};
        f2_t a4[4], h;
        const f2_t c = lstm_cell_fwd2(pv, xv, f2_t{cst[k][v0], cst[k][v1]}, a4, h);
        cst[k][v0] = c.x;
        cst[k][v1] = c.y;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ao[q][v0] = a4[q].x;
          ao[q][v1] = a4[q].y;
        }
        co[v0] = c.x;
        co[v1] = c.y;
        ho[v0] = h.x;
        ho[v1] = h.y;
        pk[vp] = pack_bf2(h.x, h.y);
        const bf16_t e0 = (bf16_t)pk[vp], e1 = (bf16_t)(pk[vp] >> 16);
        if (k == 0) {
          hk0[vp] = pk[vp];
        } else {  // a unit's two rows as one 4-B write into the transposed tile (chunk swizzle)
          const int ua = u4 + v0, ub_ = u4 + v1;
          *reinterpret_cast<unsigned*>(hts + ua * LDT + ((2 * brow) ^ (((ua >> 4) & 3) << 3))) =
              (hk0[vp] & 0xffffu) | ((unsigned)e0 << 16);
          *reinterpret_cast<unsigned*>(hts + ub_ * LDT + ((2 * brow) ^ (((ub_ >> 4) & 3) << 3))) =
              (hk0[vp] >> 16) | ((unsigned)e1 << 16);
        }
      }
      *reinterpret_cast<uint2*>(hsb + b * LDB + u4) = uint2{pk[0], pk[1]};
#pragma unroll
      for (int q = 0; q < 4; ++q) act[k][q] = pack_bf4(ao[q][0], ao[q][1], ao[q][2], ao[q][3]);
      cv[k] = float4{co[0], co[1], co[2], co[3]};
      hv[k] = float4{ho[0], ho[1], ho[2], ho[3]};
    }
    __syncthreads();  // hsb, hts complete
    // the hand-off: h_t bf16, 32 rows x 8 chunks of 8 units, one 16-B sc1 store per thread
    {
      const int row = tid >> 3, c = tid & 7, gb = b0 + row;
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(h_bf + (long)(t + 1) * BH, (unsigned)(BH * 2));
      if (gb < B && j0 + 8 * c < H) {
        const uint4 v = *reinterpret_cast<const uint4*>(hsb + row * LDB + 8 * c);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw,
                                               ((unsigned)gb * (unsigned)H + (unsigned)(j0 + 8 * c)) * 2u, 0,
                                               16 /* sc1 */);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && persist_arrive_ok(fault, t == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // off the critical chain: activations, c, h and hT of step t
    if (dbg & 8) continue;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const long gb = b0 + 2 * brow + k;
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
    if (hT) {  // 64 unit rows x 4 chunks of 8 batch columns (padding columns get zeros)
      const int u = tid >> 2, c = tid & 3, gb = b0 + 8 * c;
      if (gb < Bp && j0 + u < H) {
        bf16_t* row = hT + (long)(j0 + u) * ldhT;
        *reinterpret_cast<uint4*>(row + (long)(t + 1) * Bp + gb) =
            *reinterpret_cast<const uint4*>(hts + u * LDT + 8 * (c ^ ((u >> 4) & 3)));
        if (t == 0) *reinterpret_cast<uint4*>(row + gb) = uint4{0u, 0u, 0u, 0u};
      }
    }
  }
}

int sv_persist3_fwd_launch(dim3 grid, int nub, hipStream_t stream, const bf16_t* whh_bf, bf16_t* gates, float* c_tm,
                           float* h_tm, bf16_t* h_bf, bf16_t* hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt,
                           int xcd, unsigned* status, unsigned limit, int fault, const bf16_t* x_bf, int F,
                           const bf16_t* wih_bf, const float* b_ih, const float* b_hh, int dbg) {
  constexpr size_t base = (size_t)32 * (768 + 8) * 2 + (size_t)32 * (4 * 64 + 4) * 4 + (size_t)32 * 72 * 2 +
                          (size_t)64 * 40 * 2;
  // h_{t-1} staged through registers in two halves.  Measured alternatives (bit-identical results,
  // deleted): LDS-DMA staging 921 vs 843 us per layer at c3 (r05, on the scalar-addressed W3Dma: 908
  // vs 854); the second half in flight during the first half's MFMAs 4.77 vs 4.67 ms for the
  // 3-layer forward
  if (x_bf) {  // layer 0, F = 40: the W_ih fragments take registers, so more W_hh fragments live in LDS
    if (F != 40 || !wih_bf) return SV_EARG;
    constexpr int NL = 16;
    hipLaunchKernelGGL((lstm_persist3_fwd_bf16_kernel<48, NL, 4, 5>), grid, dim3(256), base + (size_t)4 * NL * 1024,
                       stream, whh_bf, gates, c_tm, h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit,
                       fault, x_bf, wih_bf, b_ih, b_hh, dbg);
  } else {
    constexpr int NL = 12;
    hipLaunchKernelGGL((lstm_persist3_fwd_bf16_kernel<48, NL, 4, 0>), grid, dim3(256), base + (size_t)4 * NL * 1024,
                       stream, whh_bf, gates, c_tm, h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit,
                       fault, nullptr, nullptr, nullptr, nullptr, dbg);
  }
  return (int)hipGetLastError();
}

// ============================================================================
// 16-row wide forward (c5's per-rank batch: 320 rows = 20 x 12 workgroups, layers without the
// fused input projection).  Tile: 16 batch rows x 64 units x 4 gates.  Against the 32 x 32 tile
// (the same 240 workgroups) each workgroup stages half the h_{t-1} bytes per step (24 KB) and
// reads half the A fragments from LDS, for the same MFMA time: v_mfma_f32_16x16x32_bf16 with
// wave g's W_hh rows of the 64 units (4 column tiles x 24 k-steps = 96 fragments: 64 in AGPRs, the
// rest in VGPRs and NL in LDS, one per k-step of the last NL) as the first operand, so a lane's
// 4 accumulators are 4 consecutive units of one row (16-B exchange writes).  Same cell helper,
// hand-off (bf16 h rows, 16-B sc1 stores, one counter per 16-row block) and outputs (activations,
// c, h^T, fp32 h_{T-1}) as the 32-row kernels.  The MFMA's k-blocking differs (32 per instruction
// against 16) but not the k order, and the outputs are bit-identical to the per-step schedule's
// (tests/test_gpu_persist.py asserts it at 320 and 288 rows).  Measured: c5 rank step 6.58-6.62 vs
// 6.67-6.69 ms.
// ============================================================================
// XF > 0 (layer 0, F = 8 XF <= 64 features): the input projection formed in the kernel from x_bf [T,B,F] and W_ih
// [4H,F] (two k-steps of 32, zero past F), rounded to bf16 with its biases as the K1 path stores it, then
// added to the recurrent part (the 32-row kernels' fused form)
template <int NL, int PA, int XF>
__global__ __launch_bounds__(256, 1) void lstm_persist16_fwd_bf16_kernel(
    const bf16_t* __restrict__ whh_bf, bf16_t* __restrict__ gates, float* __restrict__ c_tm, float* __restrict__ h_tm,
    bf16_t* h_bf, bf16_t* __restrict__ hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt, int nub, int xcd,
    unsigned* status, unsigned limit, int fault, const bf16_t* __restrict__ x_bf, const bf16_t* __restrict__ wih_bf,
    const float* __restrict__ b_ih, const float* __restrict__ b_hh) {
  constexpr int BM = 16, U = 64, K = 768, KS = K / 32;  // 24 k-steps of 32
  constexpr int NLS = KS - NL;                          // k-steps whose 4 fragments are all in registers
  constexpr int NRF = 4 * NLS + 3 * NL;                 // register fragments (84 at NL = 12)
  constexpr int NA = 64;                                // ... of which in AGPRs
  constexpr int LDA = K + 8;                            // As [BM][LDA] bf16
  constexpr int LDP = 4 * U + 4;                        // pre [BM][LDP] fp32
  constexpr int LDB = U + 8;                            // hsb [BM][LDB] bf16
  constexpr int LDT = BM + 8;                           // hts [U][LDT] bf16
  static_assert(NRF > NA && PA >= 1 && PA <= KS, "register plan");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  float* pre = reinterpret_cast<float*>(smem + BM * LDA * 2);
  bf16_t* hsb = reinterpret_cast<bf16_t*>(pre + BM * LDP);
  bf16_t* hts = hsb + BM * LDB;
  char* wl = reinterpret_cast<char*>(hts + U * LDT);  // [4 waves][NL][64 lanes][16 B]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  int ub, rb;
  persist_tile(xcd, nub, ub, rb);
  const int j0 = ub * U, b0 = rb * BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  unsigned* my_cnt = cnt + rb * SV_PCNT_STRIDE;
  const unsigned producers = nub;
  // fragment (k-step s, column tile nt) of gate g: lane -> W_hh row g H + j0 + 16 nt + fr, k = 32 s +
  // 8 fq.  Register index: 4 s + nt for s < NLS, then 3 per k-step (nt = 0..2); nt = 3 of the last NL
  // k-steps in LDS
  constexpr auto ridx = [](int s_, int nt_) { return s_ < NLS ? 4 * s_ + nt_ : 4 * NLS + 3 * (s_ - NLS) + nt_; };
  bf16x8_t wr[NRF];
  {
    const bf16_t* base = whh_bf + ((long)g * H + j0 + fr) * K + 8 * fq;
    const bf16x8_t z = {};
#pragma unroll
    for (int s_ = 0; s_ < KS; ++s_)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x8_t v = j0 + 16 * nt + fr < H ? *reinterpret_cast<const bf16x8_t*>(base + (long)16 * nt * K + 32 * s_) : z;
        if (s_ >= NLS && nt == 3)
          *reinterpret_cast<bf16x8_t*>(wl + ((g * NL + s_ - NLS) * 64 + lane) * 16) = v;
        else
          wr[ridx(s_, nt)] = v;
      }
#pragma unroll
    for (int f = 0; f < NA; ++f) asm volatile("" : "+a"(wr[f]));
  }
  auto wl_read = [&](int j) { return *reinterpret_cast<const bf16x8_t*>(wl + ((g * NL + j) * 64 + lane) * 16); };
  // fused input projection (XF > 0): W_ih fragments of the 4 column tiles (k = 32 s2 + 8 fq, zero
  // past F) and the biases of the lane's accumulator columns (unit 16 nt + 4 fq + v)
  constexpr int F = 8 * XF;
  static_assert(F <= 64, "two k-steps of 32");
  bf16x8_t wx[XF > 0 ? 2 : 1][4];
  float xb[XF > 0 ? 4 : 1][4];
  if constexpr (XF > 0) {
    const bf16x8_t z = {};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int row = g * H + j0 + 16 * nt + fr, k = 32 * s2 + 8 * fq;
        wx[s2][nt] = (k < F && j0 + 16 * nt + fr < H) ? *reinterpret_cast<const bf16x8_t*>(wih_bf + (long)row * F + k) : z;
      }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int c = g * H + j0 + 16 * nt + 4 * fq + v;
        xb[nt][v] = j0 + 16 * nt + 4 * fq + v < H ? (b_ih ? b_ih[c] : 0.f) + (b_hh ? b_hh[c] : 0.f) : 0.f;
      }
  }
  u32x4_t xa[2];
  auto load_x = [&](int tt) {  // x_t rows b0 + fr, k = 32 s2 + 8 fq (zeros past F)
    const __amdgpu_buffer_rsrc_t rxs = sv_rsrc(x_bf + (long)tt * B * F, (unsigned)((long)B * F * 2));
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int k = 32 * s2 + 8 * fq;
      xa[s2] = __builtin_amdgcn_raw_buffer_load_b128(rxs, k < F ? ((unsigned)(b0 + fr) * (unsigned)F + k) * 2u : 0xFFFFFFF0u,
                                                     0, 0);
    }
  };
  // elementwise map: thread -> row brow, 4 consecutive units u4
  const int u4 = (tid & 15) * 4, brow = tid >> 4;
  float cst[4] = {0.f, 0.f, 0.f, 0.f};
  uint2 xg[4];
  auto load_xg = [&](int tt) {  // bf16(x W_ih^T + b) of step tt (K1 output), rows past B read zeros
    if constexpr (XF > 0) {
      load_x(tt);
      return;
    }
    const __amdgpu_buffer_rsrc_t rx = sv_rsrc(gates + (long)tt * BG, (unsigned)(BG * 2));
    const long gb = b0 + brow, gbv = gb < B ? gb : (long)B + 64;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x2_t x = __builtin_amdgcn_raw_buffer_load_b64(rx, (unsigned)((gbv * G + q * H + j0 + u4) * 2), 0, 0);
      xg[q] = uint2{x.x, x.y};
    }
  };
  constexpr int CH = BM * K / 8 / 256;  // 16-B staging chunks per thread (6)
  for (int t = 0; t < T; ++t) {
    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t > 0) {
      if (tid == 0) persist_wait(my_cnt, producers * (unsigned)t, status, limit, 1u);
      __syncthreads();
      {  // h_{t-1} of the 16 rows into LDS (sc1 loads: written by other workgroups this launch)
        const __amdgpu_buffer_rsrc_t ra = sv_rsrc(h_bf + (long)t * BH, (unsigned)(BH * 2));
        uint4 v[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int q = tid + 256 * i, row = q / (K / 8), c = (q % (K / 8)) * 8;
          const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(
              ra, ((unsigned)(b0 + row) * (unsigned)H + (unsigned)c) * 2u, 0, 16 /* sc1 */);
          v[i] = uint4{x.x, x.y, x.z, x.w};
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int q = tid + 256 * i, row = q / (K / 8), c = (q % (K / 8)) * 8;
          *reinterpret_cast<uint4*>(As + row * LDA + c) = v[i];
        }
      }
      __syncthreads();
      load_xg(t);
      __builtin_amdgcn_sched_barrier(0);
      const bf16_t* A0 = As + fr * LDA + 8 * fq;
      auto afrag = [&](int s_) { return *reinterpret_cast<const bf16x8_t*>(A0 + 32 * s_); };
      bf16x8_t fa[PA], wq[2];
#pragma unroll
      for (int p_ = 0; p_ < PA; ++p_) fa[p_] = afrag(p_);
#pragma unroll
      for (int s_ = 0; s_ < KS; ++s_) {
        const bf16x8_t a = fa[s_ % PA];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(s_ >= NLS && nt == 3 ? wq[s_ & 1] : wr[ridx(s_, nt < 3 || s_ < NLS ? nt : 0)],
                                                            a, acc[nt], 0, 0, 0);
        if (s_ + PA < KS) fa[s_ % PA] = afrag(s_ + PA);
        if (s_ + 2 >= NLS && s_ + 2 < KS) wq[s_ & 1] = wl_read(s_ + 2 - NLS);  // two k-steps ahead
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      load_xg(0);
    }
    if constexpr (XF > 0) {  // pre-activation = recurrent part + bf16(x_t W_ih^T + b_ih + b_hh)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wx[s2][nt], __builtin_bit_cast(bf16x8_t, xa[s2]), x, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 4; v += 2) {
          const f2_t r = round_bf2(f2_t{x[v], x[v + 1]} + f2_t{xb[nt][v], xb[nt][v + 1]});
          const f2_t sm = f2_t{acc[nt][v], acc[nt][v + 1]} + r;
          acc[nt][v] = sm.x;
          acc[nt][v + 1] = sm.y;
        }
      }
    }
    // gate exchange: wave g's [16 rows][64 units] -> pre[row][g * 64 + unit]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) *reinterpret_cast<f32x4*>(pre + fr * LDP + g * U + 16 * nt + 4 * fq) = acc[nt];
    __syncthreads();
    uint2 act[4];
    float4 cv, hv;
    {
      const int b = brow;
      float4 pq[4], xf[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pq[q] = *reinterpret_cast<const float4*>(pre + b * LDP + q * U + u4);
        xf[q] = XF > 0 ? float4{0.f, 0.f, 0.f, 0.f} : unpack_bf4(xg[q]);
      }
      float ao[4][4], co[4], ho[4];
#pragma unroll
      for (int vp = 0; vp < 2; ++vp) {  // unit pairs in packed fp32
        const int v0 = 2 * vp, v1 = v0 + 1;
        const f2_t pv[4] = {f2_t{pq[0][v0], pq[0][v1]}, f2_t{pq[1][v0], pq[1][v1]}, f2_t{pq[2][v0], pq[2][v1]},
                            f2_t{pq[3][v0], pq[3][v1]}};
        const f2_t xv[4] = {f2_t{xf[0][v0], xf[0][v1]}, f2_t{xf[1][v0], xf[1][v1]}, f2_t{xf[2][v0], xf[2][v1]},
                            f2_t{xf[3][v0], xf[3][v1]}};
        f2_t a4[4], h;
        const f2_t c = lstm_cell_fwd2(pv, xv, f2_t{cst[v0], cst[v1]}, a4, h);
        cst[v0] = c.x;
        cst[v1] = c.y;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ao[q][v0] = a4[q].x;
          ao[q][v1] = a4[q].y;
        }
        co[v0] = c.x;
        co[v1] = c.y;
        ho[v0] = h.x;
        ho[v1] = h.y;
      }
      const unsigned pk0 = pack_bf2(ho[0], ho[1]), pk1 = pack_bf2(ho[2], ho[3]);
      *reinterpret_cast<uint2*>(hsb + b * LDB + u4) = uint2{pk0, pk1};
      hts[(u4 + 0) * LDT + b] = (bf16_t)pk0;
      hts[(u4 + 1) * LDT + b] = (bf16_t)(pk0 >> 16);
      hts[(u4 + 2) * LDT + b] = (bf16_t)pk1;
      hts[(u4 + 3) * LDT + b] = (bf16_t)(pk1 >> 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) act[q] = pack_bf4(ao[q][0], ao[q][1], ao[q][2], ao[q][3]);
      cv = float4{co[0], co[1], co[2], co[3]};
      hv = float4{ho[0], ho[1], ho[2], ho[3]};
    }
    __syncthreads();  // hsb, hts complete
    // the hand-off: h_t bf16, 16 rows x 8 chunks of 8 units, one 16-B sc1 store per thread of 128
    if (tid < BM * 8) {
      const int row = tid >> 3, c = tid & 7, gb = b0 + row;
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(h_bf + (long)(t + 1) * BH, (unsigned)(BH * 2));
      if (gb < B && j0 + 8 * c < H) {
        const uint4 v = *reinterpret_cast<const uint4*>(hsb + row * LDB + 8 * c);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw,
                                               ((unsigned)gb * (unsigned)H + (unsigned)(j0 + 8 * c)) * 2u, 0,
                                               16 /* sc1 */);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && persist_arrive_ok(fault, t == 0))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // off the critical chain: activations, c, h and h^T of step t
    {
      const long gb = b0 + brow;
      if (gb < B) {
        bf16_t* gp = gates + (long)t * BG + gb * G + j0 + u4;
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(gp + q * H) = act[q];
        *reinterpret_cast<float4*>(c_tm + (long)t * BH + gb * H + j0 + u4) = cv;
        if (t == T - 1) *reinterpret_cast<float4*>(h_tm + (long)(t + 1) * BH + gb * H + j0 + u4) = hv;
      }
    }
    if (hT && tid < U * 2) {  // 64 unit rows x 2 chunks of 8 batch columns
      const int u = tid >> 1, c = tid & 1, gb = b0 + 8 * c;
      if (gb < Bp && j0 + u < H) {
        bf16_t* row = hT + (long)(j0 + u) * ldhT;
        *reinterpret_cast<uint4*>(row + (long)(t + 1) * Bp + gb) = *reinterpret_cast<const uint4*>(hts + u * LDT + 8 * c);
        if (t == 0) *reinterpret_cast<uint4*>(row + gb) = uint4{0u, 0u, 0u, 0u};
      }
    }
  }
}

int sv_persist16_fwd_launch(int nrb, int nub, hipStream_t stream, const bf16_t* whh_bf, bf16_t* gates, float* c_tm,
                            float* h_tm, bf16_t* h_bf, bf16_t* hT, long ldhT, int T, int Bp, int B, int H, unsigned* cnt,
                            int xcd, unsigned* status, unsigned limit, int fault, const bf16_t* x_bf, int F,
                            const bf16_t* wih_bf, const float* b_ih, const float* b_hh) {
  constexpr int NL = 12;
  constexpr size_t lds = (size_t)16 * (768 + 8) * 2 + (size_t)16 * (4 * 64 + 4) * 4 + (size_t)16 * 72 * 2 +
                         (size_t)64 * 24 * 2 + (size_t)4 * NL * 1024;
  if (H != 768 || B % 16 || nub != H / 64) return SV_EARG;
  if (x_bf) {  // layer 0, F = 40
    if (F != 40 || !wih_bf) return SV_EARG;
    hipLaunchKernelGGL((lstm_persist16_fwd_bf16_kernel<NL, 4, 5>), dim3(nrb * nub), dim3(256), lds, stream, whh_bf,
                       gates, c_tm, h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, x_bf, wih_bf,
                       b_ih, b_hh);
  } else {
    hipLaunchKernelGGL((lstm_persist16_fwd_bf16_kernel<NL, 4, 0>), dim3(nrb * nub), dim3(256), lds, stream, whh_bf,
                       gates, c_tm, h_tm, h_bf, hT, ldhT, T, Bp, B, H, cnt, nub, xcd, status, limit, fault, nullptr,
                       nullptr, nullptr, nullptr);
  }
  return (int)hipGetLastError();
}

// ============================================================================
// Layer-wavefront backward for small per-GPU batches (c4's 80 rows per rank): ONE launch runs the
// backward recurrences of all L layers.  The per-layer schedule at B = 80 runs 72 workgroups per
// layer, one layer after another, each followed by its dx = dG W_ih GEMM; here workgroup (l, ub,
// rb) -- 32 rows x 32 units, 4 waves, one per gate -- holds BOTH of its gate's weight slices, W_hh^T
// (for dh_rec = dG_{t+1} W_hh) and W_ih^T (for layer l-1's upstream gradient dx_{t+1} =
// dG_{t+1} W_ih), and streams dG_{t+1} once for both: two accumulators per A fragment (the wide
// backward's register plan: 256 AGPRs + VGPRs + NL LDS-resident fragments).  Layer l's iteration t
// computes dh_rec_t and dx_{t+1}, hands dx_{t+1} (fp32, 16-B sc1 stores) to layer l-1 with its dG_t,
// and consumes dx_t from layer l+1's iteration t-1 as dh_up: so layer l runs two iterations behind
// layer l+1, and the chain is T + 2(L-1) + 1 dependent steps (layers >= 1 run one extra iteration,
// t = -1, that only forms dx_0).  One counter per (layer, row block) counts finished iterations;
// both hand-offs of an iteration are drained before its arrival (hand-off table row 1).
//   own layer:   iteration t needs dG_{t+1}  -> counter >= nub (T - 1 - t)
//   layer above: iteration t needs dx_t      -> its counter >= nub (T - t + 1)
// Outputs as the per-layer schedule (dG^T per layer, bias partials, the dx buffers), except the
// in-kernel dx sums the gates' k-ordered partials in gate order (the dx GEMM sums K = 4H in
// k-tile order): bf16-level agreement, not bitwise.
// ============================================================================
template <int NS, int P, int NL>
__global__ __launch_bounds__(256, 1) void lstm_wave_bwd_bf16_kernel(const WaveBwdArgs a) {
  constexpr int BM = 32, U = 32;
  constexpr int LDR = U + 4;         // red0 / red1 [4][BM][LDR] fp32
  constexpr int LDG = 4 * U + 8;     // dgs [BM][LDG] bf16
  constexpr int LDT = BM + 8;        // gts [4U][LDT] bf16
  constexpr int FRAG = NS * 64 * 8;  // dgf elements of one (row block, gate)
  constexpr int NR = NS - NL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red0 = reinterpret_cast<float*>(smem);
  float* red1 = red0 + 4 * BM * LDR;
  bf16_t* dgs = reinterpret_cast<bf16_t*>(red1 + 4 * BM * LDR);
  bf16_t* gts = dgs + BM * LDG;
  char* ewa = reinterpret_cast<char*>(gts + 4 * U * LDT);  // [BM][256 B]: gate q's 64 B at ((q + row) & 3) * 64
  float* ewc = reinterpret_cast<float*>(ewa + BM * 256);    // [BM][U] c_{t-1}
  char* wl = reinterpret_cast<char*>(ewc + BM * U);         // [4 waves][NL][64 lanes][16 B]
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int T = a.T, B = a.B, H = a.H, nub = a.nub, nrb = a.nrb;
  int ub, rb, l;
  {
    const int i = blockIdx.x, n = gridDim.x;
    const int x = i & 7, q = n >> 3, rr = n & 7;
    const int Lg = x * q + min(x, rr) + (i >> 3);
    ub = Lg % nub;
    rb = (Lg / nub) % nrb;
    l = Lg / (nub * nrb);
  }
  const int j0 = ub * U, b0 = rb * BM;
  const long G = 4L * H, BH = (long)B * H, BG = (long)B * G;
  const long FS = (long)nrb * BM * G;
  const bool has_dx = l > 0, has_up = l < WB_L - 1;
  unsigned* my_cnt = a.cnt[l] + rb * SV_PCNT_STRIDE;
  unsigned* up_cnt = has_up ? a.cnt[l + 1] + rb * SV_PCNT_STRIDE : nullptr;
  const unsigned producers = nub;
  // gate g's fragments: W_hh^T (wa) and W_ih^T (wb, layers >= 1): B[k][n] = W[g H + k][j0 + n]
  bf16x8_t wa[NS], wb[NR];
  {
    const bf16_t* ra = a.whhT[l] + (long)(j0 + r) * G + (long)g * H + 8 * hh;
    const bf16_t* rbp = has_dx ? a.wihT[l] + (long)(j0 + r) * a.ldwih + (long)g * H + 8 * hh : ra;
    const bool ok = j0 + r < H;
    const bf16x8_t z = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) wa[s] = ok ? *reinterpret_cast<const bf16x8_t*>(ra + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NR; ++s) wb[s] = (ok && has_dx) ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = NR; s < NS; ++s)
      *reinterpret_cast<bf16x8_t*>(wl + ((g * NL + s - NR) * 64 + lane) * 16) =
          (ok && has_dx) ? *reinterpret_cast<const bf16x8_t*>(rbp + 16 * s) : z;
#pragma unroll
    for (int s = 0; s < NS; ++s) asm volatile("" : "+a"(wa[s]));
#pragma unroll
    for (int s = 0; s < 64 - NS; ++s) asm volatile("" : "+a"(wb[s]));
  }
  auto wl_read = [&](int j) { return *reinterpret_cast<const bf16x8_t*>(wl + ((g * NL + j) * 64 + lane) * 16); };
  // elementwise map: thread -> 4 consecutive units (u4) of row brow
  const int u4 = (tid & 7) * 4, brow = tid >> 3;
  const long gb = b0 + brow, Bv = B;
  const long gbv = gb < Bv ? gb : Bv + 64;  // rows past B: offsets past every range
  float4 cv;
  float dcf[4] = {0.f, 0.f, 0.f, 0.f};
  float dbs[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) dbs[q][v] = 0.f;
  // step tt's activations and c_{tt-1} into LDS (LDS-DMA; not hand-off data)
  auto load_ew = [&](int tt) {
    const __amdgpu_buffer_rsrc_t ra_ = sv_rsrc(a.acts[l] + (long)tt * BG, (unsigned)(BG * 2));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = (g * 2 + j) * 64 + lane, row = p >> 4, sl = p & 15;
      const int q = ((sl >> 2) - row) & 3, c = sl & 3;
      const long rg = b0 + row, rgv = rg < Bv ? rg : Bv + 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, (lds_ptr_t)(ewa + (g * 2 + j) * 1024), 16,
                                               (unsigned)((rgv * G + q * H + j0 + 8 * c) * 2), 0, 0, 0);
    }
    // (readfirstlane: hipcc formed tt - 1 clamped on the VALU and wrapped the DMA in a waterfall loop)
    const int tm1 = __builtin_amdgcn_readfirstlane(tt > 0 ? tt - 1 : 0);
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(a.c[l] + (long)tm1 * BH, tt > 0 ? (unsigned)(BH * 4) : 0u);
    {
      const int p = g * 64 + lane, row = p >> 3, c = p & 7;
      const long rg = b0 + row, rgv = rg < Bv ? rg : Bv + 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rc_, (lds_ptr_t)((char*)ewc + g * 1024), 16,
                                               (unsigned)((rgv * H + j0 + 4 * c) * 4), 0, 0, 0);
    }
  };
  {
    const __amdgpu_buffer_rsrc_t rc_ = sv_rsrc(a.c[l] + (long)(T - 1) * BH, (unsigned)(BH * 4));
    const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(rc_, (unsigned)((gbv * H + j0 + u4) * 4), 0, 0);
    cv = float4{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
  }
  load_ew(T - 1);
  const int t_end = has_dx ? -1 : 0;
#ifdef SV_WB_STAMP  // A/B stamp builds only: wave 0's cycles per phase, summed over t = T-2 .. 0
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tl = __builtin_amdgcn_s_memtime();
  auto wmark = [&](int i, int t_) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    if (t_ < T - 1 && t_ >= 0) ph[i] += n - tl;
    tl = n;
  };
#define WB_MARK(i) wmark(i, t)
#else
#define WB_MARK(i)
#endif
  for (int t = T - 1; t >= t_end; --t) {
    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0.f;
    if (tid == 0) {
      if (t < T - 1) persist_wait(my_cnt, producers * (unsigned)(T - 1 - t), a.status, a.limit, 2u);
      if (has_up && t >= 0) persist_wait(up_cnt, producers * (unsigned)(T - t + 1), a.status, a.limit, 2u);
    }
    __syncthreads();
    WB_MARK(0);  // 0: hand-off waits (own layer, layer above) + the previous step's operand DMA
    // dh_up_t (hand-off from the layer above, sc1 loads) or the top layer's dh_last: issued before
    // the k-loop, so its round trip overlaps the MFMAs instead of opening the epilogue (the layer
    // above's counter was polled just now)
    float4 upv = float4{0.f, 0.f, 0.f, 0.f};
    u32x4_t upx = u32x4_t{0u, 0u, 0u, 0u};
    const float* upp = t >= 0 ? (has_up ? a.dx[l + 1] + (long)t * BH : (t == T - 1 ? a.dh_last : nullptr)) : nullptr;
    if (upp)
      upx = __builtin_amdgcn_raw_buffer_load_b128(sv_rsrc(upp, (unsigned)(BH * 4)), (unsigned)((gbv * H + j0 + u4) * 4),
                                                  0, 16 /* sc1: hand-off */);
    if (t < T - 1) {
      // A fragments of dG_{t+1} (this layer's hand-off slot): k-step s at (rb 4 + g) FRAG + s 512
      const __amdgpu_buffer_rsrc_t ra = sv_rsrc(a.dgf[l] + (long)(t + 1) * FS, (unsigned)(FS * 2));
      constexpr unsigned kstep = 1024u;
      const unsigned base0 = ((unsigned)(rb * 4 + g) * (unsigned)FRAG + (unsigned)lane * 8u) * 2u;
      u32x4_t fa[P];
#pragma unroll
      for (int s = 0; s < P; ++s) fa[s] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * s, 0, 16 /* sc1 */);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8_t wq[2];
      if (has_dx) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8_t av = __builtin_bit_cast(bf16x8_t, fa[s % P]);
          acc0 = mfma_bf16(av, wa[s], acc0);  // unused at t = -1
          acc1 = mfma_bf16(av, s < NR ? wb[s < NR ? s : 0] : wq[s & 1], acc1);
          if (s + 2 >= NR && s + 2 < NS) wq[s & 1] = wl_read(s + 2 - NR);
          if (s + P < NS) fa[s % P] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * (s + P), 0, 16);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          acc0 = mfma_bf16(__builtin_bit_cast(bf16x8_t, fa[s % P]), wa[s], acc0);
          if (s + P < NS) fa[s % P] = __builtin_amdgcn_raw_buffer_load_b128(ra, base0 + kstep * (s + P), 0, 16);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    WB_MARK(1);  // 1: k-loop (A fragments of dG_{t+1} from the hand-off + MFMAs)
    // per-gate partials: red0 = dh_rec, red1 = dx
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      red0[(g * BM + acc_row(i, lane)) * LDR + r] = acc0[i];
      red1[(g * BM + acc_row(i, lane)) * LDR + r] = acc1[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's operand DMA landed
    __syncthreads();
    upv = float4{__uint_as_float(upx.x), __uint_as_float(upx.y), __uint_as_float(upx.z), __uint_as_float(upx.w)};
    // dx_{t+1} of this layer: gate partials summed in gate order, 16-B sc1 stores (hand-off)
    if (has_dx && t < T - 1) {
      const int b = brow;
      const float4 p0 = *reinterpret_cast<const float4*>(red1 + (0 * BM + b) * LDR + u4);
      const float4 p1 = *reinterpret_cast<const float4*>(red1 + (1 * BM + b) * LDR + u4);
      const float4 p2 = *reinterpret_cast<const float4*>(red1 + (2 * BM + b) * LDR + u4);
      const float4 p3 = *reinterpret_cast<const float4*>(red1 + (3 * BM + b) * LDR + u4);
      float dxv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float s_ = p0[v];
        s_ += p1[v];
        s_ += p2[v];
        s_ += p3[v];
        dxv[v] = s_;
      }
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(a.dx[l] + (long)(t + 1) * BH, (unsigned)(BH * 4));
      if (gb < Bv && j0 + u4 < H)
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4_t{__float_as_uint(dxv[0]), __float_as_uint(dxv[1]), __float_as_uint(dxv[2]), __float_as_uint(dxv[3])},
            rw, (unsigned)((gb * H + j0 + u4) * 4), 0, 16 /* sc1 */);
    }
    if (t >= 0) {  // the cell backward of step t
      const int b = brow;
      const float4 r0 = *reinterpret_cast<const float4*>(red0 + (0 * BM + b) * LDR + u4);
      const float4 r1 = *reinterpret_cast<const float4*>(red0 + (1 * BM + b) * LDR + u4);
      const float4 r2 = *reinterpret_cast<const float4*>(red0 + (2 * BM + b) * LDR + u4);
      const float4 r3 = *reinterpret_cast<const float4*>(red0 + (3 * BM + b) * LDR + u4);
      const float4 cpv = *reinterpret_cast<const float4*>(ewc + b * U + u4);
      float4 f[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        f[q] = unpack_bf4(*reinterpret_cast<const uint2*>(ewa + b * 256 + ((q + b) & 3) * 64 + (u4 >> 3) * 16 +
                                                          (u4 & 7) * 2));
      unsigned pk[4][2] = {{0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}};
      float4 dh4 = r0;  // (elementwise, the scalar order)
      dh4 += r1;
      dh4 += r2;
      dh4 += r3;
      dh4 += upv;
      float ddv[4][4];
      lstm_cell_bwd_x4(dh4, f[0], f[1], f[2], f[3], cv, cpv, dcf, ddv);
      // (per element here: the packed pairs of pack_dg4 measured +10 us per c4 rank step)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float (&dd)[4] = ddv[v];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bf16_t e = to_bf(dd[q]);
          gts[(q * U + u4 + v) * LDT + b] = e;
          pk[q][v >> 1] |= (unsigned)e << (16 * (v & 1));
          dbs[q][v] += __uint_as_float((unsigned)e << 16);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(dgs + b * LDG + q * U + u4) = uint2{pk[q][0], pk[q][1]};
      cv = cpv;
    }
    __syncthreads();
    WB_MARK(2);  // 2: exchange, dh_up, dx_{t+1} hand-off stores, cell backward, dG tiles
    // the dG_t hand-off: 8 KB per workgroup in fragment order (gate, 2 k-steps), 16-B sc1 stores
    if (t >= 0) {
      const __amdgpu_buffer_rsrc_t rw = sv_rsrc(a.dgf[l] + (long)t * FS, (unsigned)(FS * 2));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = tid + 256 * i, c = p >> 6, ln = p & 63;
        const int gq = c >> 1, sl = c & 1;
        const uint4 v = *reinterpret_cast<const uint4*>(dgs + (ln & 31) * LDG + gq * U + 16 * sl + 8 * (ln >> 5));
        const unsigned off =
            ((unsigned)(rb * 4 + gq) * (unsigned)FRAG + (unsigned)(2 * ub + sl) * 512u + (unsigned)ln * 8u) * 2u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rw, off, 0, 16 /* sc1 */);
      }
    }
    // the 2 dG_t^T stores per thread (buffer stores; a piece past Bp to a dropped offset)
    // behind the hand-off stores, before their drain, which counts them (vmcnt(2): this wave's
    // older hand-off and dx stores done; a raw barrier: __syncthreads' fence would drain them)
    const bool ovl = t >= 0 && a.dgT[l] && 4L * H * a.lddgT * 2 < (1L << 32) - 64;
    if (ovl) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // (the dG^T stores stay younger than the hand-off's)
      const __amdgpu_buffer_rsrc_t rt = sv_rsrc(a.dgT[l], (unsigned)(4L * H * a.lddgT * 2));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = tid + 256 * i, gu = q >> 2, c = q & 3;
        const int gq = gu / U, gj = j0 + gu % U, gc = b0 + 8 * c;
        const long eo = ((long)gq * H + gj) * a.lddgT + (long)t * a.Bp + gc;
        const uint4 v = *reinterpret_cast<const uint4*>(gts + gu * LDT + 8 * c);
        const unsigned off = gc < a.Bp && gj < H ? (unsigned)(eo * 2) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rt, off, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if (tid == 0 && persist_arrive_ok(a.fault, t == T - 1))
      __hip_atomic_fetch_add(my_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    WB_MARK(3);  // 3: dG_t hand-off stores + drain + arrival
    if (!ovl && t >= 0 && a.dgT[l]) {  // dG_t^T (the dW GEMMs' operand), then the next step's operands
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = tid + 256 * i, gu = q >> 2, c = q & 3;
        const int gq = gu / U, gj = j0 + gu % U, gc = b0 + 8 * c;
        if (gc < a.Bp && gj < H) {
          const long eo = ((long)gq * H + gj) * a.lddgT + (long)t * a.Bp + gc;
          const uint4 v = *reinterpret_cast<const uint4*>(gts + gu * LDT + 8 * c);
          *reinterpret_cast<uint4*>(a.dgT[l] + eo) = v;
        }
      }
    }
    if (t > 0) load_ew(t - 1);
    WB_MARK(4);  // 4: dG^T stores + next operand DMA issue
  }
#ifdef SV_WB_STAMP
  if (tid == 0 && blockIdx.x < SV_NSTAMP_WG / 2) {  // second half of the stamp slots (the forward's use the first)
    unsigned long long* st =
        reinterpret_cast<unsigned long long*>(a.status + SV_SYNC_STAMP) + (SV_NSTAMP_WG / 2 + blockIdx.x) * SV_NSTAMP;
    for (int i = 0; i < 5; ++i) st[i] = ph[i];
    st[5] = (unsigned long long)l;
  }
#endif
#undef WB_MARK
  // bias gradients: this tile's column sums over its rows (in order), one partial per row block
  if (a.dbp[l]) {
    __syncthreads();
    float* dsum = red0;  // [BM][4U] fp32
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(dsum + brow * (4 * U) + q * U + u4) = float4{dbs[q][0], dbs[q][1], dbs[q][2], dbs[q][3]};
    __syncthreads();
    if (tid < 4 * U) {
      const int q = tid / U, gj = j0 + tid % U;
      float sum = 0.f;
      for (int b = 0; b < BM; ++b) sum += dsum[b * (4 * U) + tid];
      if (gj < H) a.dbp[l][(long)rb * G + (long)q * H + gj] = sum;
    }
  }
}

int sv_wave_bwd_launch(const WaveBwdArgs& a, hipStream_t stream) {
  constexpr int NL = 12;
  constexpr size_t lds = (size_t)2 * 4 * 32 * 36 * 4 + (size_t)32 * 136 * 2 + (size_t)128 * 40 * 2 + (size_t)32 * 256 +
                         (size_t)32 * 32 * 4 + (size_t)4 * NL * 1024;
  hipLaunchKernelGGL((lstm_wave_bwd_bf16_kernel<48, 8, NL>), dim3(WB_L * a.nub * a.nrb), dim3(256), lds, stream, a);
  return (int)hipGetLastError();
}
