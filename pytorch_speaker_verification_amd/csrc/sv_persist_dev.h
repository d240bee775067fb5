// Device helpers shared by the persistent-recurrence kernels (sv_persist.hip, sv_persist3.hip).
#pragma once
#include "sv_bf16.h"

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;


__device__ __forceinline__ __amdgpu_buffer_rsrc_t sv_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

// Tile order of the W-stationary kernels (1-D grid of nub x nrb workgroups).  Workgroup i is
// dispatched to XCD i % 8; with xcd = 1 each XCD gets a contiguous range of logical tiles, so
// the workgroups that share a row block (and read the same handed-off rows) sit mostly on one
// XCD and the second and later readers hit that XCD's L2 instead of the fabric.
// ncomp: the compute workgroups (blocks past them, if any, are helper workgroups)
__device__ __forceinline__ void persist_tile(int xcd, int nub, int& ub, int& rb, int ncomp = 0) {
  const int i = blockIdx.x, n = ncomp ? ncomp : gridDim.x;
  int L = i;
  if (xcd) {
    const int x = i & 7, q = n >> 3, r = n & 7;
    L = x * q + min(x, r) + (i >> 3);
  }
  ub = L % nub;
  rb = L / nub;
}

// lane 0 of the workgroup: wait until *c >= target.  Bounded: after `limit` polls the wait sets
// `code` in the sync block's status word and returns; once the status is nonzero every wait on
// the block returns at once, so a broken launch drains instead of hanging the GPU.
__device__ __forceinline__ void persist_wait(unsigned* c, unsigned target, unsigned* status, unsigned limit,
                                             unsigned code) {
  unsigned spins = 0;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    __builtin_amdgcn_s_sleep(2);
    if (++spins > limit) {
      __hip_atomic_fetch_or(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
}
// test-only fault injection (SV_PERSIST_FAULT=1, read by the host): workgroup 0 withholds its
// first arrival, so its row block's consumers time out (short spin limit) and the status is set
__device__ __forceinline__ bool persist_arrive_ok(int fault, int first) { return !(fault && first && blockIdx.x == 0); }

// LDS-DMA image of one 32-row x H bf16 tile (H = 768; sv_wave.hip's wave3 forward and
// sv_persist3.hip's wide forward), two regions:
//   A: units [0, 512) as 32 rows of 1024 B + 16 B pad (a 1040-B row stride);
//   B: units [512, 768) as 32 rows of 512 B, unpadded, the 16-B chunk c of row r at slot
//      c ^ (r & 15) (an XOR swizzle in place of a pad: one DMA instruction fills two whole rows).
// Fragment reads (lanes 0-15 = rows 0-15 at one k offset) are conflict-free in both; every DMA
// instruction reads whole 128-B lines (one 1 KB row piece, or two 512-B ones).
constexpr int W3_RA = 1040, W3_RB = 512;
constexpr int W3_TILE = 32 * (W3_RA + W3_RB);
constexpr int W3_DMA = 12;  // DMA instructions per wave per tile (8 A + 4 B)

// stage a 32-row tile of slot `ts` of `ra` (a [T+1][B][H] bf16 buffer, H = 768; the descriptor is
// built once, outside the time loop, so it stays scalar): wave w stages rows 8 w .. 8 w + 7; rows
// past B read zeros.  The wave index goes through an opaque SGPR copy: the 24 per-instruction
// addresses are not hoisted out of the time loop (held live across it they pushed weight fragments
// into scratch) yet stay scalar -- a row's base is SALU arithmetic passed as soffset (region A) or
// one select per lane (region B) -- where an opaque VGPR zero made every address a VALU chain with
// a quarter-rate v_mul_lo_u32 and a v_readfirstlane for M0
struct W3Dma {
  __amdgpu_buffer_rsrc_t ra;
  unsigned slot, vl, xs, h2;
  int B, H, b0, g;
  char* tile;
  __device__ __forceinline__ W3Dma(__amdgpu_buffer_rsrc_t ra_, int ts, int B_, int H_, int b0_, char* tile_, int g_,
                                   int lane)
      : ra(ra_), B(B_), H(H_), b0(b0_), tile(tile_) {
    int gz = __builtin_amdgcn_readfirstlane(g_);  // (wave-uniform)
    asm volatile("" : "+s"(gz));
    g = gz;
    slot = (unsigned)ts * (unsigned)B * (unsigned)H * 2u;
    vl = 16u * (unsigned)lane;
    const unsigned hh = (unsigned)lane >> 5;
    xs = ((unsigned)lane & 31u) ^ hh;  // (sl ^ ((2 p + hh) & 15)) = xs ^ (2 p & 14)
    h2 = hh;
  }
  __device__ __forceinline__ unsigned row_base(int row) const {
    return b0 + row < B ? slot + (unsigned)(b0 + row) * (unsigned)H * 2u : 0xFFFFE000u;
  }
  __device__ __forceinline__ void piece(int i) const {
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    if (i < 8) {  // region A: row g 8 + i, one 1-KB row per instruction
      const int row = g * 8 + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(tile + row * W3_RA), 16, vl, row_base(row), 0,
                                               16 /* sc1 */);
    } else {  // region B: rows 2 p, 2 p + 1 (lane halves), 512 B each, chunk c at c ^ (row & 15)
      const int p = g * 4 + (i - 8);
      const unsigned r0 = row_base(2 * p), r1 = row_base(2 * p + 1);
      const unsigned c = 64u + (xs ^ (unsigned)((2 * p) & 14));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(tile + 32 * W3_RA + p * 1024), 16,
                                               (h2 ? r1 : r0) + 16u * c, 0, 0, 16 /* sc1 */);
    }
  }
};
__device__ __forceinline__ void w3_dma(__amdgpu_buffer_rsrc_t ra, int ts, int B, int H, int b0, char* tile, int g,
                                       int lane) {
  const W3Dma d(ra, ts, B, H, b0, tile, g, lane);
#pragma unroll
  for (int i = 0; i < W3_DMA; ++i) d.piece(i);
}

// piece i (0 .. W3_DMA - 1) of w3_dma alone (the same addresses), for issue spread over a k-loop
__device__ __forceinline__ void w3_dma_piece(__amdgpu_buffer_rsrc_t ra, int ts, int B, int H, int b0, char* tile, int g,
                                             int lane, int i) {
  W3Dma(ra, ts, B, H, b0, tile, g, lane).piece(i);
}

// byte offset of A fragment s (k-step, 16 bf16) of lane (r, hh) in a w3_dma tile image
struct W3Frag {
  const char* pa;
  const char* pb;
  unsigned fb;
  __device__ __forceinline__ W3Frag(const char* tile, int lane) {
    const int r = lane & 31, hh = lane >> 5;
    pa = tile + r * W3_RA + hh * 16;
    fb = (unsigned)(((r & 15) ^ hh) << 4);
    pb = tile + 32 * W3_RA + r * W3_RB;
  }
  __device__ __forceinline__ bf16x8_t operator()(int s) const {
    if (s < 32) return *reinterpret_cast<const bf16x8_t*>(pa + 32 * s);
    return *reinterpret_cast<const bf16x8_t*>(pb + ((unsigned)(32 * (s - 32)) ^ fb));
  }
};

// The logical tiles [l0, l1) that persist_tile (xcd = 1) gives the blocks of XCD group x (blocks
// b with b % 8 == x) of an n-block grid
__device__ __forceinline__ void persist_xcd_tiles(int x, int n, int& l0, int& l1) {
  const int q = n >> 3, r = n & 7;
  l0 = x * q + min(x, r);
  l1 = l0 + q + (x < r ? 1 : 0);
}

// Operand prefetch by the helper workgroups of a persistent grid (blocks ncomp .. ncomp + npf - 1,
// npf a multiple of 8, so every XCD group gets npf / 8 of them): pull 16-B pieces of the bytes the
// XCD group's compute workgroups will DMA a few steps later into that XCD's L2 (and the
// Infinity Cache) by LDS-DMA into a scratch LDS slot -- no registers, no waits on the compute
// waves' in-order vmcnt.  Speed only: nothing reads the scratch slot, and a prefetch that comes
// late (or never) changes no result.
__device__ __forceinline__ void persist_prefetch16(const void* p, char* lds_scratch) {
  typedef __attribute__((address_space(1))) void* glb_ptr_t;
  __builtin_amdgcn_global_load_lds((glb_ptr_t)p, (lds_ptr_t)lds_scratch, 16, 0, 0);
}
