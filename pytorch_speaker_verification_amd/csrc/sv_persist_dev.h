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
__device__ __forceinline__ void persist_tile(int xcd, int nub, int& ub, int& rb) {
  const int i = blockIdx.x, n = gridDim.x;
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

