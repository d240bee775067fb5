// Shared device helpers for the gfx950 (CDNA4) GE2E speaker-embedding kernels.
// Wave = 64 lanes; MFMA accumulator layout of the 32x32 family (dtype independent on
// gfx950): acc reg r of lane l holds C[row = (r&3) + 8*(r>>2) + 4*(l>>5)][col = l&31].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define SV_WAVE 64

// return codes of the C ABI (0 = OK, > 0 = hipError_t, < 0 = argument error)
#define SV_OK 0
#define SV_EARG -1
#define SV_EALIGN -2
#define SV_ESHAPE -3

// fp32 GEMM of the C ABI's sv_gemm_f32 (include/sv_ge2e.h) under the calling thread's current
// product mode; F32ProductScope sets that mode for one entry point's duration
// fine: split K in chunks down to 128 when the tiles leave most of the chip idle (the projection's
// GEMMs; their workspace comes from sv_gemm_f32_workspace, which covers both plans)
int gemm_f32(int a_kcontig, int b_kcontig, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
             float* C, long ldc, const float* bias0, const float* bias1, float beta, float* workspace,
             hipStream_t stream, bool fine = false);
// the projection forward with the row norm fused into the split-K reduce (sv_lstm.hip); returns 0
// where that form does not apply (the caller then runs gemm_f32 and its own norm)
int proj_norm_fused(const float* h, int B, int K, int P, const float* W, const float* bias, float* y, float* emb,
                    float* ynorm, float* workspace, hipStream_t stream, int* rc);
struct F32ProductScope {
  int prev;
  explicit F32ProductScope(int mode);
  ~F32ProductScope();
};

// fp32 W-stationary persistent recurrences of one layer (sv_persist_f32.hip): H = 768, 64-row x
// 32-unit tiles co-resident on `cus` CUs; dgf: sv_persist_f32_bwd_scratch bytes (16-B aligned)
int sv_persist_f32_fits(int B, int H, int cus);
int sv_stream_cus(hipStream_t stream);  // CUs of the stream's device (sv_persist.hip)
// zero `words` arrival-counter words in each of `nchan` channels (channel c at cnt + c * chan_stride)
// with ONE kernel on `stream` (sv_persist.hip).  Never hipMemsetAsync for the counters: replayed
// from a HIP graph, a memset node's reset was not reliably seen by the persistent kernel's
// agent-scope atomics and polls (scripts/f32_replay_diag.py)
int sv_zero_counters(unsigned* cnt, int nchan, long chan_stride, int words, hipStream_t stream);
// zero `bytes` bytes at p with a kernel on `stream` (0 or a hipError_t).  Used for every zeroing
// in the library instead of hipMemsetAsync: replayed from a HIP graph, memset nodes left junk
// behind (the initial-state slots and the arrival counters; scripts/f32_replay_diag.py)
int sv_zero_bytes(void* p, size_t bytes, hipStream_t stream);
// up to SV_ZB_MAX zeroings in one launch (n buffers of bytes[i] bytes each)
#define SV_ZB_MAX 12
int sv_zero_bytes_multi(int n, void* const* ptrs, const size_t* bytes, hipStream_t stream);
inline hipError_t sv_memset0(void* p, size_t bytes, hipStream_t stream) {
  return (hipError_t)sv_zero_bytes(p, bytes, stream);
}
size_t sv_persist_f32_bwd_scratch(int T, int B, int H);
// x_tm (may be NULL): layer 0's input [T,B,F] (F = 40): the input projection x W_ih^T + b_ih + b_hh
// is formed inside the recurrence (no K1 GEMM; `gates` is then output only)
int sv_persist_fwd_f32(int T, int B, int H, const float* whh, float* gates, float* c_tm, float* h_tm, float* hT,
                       hipStream_t stream, unsigned* sync, int chan, hipEvent_t pre, hipEvent_t post,
                       const float* x_tm = nullptr, int F = 0, const float* wih = nullptr,
                       const float* b_ih = nullptr, const float* b_hh = nullptr);
int sv_persist_bwd_f32(int T, int B, int H, const float* whhT, const float* acts, const float* c_tm,
                       const float* dhup, int up_full, float* dg, float* dgT, float* dgf, hipStream_t stream,
                       unsigned* sync, hipEvent_t pre, hipEvent_t post, float* db_ih = nullptr,
                       float* db_hh = nullptr);
// db_ih (= db_hh when given) = sum over nrb row blocks, in order, of the partials dbp [nrb][G]
int sv_persist_db_finalize(const float* dbp, int nrb, int G, float* db_ih, float* db_hh, hipStream_t stream);
#define SV_LAUNCH_CHECK()                                  \
  do {                                                     \
    hipError_t e__ = hipGetLastError();                    \
    if (e__ != hipSuccess) return (int)e__;                \
  } while (0)

// The fp32 path's LSTM cell activations (every fp32 cell: per-step K2 / K3 and the persistent
// recurrences, so the schedules stay bit-identical).  v_exp_f32 + v_rcp_f32 forms: the libm tanhf
// and an IEEE divide made the persistent forward's cell phase 5.1k cycles per step (of 62.6k;
// stamps).  Error: sigmoid a few fp32 ulps; tanh within ~1e-7 absolute (the
// 1 - e cancellation near 0), far inside the fp32 path's tolerances (north_star: 1e-4 on the loss).
__device__ __forceinline__ float sv_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float sv_tanh(float x) {
  const float e = __expf(-2.0f * fabsf(x));  // (0, 1]
  return copysignf((1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e), x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// sum over aligned groups of GL = 8 or 16 lanes (xor 1, xor 2, then the half-row mirror and, for
// 16, the row mirror: each step pairs lanes of the two halves of the previous span), every lane of
// the group getting the same sum; VALU only -- no LDS crossbar traffic
template <int GL>
__device__ __forceinline__ float dpp_group_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  if constexpr (GL == 16)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// whole-wave sum / max: the 16-lane DPP steps, then the four row results read into SGPRs (the
// result is wave-uniform); no LDS crossbar round trips, unlike the __shfl_xor butterfly
__device__ __forceinline__ float dpp_row16_max(float v) {
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)));
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = dpp_group_sum<16>(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = dpp_row16_max(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// f32 -> bf16 bits, round-to-nearest-even (inputs are finite activations/weights)
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x32x16bf(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
