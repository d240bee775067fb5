// Projection + L2 normalisation (speech_embedder_net.py:30-32, SURVEY §8 a-C) and the
// fused gradient-clip + SGD update (train_speech_embedder.py:63-65, SURVEY §8 a-I).
#include <algorithm>
#include "sv_common.h"
#include "sv_gemm.h"
#include "../../include/sv_ge2e.h"

// emb = y / |y|_2 (torch.norm, no eps).  One wave per row.
__global__ __launch_bounds__(256) void rownorm_fwd_kernel(const float* __restrict__ y, int B, int P,
                                                          float* __restrict__ emb, float* __restrict__ ynorm) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= B) return;
  const float* yr = y + (long)r * P;
  float ss = 0.f;
  for (int p = lane; p < P; p += 64) ss += yr[p] * yr[p];
  const float n = sqrtf(wave_sum(ss));
  const float inv = 1.0f / n;
  for (int p = lane; p < P; p += 64) emb[(long)r * P + p] = yr[p] * inv;
  if (lane == 0) ynorm[r] = n;
}

// dy = (de - e <e, de>) / |y|
__global__ __launch_bounds__(256) void rownorm_bwd_kernel(const float* __restrict__ demb, const float* __restrict__ emb,
                                                          const float* __restrict__ ynorm, int B, int P,
                                                          float* __restrict__ dy) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= B) return;
  const float* de = demb + (long)r * P;
  const float* e = emb + (long)r * P;
  float dot = 0.f;
  for (int p = lane; p < P; p += 64) dot += e[p] * de[p];
  dot = wave_sum(dot);
  const float inv = 1.0f / ynorm[r];
  for (int p = lane; p < P; p += 64) dy[(long)r * P + p] = (de[p] - e[p] * dot) * inv;
}

// ---- the projection backward in one launch (P <= 256, H % 4 == 0, B <= 128) ----
// The GEMM path takes 5 launches after the row-norm backward (the dWp GEMM, a two-level column
// sum, the dh GEMM, their slab reduce); at the rank shapes each is a ~5 us latency-bound launch
// (r06 c4 rank timeline: 27 us for the five).  Here ONE launch: workgroups of PJ_R rows x 64
// columns of H form dh = dy Wp (K = P, Wp rows read coalesced), workgroups of 8 rows of P x 64
// columns form dWp = dy^T h (K = B, h rows read coalesced), those of column block 0 also
// db = colsum(dy); dy's slice staged in LDS, each of the 4 waves a quarter of K, PJ_U loads in
// flight per lane.  Exact fp32 products, fp32 accumulation in a fixed
// order (another order than the MFMA GEMMs': results agree to fp32 rounding).  Measured (traces):
// c4 rank (B = 80) 18-20 us against 27; c5 rank (B = 320) 59 us against 39 -- its K = B loop
// grows with the batch while the GEMM path's does not, hence B <= 128.  Since r06 the MFMA-tile
// kernel below is faster at every B; this one serves unaligned operands.
#define PJ_R 4
#define PJ_U 32  // loads in flight per thread
__global__ __launch_bounds__(256) void proj_bwd_small_kernel(const float* __restrict__ dy, const float* __restrict__ h,
                                                             int B, int H, int P, const float* __restrict__ W,
                                                             float* __restrict__ dW, float* __restrict__ db,
                                                             float* __restrict__ dh, int ndh) {
  // workgroup = 64 columns of H (lane = column) x 4 waves, each wave one quarter of the reduction
  // dimension; the waves' partials added through LDS in wave order (fixed summation order)
  extern __shared__ float sm[];  // staged dy slice, then [4 waves][8][64] partials
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ncb = (H + 63) / 64;
  if ((int)blockIdx.x < ndh) {  // dh[r][c] = sum_p dy[r][p] W[p][c], r in [r0, r0 + PJ_R)
    const int r0 = (blockIdx.x / ncb) * PJ_R, c = (blockIdx.x % ncb) * 64 + lane;
    float* part = sm + PJ_R * P;
    {  // PJ_R * P <= 1024: four predicated loads per thread in flight at once
      float v[PJ_R];
#pragma unroll
      for (int k = 0; k < PJ_R; ++k) {
        const int i = tid + 256 * k;
        v[k] = (i < PJ_R * P && r0 + i / P < B) ? dy[(long)r0 * P + i] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < PJ_R; ++k)
        if (tid + 256 * k < PJ_R * P) sm[tid + 256 * k] = v[k];
    }
    __syncthreads();
    const int q = (P + 3) / 4, pa = wv * q, pe = min(P, pa + q);
    float acc[PJ_R];
#pragma unroll
    for (int r = 0; r < PJ_R; ++r) acc[r] = 0.f;
    for (int p0 = pa; p0 < pe; p0 += PJ_U) {
      float wv_[PJ_U];
#pragma unroll
      for (int u = 0; u < PJ_U; ++u) wv_[u] = (p0 + u < pe && c < H) ? W[(long)(p0 + u) * H + c] : 0.f;
#pragma unroll
      for (int u = 0; u < PJ_U; ++u)
#pragma unroll
        for (int r = 0; r < PJ_R; ++r) acc[r] = fmaf(p0 + u < pe ? sm[r * P + p0 + u] : 0.f, wv_[u], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < PJ_R; ++r) part[(wv * PJ_R + r) * 64 + lane] = acc[r];
    __syncthreads();
    if (tid < PJ_R * 64) {
      const int r = tid >> 6;
      const float v = part[(0 * PJ_R + r) * 64 + lane] + part[(1 * PJ_R + r) * 64 + lane] +
                      part[(2 * PJ_R + r) * 64 + lane] + part[(3 * PJ_R + r) * 64 + lane];
      if (r0 + r < B && c < H) dh[(long)(r0 + r) * H + c] = v;
    }
    return;
  }
  // dW[p][c] = sum_b dy[b][p] h[b][c], p in [p0, p0 + 8); db[p] = sum_b dy[b][p] (column block 0)
  const int j = blockIdx.x - ndh, p0 = (j / ncb) * 8, c = (j % ncb) * 64 + lane;
  float* part = sm + B * 8;
  for (int i0 = 0; i0 < B * 8; i0 += 256 * 8) {  // 8 predicated loads per thread in flight at once
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + tid + 256 * k;
      v[k] = (i < B * 8 && p0 + (i & 7) < P) ? dy[(long)(i >> 3) * P + p0 + (i & 7)] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i0 + tid + 256 * k < B * 8) sm[i0 + tid + 256 * k] = v[k];
  }
  __syncthreads();
  if (j % ncb == 0 && tid < 8 && p0 + tid < P) {
    float s_ = 0.f;
    for (int b = 0; b < B; ++b) s_ += sm[b * 8 + tid];
    db[p0 + tid] = s_;
  }
  const int q = (B + 3) / 4, ba = wv * q, be = min(B, ba + q);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  for (int b0 = ba; b0 < be; b0 += PJ_U) {
    float hv[PJ_U];
#pragma unroll
    for (int u = 0; u < PJ_U; ++u) hv[u] = (b0 + u < be && c < H) ? h[(long)(b0 + u) * H + c] : 0.f;
#pragma unroll
    for (int u = 0; u < PJ_U; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = fmaf(b0 + u < be ? sm[(b0 + u) * 8 + k] : 0.f, hv[u], acc[k]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[(wv * 8 + k) * 64 + lane] = acc[k];
  __syncthreads();
  for (int k = wv; k < 8; k += 4) {
    const float v = part[(0 * 8 + k) * 64 + lane] + part[(1 * 8 + k) * 64 + lane] + part[(2 * 8 + k) * 64 + lane] +
                    part[(3 * 8 + k) * 64 + lane];
    if (p0 + k < P && c < H) dW[(long)(p0 + k) * H + c] = v;
  }
}
// ---- the projection backward in one launch (16-B aligned operands, any B: every config) ----
// The GEMM path's 6 launches (the dWp GEMM + its split-K reduce, a two-level column sum, the dh
// GEMM + reduce) cost ~37 us at B = 640 for ~0.5 GFLOP.  Here one launch: 64 x 64 tiles of
// dWp = dy^T h (K = B) and of dh = dy Wp (K = P) on the fp32 MFMA main loop (sv_gemm.h; exact fp32
// products, one accumulator over K), and db = colsum(dy) in PB_DBW workgroups of 64 columns x 4
// row quarters (PB_U loads in flight per thread, the quarters added in order).
#define PB_DBW_COLS 64
#define PB_U 16
__global__ __launch_bounds__(256) void proj_bwd_tiles_kernel(const float* __restrict__ dy, const float* __restrict__ h,
                                                             int B, int H, int P, const float* __restrict__ W,
                                                             float* __restrict__ dW, float* __restrict__ db,
                                                             float* __restrict__ dh, int ndw, int ndh) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles_h = (H + 63) / 64;
  const int wm0 = (w >> 1) * 32, wn0 = (w & 1) * 32;
  int id = blockIdx.x;
  if (id < ndw + ndh) {
    const bool isdw = id < ndw;
    if (!isdw) id -= ndw;
    const int tm = id / tiles_h, tn = id % tiles_h;
    f32x16 acc[1][1];
    zero_acc(acc);
    const int M = isdw ? P : B;
    if (isdw)  // A = dy as [K = B][M = P], B = h as [K = B][N = H]
      gemm_mainloop<64, 64, 256, false, false, 1, 1>(dy, P, RowMapLinear{tm * 64, P}, h, H, RowMapLinear{tn * 64, H}, 0,
                                                     B, lds, tid, wm0, wn0, acc);
    else       // A = dy [M = B][K = P] k-contiguous, B = Wp as [K = P][N = H]
      gemm_mainloop<64, 64, 256, true, false, 1, 1>(dy, P, RowMapLinear{tm * 64, B}, W, H, RowMapLinear{tn * 64, H}, 0,
                                                    P, lds, tid, wm0, wn0, acc);
    float* C = isdw ? dW : dh;
    const int col = tn * 64 + wn0 + (lane & 31);
    if (col < H) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tm * 64 + wm0 + acc_row(r, lane);
        if (row < M) C[(long)row * H + col] = acc[0][0][r];
      }
    }
    return;
  }
  // db[c] = sum_b dy[b][c]: lane = column, wave = row quarter
  const int c = (id - ndw - ndh) * PB_DBW_COLS + lane;
  const int q = (B + 3) / 4, ba = w * q, be = min(B, ba + q);
  float s_ = 0.f;
  for (int b0 = ba; b0 < be; b0 += PB_U) {
    float v[PB_U];
#pragma unroll
    for (int u = 0; u < PB_U; ++u) v[u] = (b0 + u < be && c < P) ? dy[(long)(b0 + u) * P + c] : 0.f;
#pragma unroll
    for (int u = 0; u < PB_U; ++u) s_ += v[u];
  }
  lds[w * 64 + lane] = s_;
  __syncthreads();
  if (w == 0 && c < P) db[c] = lds[lane] + lds[64 + lane] + lds[128 + lane] + lds[192 + lane];
}
static bool proj_tiles_ok(int B, int H, int P, const void* h, const void* W, const void* dy) {
  return H % 4 == 0 && P % 4 == 0 && !(((uintptr_t)h | (uintptr_t)W | (uintptr_t)dy) & 15);
}

static bool proj_small_ok(int B, int H, int P, const void* h, const void* W) {
  return P <= 256 && H % 4 == 0 && B <= 128 && !(((uintptr_t)h | (uintptr_t)W) & 15);
}

extern "C" size_t sv_proj_norm_workspace(int B, int H, int P) {
  size_t g = std::max(sv_gemm_f32_workspace(B, P, H), std::max(sv_gemm_f32_workspace(P, H, B), sv_gemm_f32_workspace(B, H, P)));
  g = std::max(g, sv_colsum_workspace(B, P));
  return ((size_t)B * P * sizeof(float) + 255) / 256 * 256 + g;
}

extern "C" int sv_proj_norm_fwd(const float* h_last, int B, int H, int P, const float* w_p, const float* b_p, float* y,
                                float* emb, float* ynorm, float* workspace, hipStream_t stream) {
  if (!h_last || !w_p || !y || !emb || !ynorm || B <= 0 || H <= 0 || P <= 0) return SV_EARG;
  int rc;
  if (proj_norm_fused(h_last, B, H, P, w_p, b_p, y, emb, ynorm, workspace, stream, &rc)) return rc;
  rc = gemm_f32(1, 1, B, P, H, h_last, H, w_p, H, y, P, b_p, nullptr, 0.f, workspace, stream, true);
  if (rc) return rc;
  hipLaunchKernelGGL(rownorm_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, y, B, P, emb, ynorm);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_proj_norm_bwd(const float* demb, const float* emb, const float* ynorm, const float* h_last, int B,
                                int H, int P, const float* w_p, float* dw_p, float* db_p, float* dh_last,
                                float* workspace, hipStream_t stream) {
  if (!demb || !emb || !ynorm || !h_last || !w_p || !dw_p || !db_p || !dh_last || !workspace) return SV_EARG;
  float* dy = workspace;
  float* gws = workspace + ((size_t)B * P * sizeof(float) + 255) / 256 * 64;
  hipLaunchKernelGGL(rownorm_bwd_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, demb, emb, ynorm, B, P, dy);
  SV_LAUNCH_CHECK();
  if (proj_small_ok(B, H, P, h_last, w_p) && !proj_tiles_ok(B, H, P, h_last, w_p, dy)) {
    const int ncb = (H + 63) / 64, ndh = (B + PJ_R - 1) / PJ_R * ncb, ndw = (P + 7) / 8 * ncb;
    const size_t lds = std::max((size_t)PJ_R * P + 4 * PJ_R * 64, (size_t)B * 8 + 4 * 8 * 64) * sizeof(float);
    hipLaunchKernelGGL(proj_bwd_small_kernel, dim3(ndh + ndw), dim3(256), lds, stream, dy, h_last, B, H, P, w_p, dw_p,
                       db_p, dh_last, ndh);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  if (proj_tiles_ok(B, H, P, h_last, w_p, dy)) {
    const int th = (H + 63) / 64, ndw = (P + 63) / 64 * th, ndh = (B + 63) / 64 * th;
    const int ndb = (P + PB_DBW_COLS - 1) / PB_DBW_COLS;
    constexpr size_t lds = 2 * SV_BK * (TileLd<false, 64>::value + TileLd<false, 64>::value) * sizeof(float);
    static_assert(2 * SV_BK * (TileLd<true, 64>::value + TileLd<false, 64>::value) * sizeof(float) <= lds, "lds");
    hipLaunchKernelGGL(proj_bwd_tiles_kernel, dim3(ndw + ndh + ndb), dim3(256), lds, stream, dy, h_last, B, H, P, w_p,
                       dw_p, db_p, dh_last, ndw, ndh);
    SV_LAUNCH_CHECK();
    return SV_OK;
  }
  // dWp [P,H] = dy^T h_last  (A = dy as [K=B][M=P], B = h_last as [K=B][N=H])
  int rc = gemm_f32(0, 0, P, H, B, dy, P, h_last, H, dw_p, H, nullptr, nullptr, 0.f, gws, stream, true);
  if (rc) return rc;
  rc = sv_colsum(dy, B, P, db_p, gws, stream);
  if (rc) return rc;
  // dh_last [B,H] = dy Wp  (A = dy [B, K=P] k-contig, B = Wp as [K=P][N=H])
  return gemm_f32(1, 0, B, H, P, dy, P, w_p, H, dh_last, H, nullptr, nullptr, 0.f, gws, stream, true);
}

// ---------------------------------------------------------------------------
// fused clip_grad_norm_(max_norm) + SGD(lr) over one flat parameter group.
// pass 1: per-block partial sums of squares (fixed grid, fixed order)
#define CLIP_BLOCKS 512
// One group = one parameter group of the reference; the two-group launches (sv_clip_sgd_step2)
// give group 1 the blocks after group 0's, each group's blocks doing exactly what they do alone.
struct ClipGroup {
  float* p;
  float* g;
  long n;
  float max_norm;
  int blocks;   // this group's grid (the single-group formula of sv_clip_sgd_step)
  int first;    // its first block in the launch
};
__device__ __forceinline__ void sqsum_partial_body(const float* __restrict__ g, long n, int bid, int nb,
                                                   float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  const long n4 = n / 4;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  for (long i = bid * 256L + threadIdx.x; i < n4; i += (long)nb * 256) {
    const f32x4 v = g4[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + bid * 256L + threadIdx.x; i < n; i += (long)nb * 256) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[bid] = red[0] + red[1] + red[2] + red[3];
}
__global__ __launch_bounds__(256) void sqsum_partial_kernel(const float* __restrict__ g, long n,
                                                            float* __restrict__ partial) {
  sqsum_partial_body(g, n, blockIdx.x, gridDim.x, partial);
}
__global__ __launch_bounds__(256) void sqsum_partial2_kernel(ClipGroup g0, ClipGroup g1, float* __restrict__ partial) {
  const bool one = (int)blockIdx.x >= g1.first;
  const ClipGroup& c = one ? g1 : g0;
  sqsum_partial_body(c.g, c.n, blockIdx.x - c.first, c.blocks, partial + (one ? CLIP_BLOCKS : 0));
}

// pass 2: every block re-reduces the partials (fixed order, fp64), computes
// coef = min(1, max_norm / (|g| + 1e-6)) and updates p -= lr * coef * g (optionally g *= coef).
// status (optional, a persistent-recurrence sync block's status word): nonzero -> the gradients
// came from a timed-out recurrence: no update at all (parameters and gradients untouched).
__device__ __forceinline__ void clip_sgd_body(float* __restrict__ p, float* __restrict__ g, long n, int bid, int nb,
                                              const float* __restrict__ partial, int npart, float max_norm, float lr,
                                              int write_grad, float* __restrict__ norm_out,
                                              const unsigned* __restrict__ status) {
  if (status && *status) {
    if (norm_out && bid == 0 && threadIdx.x == 0) norm_out[0] = __builtin_nanf("");
    return;
  }
  __shared__ double redd[4];
  __shared__ float coef_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < npart; i += 256) s += (double)partial[i];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) redd[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(redd[0] + redd[1] + redd[2] + redd[3]);
    const float c = max_norm / (total + 1e-6f);
    coef_s = c < 1.0f ? c : 1.0f;
    if (norm_out && bid == 0) norm_out[0] = total;
  }
  __syncthreads();
  const float k = coef_s;
  const float step = lr * k;
  const long n4 = n / 4;
  f32x4* p4 = reinterpret_cast<f32x4*>(p);
  f32x4* g4 = reinterpret_cast<f32x4*>(g);
  for (long i = bid * 256L + threadIdx.x; i < n4; i += (long)nb * 256) {
    const f32x4 gv = g4[i];
    p4[i] = p4[i] - step * gv;
    if (write_grad) g4[i] = gv * k;
  }
  for (long i = n4 * 4 + bid * 256L + threadIdx.x; i < n; i += (long)nb * 256) {
    const float gv = g[i];
    p[i] -= step * gv;
    if (write_grad) g[i] = gv * k;
  }
}
__global__ __launch_bounds__(256) void clip_sgd_kernel(float* __restrict__ p, float* __restrict__ g, long n,
                                                       const float* __restrict__ partial, int npart, float max_norm,
                                                       float lr, int write_grad, float* __restrict__ norm_out,
                                                       const unsigned* __restrict__ status) {
  clip_sgd_body(p, g, n, blockIdx.x, gridDim.x, partial, npart, max_norm, lr, write_grad, norm_out, status);
}
// the training step's status report (sv_status_report's kernel) folded into the update launch
// (ABI v11, sv_clip_sgd_step2_report): workgroup 0 poisons x[0..n) when the status is set and
// stores (seq << 32) | status into the pinned host slot (slot null: no report)
struct ClipReport {
  float* x;
  int n;
  unsigned long long* slot;
  unsigned seq;
};
__global__ __launch_bounds__(256) void clip_sgd2_kernel(ClipGroup g0, ClipGroup g1, const float* __restrict__ partial,
                                                        float lr, int write_grad, float* __restrict__ norm_out,
                                                        const unsigned* __restrict__ status, const ClipReport rep) {
  if (rep.slot && blockIdx.x == 0) {
    const unsigned st = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = threadIdx.x; i < rep.n && st; i += blockDim.x) rep.x[i] = __builtin_nanf("");
    if (threadIdx.x == 0)
      __hip_atomic_store(rep.slot, ((unsigned long long)rep.seq << 32) | st, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const bool one = (int)blockIdx.x >= g1.first;
  const ClipGroup& c = one ? g1 : g0;
  clip_sgd_body(c.p, c.g, c.n, blockIdx.x - c.first, c.blocks, partial + (one ? CLIP_BLOCKS : 0), c.blocks,
                c.max_norm, lr, write_grad, norm_out ? norm_out + (one ? 1 : 0) : nullptr, status);
}

extern "C" size_t sv_clip_sgd_workspace(void) { return CLIP_BLOCKS * sizeof(float); }

extern "C" int sv_clip_sgd_step(float* params, float* grads, long n, float max_norm, float lr, int write_grad,
                                float* total_norm_out, const void* sync, float* workspace, hipStream_t stream) {
  if (!params || !grads || !workspace || n <= 0) return SV_EARG;
  if (((uintptr_t)params | (uintptr_t)grads) & 15) return SV_EALIGN;
  const int blocks = (int)std::min<long>(CLIP_BLOCKS, (n / 4 + 255) / 256 + 1);
  hipLaunchKernelGGL(sqsum_partial_kernel, dim3(blocks), dim3(256), 0, stream, grads, n, workspace);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(clip_sgd_kernel, dim3(blocks), dim3(256), 0, stream, params, grads, n, workspace, blocks, max_norm,
                     lr, write_grad, total_norm_out, reinterpret_cast<const unsigned*>(sync));
  SV_LAUNCH_CHECK();
  return SV_OK;
}

static int clip_sgd_step2(float* params0, float* grads0, long n0, float max_norm0, float* params1, float* grads1,
                          long n1, float max_norm1, float lr, int write_grad, float* total_norm_out, const void* sync,
                          float* workspace, hipStream_t stream, const ClipReport& rep);
extern "C" int sv_clip_sgd_step2(float* params0, float* grads0, long n0, float max_norm0, float* params1,
                                 float* grads1, long n1, float max_norm1, float lr, int write_grad,
                                 float* total_norm_out, const void* sync, float* workspace, hipStream_t stream) {
  return clip_sgd_step2(params0, grads0, n0, max_norm0, params1, grads1, n1, max_norm1, lr, write_grad, total_norm_out,
                        sync, workspace, stream, ClipReport{nullptr, 0, nullptr, 0});
}
extern "C" int sv_clip_sgd_step2_report(float* params0, float* grads0, long n0, float max_norm0, float* params1,
                                        float* grads1, long n1, float max_norm1, float lr, int write_grad,
                                        float* total_norm_out, const void* sync, float* workspace,
                                        float* report_x, int report_n, void* host_slot_dev, unsigned seq,
                                        hipStream_t stream) {
  if (!sync || !host_slot_dev || report_n < 0 || (report_n > 0 && !report_x) || ((uintptr_t)host_slot_dev & 7))
    return SV_EARG;
  return clip_sgd_step2(params0, grads0, n0, max_norm0, params1, grads1, n1, max_norm1, lr, write_grad, total_norm_out,
                        sync, workspace, stream,
                        ClipReport{report_x, report_n, reinterpret_cast<unsigned long long*>(host_slot_dev), seq});
}
static int clip_sgd_step2(float* params0, float* grads0, long n0, float max_norm0, float* params1, float* grads1,
                          long n1, float max_norm1, float lr, int write_grad, float* total_norm_out, const void* sync,
                          float* workspace, hipStream_t stream, const ClipReport& rep) {
  if (!params0 || !grads0 || !params1 || !grads1 || !workspace || n0 <= 0 || n1 <= 0) return SV_EARG;
  if (((uintptr_t)params0 | (uintptr_t)grads0 | (uintptr_t)params1 | (uintptr_t)grads1) & 15) return SV_EALIGN;
  ClipGroup g0{params0, grads0, n0, max_norm0, (int)std::min<long>(CLIP_BLOCKS, (n0 / 4 + 255) / 256 + 1), 0};
  ClipGroup g1{params1, grads1, n1, max_norm1, (int)std::min<long>(CLIP_BLOCKS, (n1 / 4 + 255) / 256 + 1), 0};
  g1.first = g0.blocks;
  const int blocks = g0.blocks + g1.blocks;
  hipLaunchKernelGGL(sqsum_partial2_kernel, dim3(blocks), dim3(256), 0, stream, g0, g1, workspace);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(clip_sgd2_kernel, dim3(blocks), dim3(256), 0, stream, g0, g1, workspace, lr, write_grad,
                     total_norm_out, reinterpret_cast<const unsigned*>(sync), rep);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_abi_version(void) { return SV_ABI_VERSION; }
