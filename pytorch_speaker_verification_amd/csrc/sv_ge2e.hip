// GE2E loss (forward + closed-form backward) on gfx950.
//
// Replaces the reference's GE2ELoss.forward (speech_embedder_net.py:43-49) and the ATen
// ops of utils.py:27-132 (get_centroids, get_utterance_centroids, get_cossim, calc_loss)
// plus their autograd backward -- SURVEY §8 rows a-D .. a-G.
//
// Rows r = j*M + i of the local embedding block E[N_local, M, D] belong to speaker
// s0 + j of the N speakers in the (possibly multi-GPU) batch.  Centroids come from the
// speaker sums Ssum[N, D] (all-gathered across ranks in data-parallel runs).
//
//   cos[r, k]   = <E^_r, C^_k>                      (fp32 MFMA GEMM, C^ tiles in LDS)
//   cos[r, s(r)] := <E^_r, U^_r>, U_r = (Ssum_s(r) - E_r) / (M - 1)   (leave-one-out)
//   S = w (cos + 1e-6) + b;  per_r = log(sum_k e^S + 1e-6) - S[r, s(r)];  loss = sum per
// with x^ = x / max(|x|, 1e-8) (torch cosine_similarity).
#include <algorithm>
#include "sv_common.h"
#include "../../include/sv_ge2e.h"

#define EPS_COS 1e-8f
#define EPS_SIM 1e-6f
#define EPS_LOG 1e-6f

namespace {

// workspace carve (all fp32), see sv_ge2e_workspace_size
struct Ge2eWs {
  float *Ehat, *Uhat, *En, *Un, *rawd, *cos, *logz, *Chat, *Cn, *dcos, *alpha, *G1, *dwdb_rows, *betap, *dcd, *gemm;
  size_t total;
};

size_t al(size_t n) { return (n + 63) & ~size_t(63); }  // 256-byte granules

Ge2eWs carve(float* base, int Nl, int M, int D, int N) {
  Ge2eWs w;
  N = (N + 3) & ~3;  // speaker dimension padded to a multiple of 4 (zero rows/cols)
  const size_t Bl = (size_t)Nl * M;
  size_t off = 0;
  auto take = [&](size_t n) {
    float* p = base ? base + off : nullptr;
    off += al(n);
    return p;
  };
  w.Ehat = take(Bl * D);
  w.Uhat = take(Bl * D);
  w.En = take(Bl);
  w.Un = take(Bl);
  w.rawd = take(Bl);
  w.cos = take(Bl * N);
  w.logz = take(Bl);
  w.Chat = take((size_t)N * D);
  w.Cn = take(N);
  w.dcos = take(Bl * N);
  w.alpha = take(Bl);
  w.G1 = take(Bl * D);
  w.dwdb_rows = take(2 * Bl);
  w.betap = take(((Bl + 63) / 64) * (size_t)N);
  w.dcd = take(Bl);
  const size_t g1 = sv_gemm_f32_workspace((int)Bl, D, N);
  const size_t g2 = sv_gemm_f32_workspace(N, D, (int)Bl);
  w.gemm = take((std::max(g1, g2) + 3) / 4);
  w.total = off * sizeof(float);
  return w;
}

}  // namespace

// ---------------------------------------------------------------------------
// K6a: per-speaker sums Ssum[j, :] = sum_i E[j, i, :]  (fixed order i = 0..M-1)
__global__ void ge2e_sums_kernel(const float* __restrict__ E, int M, int D, float* __restrict__ ssum) {
  const int j = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < M; ++i) s += E[((long)j * M + i) * D + d];
    ssum[(long)j * D + d] = s;
  }
}

// block-wide sum (blockDim = 256)
__device__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// K6b: centroids C = Ssum / M (get_centroids, utils.py:27-29), C^ and |C|
__global__ __launch_bounds__(256) void ge2e_centroid_kernel(const float* __restrict__ ssum, int N, int M, int D,
                                                            float* __restrict__ Chat, float* __restrict__ Cn) {
  __shared__ float red[4];
  const int k = blockIdx.x;
  if (k >= N) {  // padding rows of C^ (speaker dim rounded up to 4)
    for (int d = threadIdx.x; d < D; d += 256) Chat[(long)k * D + d] = 0.f;
    if (threadIdx.x == 0) Cn[k] = 0.f;
    return;
  }
  float ss = 0.f;
  for (int d = threadIdx.x; d < D; d += 256) {
    const float c = ssum[(long)k * D + d] / (float)M;
    ss += c * c;
  }
  const float n = sqrtf(block_sum256(ss, red));
  const float inv = 1.0f / fmaxf(n, EPS_COS);
  for (int d = threadIdx.x; d < D; d += 256) Chat[(long)k * D + d] = (ssum[(long)k * D + d] / (float)M) * inv;
  if (threadIdx.x == 0) Cn[k] = n;
}

// K6c: per-row normalisation, leave-one-out centroid and the diagonal cosine.  One wave per row.
__global__ __launch_bounds__(256) void ge2e_rowprep_kernel(const float* __restrict__ E, const float* __restrict__ ssum,
                                                           int Bl, int M, int D, int s0, float* __restrict__ Ehat,
                                                           float* __restrict__ Uhat, float* __restrict__ En,
                                                           float* __restrict__ Un, float* __restrict__ rawd) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int sg = s0 + r / M;
  const float* e = E + (long)r * D;
  const float* s = ssum + (long)sg * D;
  const float invm1 = 1.0f / (float)(M - 1);
  float ee = 0.f, uu = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float x = e[d];
    const float u = (s[d] - x) * invm1;
    ee += x * x;
    uu += u * u;
  }
  const float ne = sqrtf(wave_sum(ee)), nu = sqrtf(wave_sum(uu));
  const float ie = 1.0f / fmaxf(ne, EPS_COS), iu = 1.0f / fmaxf(nu, EPS_COS);
  float dot = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float x = e[d] * ie;
    const float u = ((s[d] - e[d]) * invm1) * iu;
    Ehat[(long)r * D + d] = x;
    Uhat[(long)r * D + d] = u;
    dot += x * u;
  }
  dot = wave_sum(dot);
  if (lane == 0) {
    En[r] = ne;
    Un[r] = nu;
    rawd[r] = dot;
  }
}

// K6d: row softmax-contrast loss.  One wave per row; lanes stride the N speakers.
__global__ __launch_bounds__(256) void ge2e_rowloss_kernel(float* __restrict__ cos, const float* __restrict__ rawd,
                                                           int Bl, int M, int N, int ldc, int s0,
                                                           const float* __restrict__ wp,
                                                           const float* __restrict__ bp, float* __restrict__ per,
                                                           float* __restrict__ logz) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int sg = s0 + r / M;
  const float w = *wp, b = *bp;
  float* c = cos + (long)r * ldc;
  if (lane == 0) c[sg] = rawd[r];  // get_cossim's diagonal overwrite (utils.py:112-113)
  float mx = -INFINITY;
  for (int k = lane; k < N; k += 64) {
    const float cr = (k == sg) ? rawd[r] : c[k];
    mx = fmaxf(mx, w * (cr + EPS_SIM) + b);
  }
  mx = fmaxf(wave_max(mx), 0.f);
  float z = 0.f;
  for (int k = lane; k < N; k += 64) {
    const float cr = (k == sg) ? rawd[r] : c[k];
    z += expf(w * (cr + EPS_SIM) + b - mx);
  }
  z = wave_sum(z);
  // log(sum_k e^S + 1e-6) = mx + log(sum_k e^{S-mx} + 1e-6 e^{-mx}), mx >= 0
  const float lz = mx + logf(z + EPS_LOG * expf(-mx));
  if (lane == 0) {
    const float spos = w * (rawd[r] + EPS_SIM) + b;
    per[r] = lz - spos;
    logz[r] = lz;
  }
}

// fixed-order sum of n floats into out[0] (single block of 256)
__global__ __launch_bounds__(256) void sum_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += x[i];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

// ---------------------------------------------------------------------------
// K7a: row backward.  dS = p - delta, dcos = w dS; writes dcos with the diagonal
// zeroed (centroid side), alpha_r = sum_k dcos_rk raw_rk, and per-row dw/db partials.
__global__ __launch_bounds__(256) void ge2e_rowbwd_kernel(const float* __restrict__ cos, const float* __restrict__ logz,
                                                          int Bl, int M, int N, int ldc, int s0,
                                                          const float* __restrict__ wp,
                                                          const float* __restrict__ bp, const float* __restrict__ gl,
                                                          float* __restrict__ dcos, float* __restrict__ alpha,
                                                          float* __restrict__ dwdb) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int sg = s0 + r / M;
  const float w = *wp, b = *bp, g = gl ? *gl : 1.0f;
  const float lz = logz[r];
  const float* c = cos + (long)r * ldc;
  float* dc = dcos + (long)r * ldc;
  // sum_k dS_k x_k with dS = p - delta is a difference of two O(1) sums (sum_k p_k = 1 - 1e-6 e^-lz):
  // summed as sum_k p_k (x_k - x_d) - x_d 1e-6 e^-lz, i.e. only the small differences accumulate
  // (the reference's fp32 dw is within 5e-8 of fp64 at c2; the direct form was 5e-5 off)
  const float cd = c[sg];
  const float tail = EPS_LOG * expf(-lz);  // 1 - sum_k p_k
  float a = 0.f, dw = 0.f;
  for (int k = lane; k < N; k += 64) {
    const float cr = c[k];
    const float p = expf(w * (cr + EPS_SIM) + b - lz);
    const float ds = g * (p - (k == sg ? 1.0f : 0.0f));
    const float pd = p * (cr - cd);
    a += pd;
    dw += pd;
    dc[k] = (k == sg) ? 0.f : w * ds;
  }
  for (int k = N + lane; k < ldc; k += 64) dc[k] = 0.f;
  a = wave_sum(a);
  dw = wave_sum(dw);
  if (lane == 0) {
    alpha[r] = w * g * (a - cd * tail);
    dwdb[r] = g * (dw - (cd + EPS_SIM) * tail);
    dwdb[Bl + r] = -g * tail;
  }
}

// K7b: beta_k = sum_r dcos_off[r,k] raw[r,k]  (column reduction over rows, two levels:
// block (k-chunk of 64, row-chunk of 64) -> partial[row-chunk][k]; then a fixed-order sum)
__global__ __launch_bounds__(256) void ge2e_beta_partial_kernel(const float* __restrict__ dcos,
                                                                const float* __restrict__ cos, int Bl, int N, int ldc,
                                                                float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int k = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int r0 = blockIdx.y * 64 + w * 16;
  float s = 0.f;
  if (k < N)
    for (int r = r0; r < min(r0 + 16, Bl); ++r) s += dcos[(long)r * ldc + k] * cos[(long)r * ldc + k];
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && k < N) partial[(long)blockIdx.y * N + k] = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                                            (red[2][threadIdx.x] + red[3][threadIdx.x]);
}
__global__ void ge2e_beta_final_kernel(const float* __restrict__ partial, int nchunk, int N,
                                       float* __restrict__ beta) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  float s = 0.f;
  for (int c = 0; c < nchunk; ++c) s += partial[(long)c * N + k];
  beta[k] = s;
}

// K7c: dw, db = fixed-order sums of the per-row partials
__global__ __launch_bounds__(256) void ge2e_dwdb_kernel(const float* __restrict__ dwdb_rows, int Bl,
                                                        float* __restrict__ out) {
  __shared__ float red[4];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < Bl; i += 256) {
    a += dwdb_rows[i];
    b += dwdb_rows[Bl + i];
  }
  a = block_sum256(a, red);
  b = block_sum256(b, red);
  if (threadIdx.x == 0) {
    out[0] = a;
    out[1] = b;
  }
}

// K7d: finalize dE for one local speaker per block:
//   dC_j  = (dChat_j - beta_j C^_j [|C|>eps]) / max(|C_j|, eps)
//   dU_r  = dcos_d (E^_r - raw_d U^_r [|U|>eps]) / max(|U_r|, eps)
//   dE_r  = (G1_r + dcos_d U^_r - alpha_r E^_r [|E|>eps]) / max(|E_r|, eps)
//           + dC_j / M + (sum_i' dU_ji' - dU_r) / (M - 1)
// where dcos_d = w dS[r, s(r)] is recovered from alpha_r's definition inputs.
// any M (the split path's general form): one thread per d walks the speaker's M rows twice
__global__ __launch_bounds__(256) void ge2e_finalize_serial_kernel(
    int M, int D, int s0, const float* __restrict__ dchat, const float* __restrict__ beta,
    const float* __restrict__ Chat, const float* __restrict__ Cn, const float* __restrict__ Ehat,
    const float* __restrict__ Uhat, const float* __restrict__ En, const float* __restrict__ Un,
    const float* __restrict__ rawd, const float* __restrict__ dcd, const float* __restrict__ alpha,
    const float* __restrict__ G1, float* __restrict__ dE) {
  const int j = blockIdx.x;
  const int sg = s0 + j;
  const float cn = Cn[sg];
  const float icn = 1.0f / fmaxf(cn, EPS_COS);
  const float pc = cn > EPS_COS ? 1.f : 0.f;
  const float bj = beta[sg];
  const float invM = 1.0f / (float)M, invm1 = 1.0f / (float)(M - 1);
  for (int d = threadIdx.x; d < D; d += 256) {
    const long cd = (long)sg * D + d;
    const float dC = (dchat[cd] - bj * Chat[cd] * pc) * icn;
    float sumdU = 0.f;
    for (int i = 0; i < M; ++i) {
      const int r = j * M + i;
      const float iu = 1.0f / fmaxf(Un[r], EPS_COS);
      const float pu = Un[r] > EPS_COS ? 1.f : 0.f;
      sumdU += dcd[r] * (Ehat[(long)r * D + d] - rawd[r] * Uhat[(long)r * D + d] * pu) * iu;
    }
    for (int i = 0; i < M; ++i) {
      const int r = j * M + i;
      const long rd = (long)r * D + d;
      const float iu = 1.0f / fmaxf(Un[r], EPS_COS);
      const float pu = Un[r] > EPS_COS ? 1.f : 0.f;
      const float dU = dcd[r] * (Ehat[rd] - rawd[r] * Uhat[rd] * pu) * iu;
      const float ie = 1.0f / fmaxf(En[r], EPS_COS);
      const float pe = En[r] > EPS_COS ? 1.f : 0.f;
      const float gE = (G1[rd] + dcd[r] * Uhat[rd] - alpha[r] * Ehat[rd] * pe) * ie;
      dE[rd] = gE + dC * invM + (sumdU - dU) * invm1;
    }
  }
}

#define GF_MMAX_FIN 16  // utterances per speaker of the one-pass finalize (one wave each)
__global__ __launch_bounds__(1024) void ge2e_finalize_kernel(
    int M, int D, int s0, const float* __restrict__ dchat, const float* __restrict__ beta,
    const float* __restrict__ Chat, const float* __restrict__ Cn, const float* __restrict__ Ehat,
    const float* __restrict__ Uhat, const float* __restrict__ En, const float* __restrict__ Un,
    const float* __restrict__ rawd, const float* __restrict__ dcd, const float* __restrict__ alpha,
    const float* __restrict__ G1, float* __restrict__ dE) {
  // workgroup (speaker j, 64-wide d slice q), wave i = the speaker's utterance i (M <= 16 waves):
  // every (row, d) of the slice in one pass, the leave-one-out sum of dU through LDS (the cols
  // kernel's epilogue; the former one-thread-per-d form walked the M rows twice, serially)
  __shared__ float dUs[GF_MMAX_FIN][64];
  const int j = blockIdx.x, q = blockIdx.y;
  const int lane = threadIdx.x & 63, i = threadIdx.x >> 6;
  const int sg = s0 + j;
  const int d = q * 64 + lane;
  const bool mine = d < D && i < M;
  const int r = j * M + i;
  const long rd = (long)r * D + d;
  float dU = 0.f, gE = 0.f;
  if (mine) {
    const float un = Un[r], en = En[r], dd = dcd[r];
    const float iu = 1.0f / fmaxf(un, EPS_COS);
    const float pu = un > EPS_COS ? 1.f : 0.f;
    const float eh = Ehat[rd], uh = Uhat[rd];
    dU = dd * (eh - rawd[r] * uh * pu) * iu;
    const float ie = 1.0f / fmaxf(en, EPS_COS);
    const float pe = en > EPS_COS ? 1.f : 0.f;
    gE = (G1[rd] + dd * uh - alpha[r] * eh * pe) * ie;
    dUs[i][lane] = dU;
  }
  __syncthreads();
  if (!mine) return;
  const float cn = Cn[sg];
  const float icn = 1.0f / fmaxf(cn, EPS_COS);
  const float pc = cn > EPS_COS ? 1.f : 0.f;
  const long cd = (long)sg * D + d;
  const float dC = (dchat[cd] - beta[sg] * Chat[cd] * pc) * icn;
  float sumdU = 0.f;
  for (int k = 0; k < M; ++k) sumdU += dUs[k][lane];
  const float invM = 1.0f / (float)M, invm1 = 1.0f / (float)(M - 1);
  dE[rd] = gE + dC * invM + (sumdU - dU) * invm1;
}

// dE of a shard's speakers from the reduced [dC^ | beta]: the one-pass 2-D form up to GF_MMAX_FIN
// utterances per speaker, else the serial form
static void launch_finalize(int N_local, int M, int D, int s0, const float* dchat, const float* beta, const Ge2eWs& ws,
                            const float* dcd, float* dE, hipStream_t stream) {
  if (M <= GF_MMAX_FIN)
    hipLaunchKernelGGL(ge2e_finalize_kernel, dim3(N_local, (D + 63) / 64), dim3(64 * M), 0, stream, M, D, s0, dchat, beta,
                       ws.Chat, ws.Cn, ws.Ehat, ws.Uhat, ws.En, ws.Un, ws.rawd, dcd, ws.alpha, ws.G1, dE);
  else
    hipLaunchKernelGGL(ge2e_finalize_serial_kernel, dim3(N_local), dim3(256), 0, stream, M, D, s0, dchat, beta, ws.Chat,
                       ws.Cn, ws.Ehat, ws.Uhat, ws.En, ws.Un, ws.rawd, dcd, ws.alpha, ws.G1, dE);
}

// dcos on the diagonal (w dS[r, s(r)]) for the finalize step, recomputed from logz
__global__ void ge2e_dcd_kernel(const float* __restrict__ rawd, const float* __restrict__ logz, int Bl,
                                const float* __restrict__ wp, const float* __restrict__ bp,
                                const float* __restrict__ gl, float* __restrict__ dcd) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= Bl) return;
  const float w = *wp, b = *bp, g = gl ? *gl : 1.0f;
  const float p = expf(w * (rawd[r] + EPS_SIM) + b - logz[r]);
  dcd[r] = w * g * (p - 1.0f);
}

// ============================================================================
// C ABI
// ============================================================================
extern "C" size_t sv_ge2e_workspace_size(int N_local, int M, int D, int N) {
  return carve(nullptr, N_local, M, D, N).total;
}

static bool ge2e_args_ok(const float* E, int Nl, int M, int D, int s0, int N) {
  return E && Nl > 0 && M >= 2 && D > 0 && D % 4 == 0 && N >= Nl && s0 >= 0 && s0 + Nl <= N;
}

extern "C" int sv_ge2e_speaker_sums(const float* E, int N_local, int M, int D, float* ssum_local, hipStream_t stream) {
  if (!E || !ssum_local || N_local <= 0 || M <= 0 || D <= 0) return SV_EARG;
  hipLaunchKernelGGL(ge2e_sums_kernel, dim3(N_local), dim3(256), 0, stream, E, M, D, ssum_local);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_fwd_rows(const float* E, int N_local, int M, int D, int spk_offset, int N, const float* ssum_all,
                                const float* w, const float* b, float* per, float* loss_local, float* workspace,
                                hipStream_t stream) {
  if (!ge2e_args_ok(E, N_local, M, D, spk_offset, N) || !ssum_all || !w || !b || !per || !workspace) return SV_EARG;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N);
  const int Bl = N_local * M, Np = (N + 3) & ~3;
  hipLaunchKernelGGL(ge2e_centroid_kernel, dim3(Np), dim3(256), 0, stream, ssum_all, N, M, D, ws.Chat, ws.Cn);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_rowprep_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, E, ssum_all, Bl, M, D, spk_offset,
                     ws.Ehat, ws.Uhat, ws.En, ws.Un, ws.rawd);
  SV_LAUNCH_CHECK();
  // cos = E^ C^T  (fp32 MFMA; rows of E^ and C^ are both D-contiguous)
  int rc = gemm_f32(1, 1, Bl, Np, D, ws.Ehat, D, ws.Chat, D, ws.cos, Np, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(ge2e_rowloss_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, ws.cos, ws.rawd, Bl, M, N, Np,
                     spk_offset, w, b, per, ws.logz);
  SV_LAUNCH_CHECK();
  if (loss_local) {
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, stream, per, Bl, loss_local);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

extern "C" int sv_ge2e_fwd(const float* E, int N, int M, int D, const float* w, const float* b, float* loss, float* per,
                           float* workspace, float* ssum, hipStream_t stream) {
  if (!ssum) return SV_EARG;
  int rc = sv_ge2e_speaker_sums(E, N, M, D, ssum, stream);
  if (rc) return rc;
  return sv_ge2e_fwd_rows(E, N, M, D, 0, N, ssum, w, b, per, loss, workspace, stream);
}

extern "C" int sv_ge2e_bwd_rows(int N_local, int M, int D, int spk_offset, int N, const float* w, const float* b,
                                const float* gloss, float* dchat_partial, float* beta_partial, float* dwdb,
                                float* workspace, hipStream_t stream) {
  if (N_local <= 0 || M < 2 || D <= 0 || N < N_local || !w || !b || !dchat_partial || !beta_partial || !dwdb ||
      !workspace)
    return SV_EARG;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N);
  const int Bl = N_local * M, Np = (N + 3) & ~3;
  hipLaunchKernelGGL(ge2e_rowbwd_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, ws.cos, ws.logz, Bl, M, N, Np,
                     spk_offset, w, b, gloss, ws.dcos, ws.alpha, ws.dwdb_rows);
  SV_LAUNCH_CHECK();
  // G1 = dcos_off C^   ([Bl, N] x [N, D]; C^ read as [K=N][D] row-contiguous)
  int rc = gemm_f32(1, 0, Bl, D, Np, ws.dcos, Np, ws.Chat, D, ws.G1, D, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  // dChat (before the norm Jacobian) = dcos_off^T E^   ([Np, Bl] x [Bl, D]); rows >= N are zero
  rc = gemm_f32(0, 0, Np, D, Bl, ws.dcos, Np, ws.Ehat, D, dchat_partial, D, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  const int nchunk = (Bl + 63) / 64;
  hipLaunchKernelGGL(ge2e_beta_partial_kernel, dim3((N + 63) / 64, nchunk), dim3(256), 0, stream, ws.dcos, ws.cos, Bl,
                     N, Np, ws.betap);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_beta_final_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, ws.betap, nchunk, N,
                     beta_partial);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_dwdb_kernel, dim3(1), dim3(256), 0, stream, ws.dwdb_rows, Bl, dwdb);
  SV_LAUNCH_CHECK();
  // diagonal dcos into the (now free) dwdb_rows slot for the finalize step
  hipLaunchKernelGGL(ge2e_dcd_kernel, dim3((Bl + 255) / 256), dim3(256), 0, stream, ws.rawd, ws.logz, Bl, w, b, gloss,
                     ws.dwdb_rows);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_bwd_finalize(int N_local, int M, int D, int spk_offset, int N, const float* dchat,
                                    const float* beta, float* dE, float* workspace, hipStream_t stream) {
  if (N_local <= 0 || M < 2 || D <= 0 || !dchat || !beta || !dE || !workspace) return SV_EARG;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N);
  launch_finalize(N_local, M, D, spk_offset, dchat, beta, ws, ws.dwdb_rows, dE, stream);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_bwd(int N, int M, int D, const float* w, const float* b, const float* gloss, float* dE,
                           float* dwdb, float* dchat, float* beta, float* workspace, hipStream_t stream) {
  int rc = sv_ge2e_bwd_rows(N, M, D, 0, N, w, b, gloss, dchat, beta, dwdb, workspace, stream);
  if (rc) return rc;
  return sv_ge2e_bwd_finalize(N, M, D, 0, N, dchat, beta, dE, workspace, stream);
}

// ============================================================================
// Fused single-GPU training path: GE2E forward + closed-form backward in three launches
// (sv_ge2e_train), for N <= 256 speakers, M <= 16, D <= 256 (every c1-c5 shape, c5's global N = 256
// included):
//   F1 ge2e_prep_kernel   one workgroup per speaker: its sum, centroid C^ and |C| (LDS
//                         reduction), and per utterance row E^, U^ (leave-one-out), the norms and
//                         the diagonal cosine (a wave per row, shuffle reductions)
//   F2 ge2e_rows_kernel   one wave per row, C^ of every speaker staged in LDS once per
//                         workgroup: the row's N cosines (lanes over speakers, ds_read_b128 of
//                         conflict-free padded C^ rows, E^ broadcast), the diagonal overwrite, the
//                         shuffle softmax (max, log-sum-exp, per-row loss), dS = p - delta,
//                         dcos, alpha, dw/db row partials and G1 = sum_k dcos_k C^_k
//   F3 ge2e_cols_kernel   one workgroup per (speaker k, 64-wide d slice): beta_k and
//                         dC^_k = sum_r dcos[r,k] E^_r over every row, then dC_k and the speaker's
//                         rows of dE (the split path's finalize); workgroup (0, 0) also sums the
//                         loss and dw, db in fixed order
// The arithmetic is the split path's (same formulas, fixed-order sums; the cosines by FMA dot
// products instead of the MFMA GEMM), so results agree to fp32 rounding.
// ============================================================================
#define GF_NMAX 256
#define GF_DMAX 256
#define GF_MMAX 16

// ssum (sharded form): the speaker's sum goes out for the all-gather instead of C^ / |C| (the
// centroids of every rank's speakers are formed after it by ge2e_centroid_kernel)
__global__ __launch_bounds__(256) void ge2e_prep_kernel(const float* __restrict__ E, int M, int D,
                                                        float* __restrict__ Chat, float* __restrict__ Cn,
                                                        float* __restrict__ Ehat, float* __restrict__ Uhat,
                                                        float* __restrict__ En, float* __restrict__ Un,
                                                        float* __restrict__ rawd, float* __restrict__ ssum) {
  // one pass over the speaker's rows: wave w holds rows w, w + 4, ... (lane: d = 4 lane .. + 3,
  // D <= 256), their per-wave partial sums meet in LDS (added in wave order, rows in order)
  constexpr int RW = (GF_MMAX + 3) / 4;
  __shared__ float4 ps[4][64];
  __shared__ float red[4];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool dok = 4 * lane < D;
  const float* Ej = E + (long)j * M * D;
  float4 e[RW];
  float4 part = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int i = w + 4 * q;
    e[q] = (i < M && dok) ? *reinterpret_cast<const float4*>(Ej + (long)i * D + 4 * lane) : float4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    part.x += e[q].x;
    part.y += e[q].y;
    part.z += e[q].z;
    part.w += e[q].w;
  }
  ps[w][lane] = part;
  __syncthreads();
  const float4 p0 = ps[0][lane], p1 = ps[1][lane], p2 = ps[2][lane], p3 = ps[3][lane];
  const float4 sum = float4{((p0.x + p1.x) + p2.x) + p3.x, ((p0.y + p1.y) + p2.y) + p3.y,
                            ((p0.z + p1.z) + p2.z) + p3.z, ((p0.w + p1.w) + p2.w) + p3.w};
  const float fm = (float)M;
  const float4 c = float4{sum.x / fm, sum.y / fm, sum.z / fm, sum.w / fm};
  const float invm1 = 1.0f / (float)(M - 1);
  // every lane-partial first (|c|^2; per row |e|^2, |u|^2, e.u), then the wave sums by DPP
  // (independent chains, no LDS round trips; the sums are wave-uniform)
  float v[3 * RW + 1];
  float4 uu[RW];
  v[3 * RW] = c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w;
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const float4 x = e[q];
    uu[q] = float4{(sum.x - x.x) * invm1, (sum.y - x.y) * invm1, (sum.z - x.z) * invm1, (sum.w - x.w) * invm1};
    const float4 u = uu[q];
    v[3 * q] = x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    v[3 * q + 1] = u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
    v[3 * q + 2] = x.x * u.x + x.y * u.y + x.z * u.z + x.w * u.w;
  }
#pragma unroll
  for (int i = 0; i < 3 * RW + 1; ++i) v[i] = wave_sum_dpp(v[i]);
  const float cn = sqrtf(v[3 * RW]);
  const float icn = 1.0f / fmaxf(cn, EPS_COS);
  if (w == 0 && ssum) {
    if (dok) *reinterpret_cast<float4*>(ssum + (long)j * D + 4 * lane) = sum;
  } else if (w == 0) {
    if (dok) *reinterpret_cast<float4*>(Chat + (long)j * D + 4 * lane) = float4{c.x * icn, c.y * icn, c.z * icn, c.w * icn};
    if (lane == 0) Cn[j] = cn;
  }
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const int i = w + 4 * q;
    if (i >= M) break;
    const long r = (long)j * M + i;
    const float4 x = e[q], u = uu[q];
    const float ne = sqrtf(v[3 * q]), nu = sqrtf(v[3 * q + 1]);
    const float ie = 1.0f / fmaxf(ne, EPS_COS), iu = 1.0f / fmaxf(nu, EPS_COS);
    if (dok) {
      *reinterpret_cast<float4*>(Ehat + r * D + 4 * lane) = float4{x.x * ie, x.y * ie, x.z * ie, x.w * ie};
      *reinterpret_cast<float4*>(Uhat + r * D + 4 * lane) = float4{u.x * iu, u.y * iu, u.z * iu, u.w * iu};
    }
    if (lane == 0) {
      En[r] = ne;
      Un[r] = nu;
      rawd[r] = v[3 * q + 2] * ie * iu;  // cos(e, u) = e.u / (|e| |u|)
    }
  }
  (void)red;
}

// F2: GF_ROWW rows per workgroup, one per wave (160 workgroups of 4 waves at c2: each row's
// serial work in its own wave; 8 waves per workgroup measured slower, 11.2 vs 10.0 us at c2).
// Cs [NT][D + 4] fp32 in LDS (16-B padded rows: the 16 lanes of a ds_read_b128 group hit
// disjoint banks); the rows' E^ in Es [GF_ROWW][D]; per-row dcos in Vs [GF_ROWW][N].
// NH = 64-speaker groups per lane: 2 for N <= 128 (C^ staged once, NT = N), 4 for N <= 256 (c5's
// "centroid LDS stress": 256 fp32 rows of C^ are 266 KB, over the 160 KB LDS), where C^ is staged
// in two tiles of GF_TILE = 128 speakers (133 KB): tile 0, then tile 1 for the cosines, G1 over
// tile 1 while it is resident, then tile 0 again -- still fp32 throughout.
#define GF_ROWW 4
#define GF_TILE 128
template <int NH>
__global__ __launch_bounds__(64 * GF_ROWW) void ge2e_rows_kernel(const float* __restrict__ Chat, const float* __restrict__ Ehat,
                                                        const float* __restrict__ rawd, int Bl, int M, int N, int D,
                                                        int ldc, int s0, const float* __restrict__ wp,
                                                        const float* __restrict__ bp, float* __restrict__ per,
                                                        float* __restrict__ cos, float* __restrict__ dcos,
                                                        float* __restrict__ alpha, float* __restrict__ dcd,
                                                        float* __restrict__ dwdb_rows, float* __restrict__ G1) {
  static_assert(NH == 2 || NH == 4, "NH: 64-speaker groups per lane");
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  const int LDC = D + 4;
  const int NT = NH == 2 ? N : GF_TILE;  // speakers per LDS tile
  float* Cs = gsm;                       // [NT][LDC]
  float* Es = Cs + (size_t)NT * LDC;     // [GF_ROWW][D]
  float* Vs = Es + GF_ROWW * D;          // [GF_ROWW][N]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int D4 = D / 4;
  // global -> LDS copy of C^ rows k0 .. .  D = 256 (every c1-c5 shape): by LDS-DMA, one 1 KB row per
  // wave instruction (no VGPR round trip, every row in flight at once; the register copy below kept
  // ~8 loads per lane in flight and took ~12 us per 128-speaker tile at c5's rank shape), waited for
  // by the caller's vmcnt(0) + barrier; else through registers (distinct address spaces: the unrolled
  // loads issue back to back)
  auto stage = [&](int k0) {
    const int nk = min(NT, N - k0);
    if (D == 256) {
      for (int row = w; row < nk; row += GF_ROWW)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(Chat + (long)(k0 + row) * D + lane * 4),
                                         (__attribute__((address_space(3))) void*)(Cs + row * LDC), 16, 0, 0);
      return;
    }
    const int NQ = nk * D4;
#pragma unroll 8
    for (int q = tid; q < NQ; q += 64 * GF_ROWW) {
      const int row = q / D4, col = (q - row * D4) * 4;
      *reinterpret_cast<float4*>(Cs + row * LDC + col) =
          *reinterpret_cast<const float4*>(Chat + (long)(k0 + row) * D + col);
    }
  };
  stage(0);
  const int r = blockIdx.x * GF_ROWW + w;   // this wave's row
  const bool live = r < Bl;
  if (live)
    for (int c = lane * 4; c < D; c += 256)
      *reinterpret_cast<float4*>(Es + w * D + c) = *reinterpret_cast<const float4*>(Ehat + (long)r * D + c);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA of C^ landed
  __syncthreads();
  if constexpr (NH == 2) {
    if (!live) return;  // (no later workgroup barrier)
  }
  const float wv = *wp, bv = *bp;
  const int sg = s0 + r / M;  // global speaker of this row (s0: the shard's first)
  const float rd = live ? rawd[r] : 0.f;
  // cosines: KS speaker lanes x DS d-slices (DS = 1 for N > 32: lane k and k + 64 over all of
  // D; small N splits D so the wave's lanes all work, the slices then meet by a butterfly), E^
  // broadcast; four independent partial sums (d mod 4), added pairwise at the end.  Speaker
  // lane + 64 h is cv[h].
  int DS = N <= 8 ? 8 : N <= 16 ? 4 : N <= 32 ? 2 : 1;
  while (DS > 1 && D % (4 * DS)) DS >>= 1;
  const int KS = 64 / DS, dlen = D / DS;
  const int kl = lane & (KS - 1), d0 = (lane / KS) * dlen;
  float cv[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) cv[h] = 0.f;
  const float* e0 = Es + w * D;
#pragma unroll
  for (int t = 0; t < NH / 2; ++t) {
    if (t > 0) {  // NH == 4: the second tile
      __syncthreads();
      stage(t * GF_TILE);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
      const int kt = kl + 64 * hk;  // speaker within the tile
      if (live && t * GF_TILE + kt < N) {
        float4 a = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
        for (int c = d0; c < d0 + dlen; c += 4) {
          const float4 cc = *reinterpret_cast<const float4*>(Cs + kt * LDC + c);
          const float4 x0 = *reinterpret_cast<const float4*>(e0 + c);
          a.x += x0.x * cc.x;
          a.y += x0.y * cc.y;
          a.z += x0.z * cc.z;
          a.w += x0.w * cc.w;
        }
        cv[2 * t + hk] = (a.x + a.y) + (a.z + a.w);
      }
    }
  }
  for (int o = KS; o < 64; o <<= 1) cv[0] += __shfl_xor(cv[0], o, 64);  // lane k < KS: speaker k
#pragma unroll
  for (int h = 0; h < NH; ++h)
    if (lane + 64 * h == sg) cv[h] = rd;  // get_cossim's diagonal overwrite (utils.py:112-113)
  // row softmax: S = w (cos + 1e-6) + b;  lz = log(sum_k e^S + 1e-6)
  float mx = -INFINITY;
#pragma unroll
  for (int h = 0; h < NH; ++h)
    if (lane + 64 * h < N) mx = fmaxf(mx, wv * (cv[h] + EPS_SIM) + bv);
  mx = fmaxf(wave_max(mx), 0.f);
  float z = 0.f;
#pragma unroll
  for (int h = 0; h < NH; ++h)
    if (lane + 64 * h < N) z += expf(wv * (cv[h] + EPS_SIM) + bv - mx);
  z = wave_sum(z);
  const float lz = mx + logf(z + EPS_LOG * expf(-mx));
  // row backward (gloss = 1): dS = p - delta, dcos = w dS; alpha, dw, db as sums of the small
  // differences p_k (x_k - x_d) and the analytic 1 - sum_k p_k = 1e-6 e^-lz (ge2e_rowbwd_kernel)
  const float tail = EPS_LOG * expf(-lz);
  float pdsum = 0.f;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int k = lane + 64 * h;
    if (live && k < N) {
      const float p = expf(wv * (cv[h] + EPS_SIM) + bv - lz);
      const float ds = p - (k == sg ? 1.0f : 0.0f);
      const float dcv = wv * ds;
      pdsum += p * (cv[h] - rd);
      const float off = (k == sg) ? 0.f : dcv;
      Vs[w * N + k] = off;
      cos[(long)r * ldc + k] = cv[h];
      dcos[(long)r * ldc + k] = off;
      if (k == sg) dcd[r] = dcv;
    }
  }
  pdsum = wave_sum(pdsum);
  if (live && lane == 0) {
    per[r] = lz - (wv * (rd + EPS_SIM) + bv);
    alpha[r] = wv * (pdsum - rd * tail);
    dwdb_rows[r] = pdsum - (rd + EPS_SIM) * tail;
    dwdb_rows[Bl + r] = -tail;
  }
  // G1_r = sum_k dcos_off[r,k] C^_k: lanes over d (4 each, D <= 256), even / odd speakers in two
  // accumulators, added at the end
  __builtin_amdgcn_wave_barrier();
  const float* vr = Vs + w * N;
  const int c = lane * 4;
  const bool cok = live && c < D;
  float4 g0 = float4{0.f, 0.f, 0.f, 0.f}, g1 = g0;
  auto g1_acc = [&](int ka, int kb, int k0) {  // speakers [ka, kb), tile in LDS from speaker k0
    int k = ka;
#pragma unroll 4
    for (; k + 1 < kb; k += 2) {
      const float d0 = vr[k], d1 = vr[k + 1];
      const float4 c0 = *reinterpret_cast<const float4*>(Cs + (k - k0) * LDC + c);
      const float4 c1 = *reinterpret_cast<const float4*>(Cs + (k + 1 - k0) * LDC + c);
      g0.x += d0 * c0.x;
      g0.y += d0 * c0.y;
      g0.z += d0 * c0.z;
      g0.w += d0 * c0.w;
      g1.x += d1 * c1.x;
      g1.y += d1 * c1.y;
      g1.z += d1 * c1.z;
      g1.w += d1 * c1.w;
    }
    if (k < kb) {
      const float d0 = vr[k];
      const float4 c0 = *reinterpret_cast<const float4*>(Cs + (k - k0) * LDC + c);
      g0.x += d0 * c0.x;
      g0.y += d0 * c0.y;
      g0.z += d0 * c0.z;
      g0.w += d0 * c0.w;
    }
  };
  if constexpr (NH == 2) {
    if (cok) g1_acc(0, N, 0);
  } else {
    if (cok) g1_acc(GF_TILE, N, GF_TILE);  // tile 1 is resident
    __syncthreads();
    stage(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (cok) g1_acc(0, GF_TILE, 0);
  }
  if (cok) *reinterpret_cast<float4*>(G1 + (long)r * D + c) = float4{g0.x + g1.x, g0.y + g1.y, g0.z + g1.z, g0.w + g1.w};
}

constexpr int GF_CH = 128;  // speakers per chunk of ge2e_rows4r_kernel

// ge2e_rows4r_kernel's centroid tile stride: 288 = 32 mod 64 banks, so the two speakers of a 16-lane
// LDS pass (8-lane groups reading 32 consecutive floats each) fall on disjoint banks
constexpr int GF_R4LDC = 288;

// a workgroup-uniform value (read from LDS) kept in an SGPR
__device__ __forceinline__ float uniform_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// F2 for 128 < N <= 256 and D = 256 (c5's global N), register-blocked: RW rows per workgroup of NWV
// waves (8 waves, 2 rows: 160 workgroups at a c5 rank's 320 rows).  The speakers pass through LDS in
// two chunks of 128 (fp32), each staged once by LDS-DMA; per chunk the cosines, then the chunk's
// share of G1 = sum_{k != j} dcos_k C^_k accumulated online (flash-attention style: weights
// e^{S_k - m} against the running row max m, the partial sum rescaled by e^{m_old - m} when a chunk
// raises it, finally scaled by w e^{m - lz}).
// FUSEC (sharded form): the chunks hold the all-gathered speaker SUMS s_k; the centroid scale
// c_k = 1 / (M max(|s_k / M|, eps)) comes from |s_k|^2 summed in the same loop as the cosine, so
// cos = (E^ . s_k) c_k and the G1 weights carry c_k -- no normalisation pass and no centroid
// launch; the workgroups also write C^ and |C| of the shard's own speakers for the finalize step.  Every centroid value leaves LDS once per WORKGROUP and
// feeds the RW rows from registers:
//   cosines: lane = GL s + g (GL = 8-lane groups) holds E^[RW rows][32 j + 4 g .. +3] (j < 8); group
//     s takes one speaker per step, reads its 256 values as 8 conflict-free float4 per lane (tile
//     stride GF_R4LDC), and the RW dot products (+ |s_k|^2 under FUSEC) are summed over the group
//     by DPP; the steps are branch-free so their reads, FMAs and sums interleave;
//   softmax: one thread per (row, speaker of the chunk), online max / sum per row as above;
//   G1: wave w takes speakers KW w .. KW w + KW - 1 of the chunk (KW = 128 / NWV), lane 4-column
//     slice d = 4 lane, its RW weights per speaker one broadcast LDS read; the
//     waves' [RW][256] partials meet once, in LDS, after the last chunk;
//   row backward: one thread per (row, speaker), cos / dcos stored coalesced.
// Measured at the c5 rank shape (scripts/ge2e_c5rank.py, kernel trace): 23.4 us for the r05 form
// with four waves per row (16 waves, 4 rows per workgroup; deleted), 22.9 here with 16 waves x 4 rows
// and 16-lane groups (the FUSEC form spilled), 17.1 with 8 waves x 2 rows, 14.5 with branch-free
// steps, 13.4 with 8-lane groups.  Phase probes (2.3 GHz shader clock): staging a chunk ~1.9 us
// (256 KB of sums per workgroup from L2, the per-CU fill rate), cosines 1.2 us, softmax 0.9 us and
// G1 ~0.9 us per chunk.
template <bool FUSEC, int NWV, int RW>
__global__ __launch_bounds__(64 * NWV) void ge2e_rows4r_kernel(const float* __restrict__ Csrc,
                                                          const float* __restrict__ Ehat,
                                                          const float* __restrict__ rawd, int Bl, int M, int N,
                                                          int ldc, int s0, const float* __restrict__ wp,
                                                          const float* __restrict__ bp, float* __restrict__ per,
                                                          float* __restrict__ cos, float* __restrict__ dcos,
                                                          float* __restrict__ alpha, float* __restrict__ dcd,
                                                          float* __restrict__ dwdb_rows, float* __restrict__ G1,
                                                          float* __restrict__ Chat_out, float* __restrict__ Cn_out) {
  constexpr int D = 256, LDC = GF_R4LDC, NCM = GF_NMAX / GF_CH, NT = 64 * NWV, KW = GF_CH / NWV;
  constexpr int GL = 8, SPS = 64 / GL, JN = D / (4 * GL), NS = KW / SPS;  // lanes per speaker, ...
  static_assert((GL == 8 || GL == 16) && KW % SPS == 0, "whole cosine steps");
  static_assert((NWV == 8 || NWV == 16) && (RW == 2 || RW == 4) && 2 * RW <= NWV && GF_CH / NWV * RW <= 64,
                "RW rows x 128 speakers of the softmax step on waves 0 .. 2 RW - 1");
  static_assert(256 * RW % NT == 0, "whole (row, speaker) items per thread in the row backward");
  auto sel = [](const auto* a, int i) {  // a[i] for a workgroup-uniform i, without dynamic indexing
    auto v = a[0];
#pragma unroll
    for (int q = 1; q < RW; ++q)
      if (i == q) v = a[q];
    return v;
  };
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  float* Cb = gsm;                     // [GF_CH][LDC]; after the last chunk: [NWV waves][RW][D] G1 partials
  float* Ss = Cb + GF_CH * LDC;        // [RW][GF_NMAX] cosines (diagonal overwritten)
  float* Vs = Ss + RW * GF_NMAX;       // [GF_CH][RW] G1 weights of the current chunk
  float* Kc = Vs + GF_CH * RW;         // [GF_CH] centroid scales of the current chunk
  float* red = Kc + GF_CH;             // [2][16]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane % GL, s = lane / GL;
  const int r0 = blockIdx.x * RW;
  const float wv = *wp, bv = *bp;
  int sg[RW];
  float rd[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const bool lv = r0 + i < Bl;
    sg[i] = s0 + (lv ? r0 + i : 0) / M;
    rd[i] = lv ? rawd[r0 + i] : 0.f;
  }
  float4 ev[RW][JN];
#pragma unroll
  for (int i = 0; i < RW; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
      ev[i][j] = *reinterpret_cast<const float4*>(Ehat + (long)min(r0 + i, Bl - 1) * D + 4 * GL * j + 4 * g);
  // (a row past Bl computes on a copy of the last row: its results are never stored; all 4 RW
  // loads in flight at once, no per-row branch)
  const int nc = (N + GF_CH - 1) / GF_CH;
  float m[RW], zsum[RW];
  float4 acc[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    m[i] = 0.f;  // (the row max is clamped at 0 as in ge2e_rows_kernel)
    zsum[i] = 0.f;
    acc[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int c = 0; c < NCM; ++c) {
    if (c >= nc) break;
    const int nk = min(GF_CH, N - c * GF_CH);
    if (c > 0) __syncthreads();  // every wave done with the previous chunk
    for (int row = w; row < nk; row += NWV)
      __builtin_amdgcn_global_load_lds(
          (__attribute__((address_space(1))) void*)(Csrc + (long)(c * GF_CH + row) * D + lane * 4),
          (__attribute__((address_space(3))) void*)(Cb + row * LDC), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // cosines of the chunk: wave w, step t, lane group s -> speaker KW w + SPS t + s; the steps are
    // independent and branch-free (a speaker past the chunk reads the chunk's last row and is not
    // stored), so their LDS reads, FMAs and DPP sums interleave
    {
      float a[NS][RW], q[NS];
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const int kr = min(KW * w + SPS * t + s, nk - 1);
        q[t] = 0.f;
#pragma unroll
        for (int i = 0; i < RW; ++i) a[t][i] = 0.f;
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const float4 cc = *reinterpret_cast<const float4*>(Cb + kr * LDC + 4 * GL * j + 4 * g);
#pragma unroll
          for (int i = 0; i < RW; ++i)
            a[t][i] += (ev[i][j].x * cc.x + ev[i][j].y * cc.y) + (ev[i][j].z * cc.z + ev[i][j].w * cc.w);
          if constexpr (FUSEC) q[t] += (cc.x * cc.x + cc.y * cc.y) + (cc.z * cc.z + cc.w * cc.w);
        }
      }
#pragma unroll
      for (int t = 0; t < NS; ++t) {
#pragma unroll
        for (int i = 0; i < RW; ++i) a[t][i] = dpp_group_sum<GL>(a[t][i]);
        if constexpr (FUSEC) q[t] = dpp_group_sum<GL>(q[t]);
      }
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const int kl = KW * w + SPS * t + s;
        float ck = 1.f;
        if constexpr (FUSEC)  // |C_k| = |s_k| / M, C^_k = s_k / (M max(|C_k|, eps))
          ck = __builtin_amdgcn_rcpf(fmaxf(__builtin_amdgcn_sqrtf(q[t]), (float)M * EPS_COS));  // (1 ulp ops)
        if (g == 0 && kl < nk) {
          const int k = c * GF_CH + kl;
          Kc[kl] = ck;
#pragma unroll
          for (int i = 0; i < RW; ++i) Ss[i * GF_NMAX + k] = (k == sg[i]) ? rd[i] : a[t][i] * ck;  // utils.py:112-113
        }
      }
    }
    if constexpr (FUSEC) {  // C^ and |C| of the shard's own speakers in this chunk (for the finalize step)
      const int nl = Bl / M;
      for (int j = (int)blockIdx.x + (int)gridDim.x * w; j < nl; j += (int)gridDim.x * NWV) {
        const int kt = s0 + j - c * GF_CH;
        if (kt < 0 || kt >= nk) continue;
        float4 v = *reinterpret_cast<const float4*>(Cb + kt * LDC + 4 * lane);
        const float cn = sqrtf(wave_sum_dpp(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w)) / (float)M;
        const float inv = 1.0f / ((float)M * fmaxf(cn, EPS_COS));
        v = float4{v.x * inv, v.y * inv, v.z * inv, v.w * inv};
        *reinterpret_cast<float4*>(Chat_out + (long)(s0 + j) * D + 4 * lane) = v;
        if (lane == 0) Cn_out[s0 + j] = cn;
      }
    }
    __syncthreads();
    // online softmax over the chunk: thread -> (row i = tid / 128, speaker kl = tid % 128), waves 0..7
    const int si = tid >> 7, skl = tid & 127, sk_g = c * GF_CH + skl;
    const bool sval = tid < 128 * RW && skl < nk && r0 + si < Bl;
    float sk = -INFINITY;
    if (sval) sk = wv * (Ss[si * GF_NMAX + sk_g] + EPS_SIM) + bv;
    if (w < 2 * RW) {
      const float tm = wave_max_dpp(sk);
      if (lane == 0) red[w] = tm;
    }
    __syncthreads();
    float resc[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const float mn = fmaxf(m[i], uniform_f(fmaxf(red[2 * i], red[2 * i + 1])));
      resc[i] = expf(m[i] - mn);
      m[i] = mn;
    }
    if (w < 2 * RW) {
      const int i = si;
      const float mi = sel(m, i);
      const int sgi = sel(sg, i);
      const float e = sval ? expf(sk - mi) : 0.f;
      // the diagonal is excluded from G1 (its gradient goes to U, utils.py:112-113)
      Vs[skl * RW + i] = (sval && sk_g != sgi) ? e * Kc[skl] : 0.f;
      const float es = wave_sum_dpp(e);
      if (lane == 0) red[16 + w] = es;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      zsum[i] = zsum[i] * resc[i] + uniform_f(red[16 + 2 * i] + red[16 + 2 * i + 1]);
      acc[i].x *= resc[i];
      acc[i].y *= resc[i];
      acc[i].z *= resc[i];
      acc[i].w *= resc[i];
    }
    // G1 partials: wave w, speakers KW w .. KW w + KW - 1, columns 4 lane .. 4 lane + 3
#pragma unroll
    for (int kk = 0; kk < KW; ++kk) {  // (past the chunk: the last row again, with weight 0)
      const int kr = min(KW * w + kk, nk - 1);
      const float4 cc = *reinterpret_cast<const float4*>(Cb + kr * LDC + 4 * lane);
      float vk[RW];  // the speaker's RW weights: one broadcast LDS read
      if constexpr (RW == 2) {
        const float2 t2 = *reinterpret_cast<const float2*>(Vs + (KW * w + kk) * RW);
        vk[0] = t2.x;
        vk[1] = t2.y;
      } else {
#pragma unroll
        for (int i = 0; i < RW; ++i) vk[i] = Vs[(KW * w + kk) * RW + i];
      }
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const float vs = vk[i];
        acc[i].x += vs * cc.x;
        acc[i].y += vs * cc.y;
        acc[i].z += vs * cc.z;
        acc[i].w += vs * cc.w;
      }
    }
  }
  float lz[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) lz[i] = m[i] + logf(zsum[i] + EPS_LOG * expf(-m[i]));
  __syncthreads();  // Cb free: the G1 partials meet there
#pragma unroll
  for (int i = 0; i < RW; ++i) *reinterpret_cast<float4*>(Cb + (w * RW + i) * D + 4 * lane) = acc[i];
  __syncthreads();
  // items (row i, speaker / column k) = (item / 256, item % 256), item = tid + NT it
  float pdv[256 * RW / NT];
#pragma unroll
  for (int it = 0; it < 256 * RW / NT; ++it) {
    const int item = tid + NT * it, i = item >> 8, k = item & 255, r = r0 + i;
    const bool live = r < Bl;
    const float lzi = sel(lz, i), mi = sel(m, i), rdi = sel(rd, i);
    const int sgi = sel(sg, i);
    float gs = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) gs += Cb[(ww * RW + i) * D + k];
    if (live) G1[(long)r * D + k] = gs * (wv * expf(mi - lzi));
    // row backward (gloss = 1): the small differences p_k (x_k - x_d), as ge2e_rows_kernel
    float pd = 0.f;
    if (live && k < N) {
      const float cv = Ss[i * GF_NMAX + k];
      const float p = expf(wv * (cv + EPS_SIM) + bv - lzi);
      const float dcv = wv * (p - (k == sgi ? 1.0f : 0.0f));
      pd = p * (cv - rdi);
      cos[(long)r * ldc + k] = cv;
      dcos[(long)r * ldc + k] = (k == sgi) ? 0.f : dcv;
      if (k == sgi) dcd[r] = dcv;
    }
    pdv[it] = wave_sum_dpp(pd);
  }
#pragma unroll
  for (int it = 0; it < 256 * RW / NT; ++it)
    if (lane == 0) red[w + NWV * it] = pdv[it];  // slot = item / 64: row i owns slots 4 i .. 4 i + 3
  __syncthreads();
  if (tid < RW) {
    const int i = tid, r = r0 + i;
    if (r < Bl) {
      const float lzi = sel(lz, i), rdi = sel(rd, i);
      // the analytic tail 1 - sum_k p_k = 1e-6 e^-lz
      const float tail = EPS_LOG * expf(-lzi);
      const float ps = (red[4 * i] + red[4 * i + 1]) + (red[4 * i + 2] + red[4 * i + 3]);
      per[r] = lzi - (wv * (rdi + EPS_SIM) + bv);
      alpha[r] = wv * (ps - rdi * tail);
      dwdb_rows[r] = ps - (rdi + EPS_SIM) * tail;
      dwdb_rows[Bl + r] = -tail;
    }
  }
}

// launch F2 for N speakers (<= GF_NMAX)
// (ssum != nullptr: the sharded form's all-gathered sums -- at 128 < N <= 256, D = 256 the rows
// kernel forms C^ itself, rows_fuse_centroids; else the caller runs ge2e_centroid_kernel first)
static bool rows_fuse_centroids(int N, int D) { return N > GF_TILE && N <= GF_NMAX && D == 256; }
static void launch_rows(int Bl, int M, int N, int D, int Np, int s0, const Ge2eWs& ws, const float* w, const float* b,
                        float* per, hipStream_t stream, const float* ssum = nullptr) {
  if (N > GF_TILE && D == 256) {
    const size_t lds = ((size_t)GF_CH * GF_R4LDC + 4 * GF_NMAX + 4 * GF_CH + GF_CH + 32) * sizeof(float);
    constexpr int R4W = 8, R4R = 2;
    const dim3 grid((Bl + R4R - 1) / R4R), block(64 * R4W);
    if (ssum)
      hipLaunchKernelGGL((ge2e_rows4r_kernel<true, R4W, R4R>), grid, block, lds, stream, ssum, ws.Ehat, ws.rawd, Bl, M, N, Np, s0, w,
                         b, per, ws.cos, ws.dcos, ws.alpha, ws.dcd, ws.dwdb_rows, ws.G1, ws.Chat, ws.Cn);
    else
      hipLaunchKernelGGL((ge2e_rows4r_kernel<false, R4W, R4R>), grid, block, lds, stream, ws.Chat, ws.Ehat, ws.rawd, Bl, M, N, Np,
                         s0, w, b, per, ws.cos, ws.dcos, ws.alpha, ws.dcd, ws.dwdb_rows, ws.G1, nullptr, nullptr);
    return;
  }
  const int NT = N <= GF_TILE ? N : GF_TILE;
  const size_t lds = ((size_t)NT * (D + 4) + GF_ROWW * (size_t)D + GF_ROWW * (size_t)N) * sizeof(float);
  const dim3 grid((Bl + GF_ROWW - 1) / GF_ROWW), block(64 * GF_ROWW);
  if (N <= GF_TILE)
    hipLaunchKernelGGL(ge2e_rows_kernel<2>, grid, block, lds, stream, ws.Chat, ws.Ehat, ws.rawd, Bl, M, N, D, Np, s0,
                       w, b, per, ws.cos, ws.dcos, ws.alpha, ws.dcd, ws.dwdb_rows, ws.G1);
  else
    hipLaunchKernelGGL(ge2e_rows_kernel<4>, grid, block, lds, stream, ws.Chat, ws.Ehat, ws.rawd, Bl, M, N, D, Np, s0,
                       w, b, per, ws.cos, ws.dcos, ws.alpha, ws.dcd, ws.dwdb_rows, ws.G1);
}

// F3: workgroup (speaker k, d slice q of 64), GF_COLW waves: beta_k, dC^_k[slice], dC_k[slice],
// then dE of speaker k's rows over the slice.  The row sum runs with lane = 16 s + t: t covers
// 4 consecutive d (16-B loads), s one of 4 row sub-groups, so a wave's batch of GF_COLU loads
// spans 4 GF_COLU rows and the whole c2 batch (640 rows) is one round trip to L2; rows in a fixed
// order per (wave, sub-group), the sub-groups then the waves added in a fixed order.
// PARTIAL (sharded form): k runs over all N speakers, the rows are this shard's; beta_k and dC^_k
// (before the norm Jacobian) go to the reduce buffer [Np][D] + [N] for the all-reduce, and the
// shard's dE is formed after it (ge2e_finalize_kernel); loss / dw / db are this shard's sums.
#define GF_COLW 16
#define GF_COLU 10
template <bool PARTIAL>
__global__ __launch_bounds__(64 * GF_COLW) void ge2e_cols_kernel(int Bl, int M, int N, int D, int ldc,
                                                        const float* __restrict__ Chat, const float* __restrict__ Cn,
                                                        const float* __restrict__ Ehat, const float* __restrict__ Uhat,
                                                        const float* __restrict__ En, const float* __restrict__ Un,
                                                        const float* __restrict__ rawd, const float* __restrict__ cos,
                                                        const float* __restrict__ dcos,
                                                        const float* __restrict__ alpha, const float* __restrict__ dcd,
                                                        const float* __restrict__ G1, const float* __restrict__ per,
                                                        const float* __restrict__ dwdb_rows, float* __restrict__ dE,
                                                        float* __restrict__ loss, float* __restrict__ dwdb,
                                                        float* __restrict__ red_dchat, float* __restrict__ red_beta) {
  constexpr int NW = GF_COLW, U = GF_COLU;
  __shared__ __attribute__((aligned(16))) float part[NW][64];
  __shared__ float bpart[NW];
  __shared__ float dCs[64];
  __shared__ float dUs[GF_MMAX][64];
  __shared__ float red3[3][NW];
  const int k = blockIdx.x, q = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int s = lane >> 4, t = lane & 15;
  const int d4 = q * 64 + 4 * t;  // D % 4 == 0: the 4 values are all in range or all out
  const bool d4ok = d4 < D;
  float4 acc = float4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int r = 4 * w + s; r < Bl; r += 4 * NW * U) {
    float dc[U], cv[U];
    float4 ev[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned rr = r + 4 * NW * u;  // 32-bit offsets: SGPR base + VGPR offset addressing
      const bool ok = rr < (unsigned)Bl;
      dc[u] = ok ? dcos[rr * (unsigned)ldc + k] : 0.f;
      cv[u] = ok ? cos[rr * (unsigned)ldc + k] : 0.f;
      ev[u] = (ok && d4ok) ? *reinterpret_cast<const float4*>(Ehat + (rr * (unsigned)D + d4)) : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc.x += dc[u] * ev[u].x;
      acc.y += dc[u] * ev[u].y;
      acc.z += dc[u] * ev[u].z;
      acc.w += dc[u] * ev[u].w;
      bsum += dc[u] * cv[u];
    }
  }
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o, 64);
    acc.y += __shfl_xor(acc.y, o, 64);
    acc.z += __shfl_xor(acc.z, o, 64);
    acc.w += __shfl_xor(acc.w, o, 64);
    bsum += __shfl_xor(bsum, o, 64);
  }
  if (lane < 16) *reinterpret_cast<float4*>(&part[w][4 * t]) = acc;
  if (lane == 0) bpart[w] = bsum;
  if constexpr (PARTIAL) {
    __syncthreads();
    if (tid < 64 && q * 64 + tid < D) {
      float dch = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) dch += part[i][tid];
      red_dchat[(long)k * D + q * 64 + tid] = dch;
    }
    if (tid == 0 && q == 0) {
      float beta = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) beta += bpart[i];
      red_beta[k] = beta;
    }
  } else {
  // this wave's dE row (speaker k's utterance w): operands loaded before the barrier, dU shared
  // through LDS so the sum over the speaker's M rows needs no second trip to memory
  const int d = q * 64 + lane;
  const bool dok = d < D;
  const bool mine = dok && w < M;
  float dU = 0.f, gE = 0.f;
  long rdx = 0;
  if (mine) {
    const int rr = k * M + w;
    rdx = (long)rr * D + d;
    const float un = Un[rr], en = En[rr], dd = dcd[rr];
    const float iu = 1.0f / fmaxf(un, EPS_COS);
    const float pu = un > EPS_COS ? 1.f : 0.f;
    const float eh = Ehat[rdx], uh = Uhat[rdx];
    dU = dd * (eh - rawd[rr] * uh * pu) * iu;
    const float ie = 1.0f / fmaxf(en, EPS_COS);
    const float pe = en > EPS_COS ? 1.f : 0.f;
    gE = (G1[rdx] + dd * uh - alpha[rr] * eh * pe) * ie;
    dUs[w][lane] = dU;
  }
  __syncthreads();
  const float cn = Cn[k];
  const float icn = 1.0f / fmaxf(cn, EPS_COS);
  const float pc = cn > EPS_COS ? 1.f : 0.f;
  float beta = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) beta += bpart[i];
  if (tid < 64 && dok) {
    float dch = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) dch += part[i][tid];
    dCs[tid] = (dch - beta * Chat[(long)k * D + d] * pc) * icn;
  }
  __syncthreads();
  if (mine) {
    const float invM = 1.0f / (float)M, invm1 = 1.0f / (float)(M - 1);
    float sumdU = 0.f;
    for (int i = 0; i < M; ++i) sumdU += dUs[i][lane];
    dE[rdx] = gE + dCs[lane] * invM + (sumdU - dU) * invm1;
  }
  }  // !PARTIAL
  if (k == 0 && q == 0) {  // loss = sum per, dw, db: fixed-order block sums (block-uniform branch)
    float l = 0.f, a = 0.f, b = 0.f;
    for (int i = tid; i < Bl; i += 64 * NW) {
      l += per[i];
      a += dwdb_rows[i];
      b += dwdb_rows[Bl + i];
    }
    l = wave_sum(l);
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      red3[0][w] = l;
      red3[1][w] = a;
      red3[2][w] = b;
    }
    __syncthreads();
    if (tid == 0) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
      for (int i = 0; i < NW; ++i) {
        s0 += red3[0][i];
        s1 += red3[1][i];
        s2 += red3[2][i];
      }
      loss[0] = s0;
      dwdb[0] = s1;
      dwdb[1] = s2;
    }
  }
}

// F3 in the sharded form for D <= 256 (the c4 / c5 ranks' small row counts): one workgroup per
// KB speakers k0 .. k0 + KB - 1 over all of D (lane: d = 4 lane .. + 3), 16 waves over the shard's
// rows (row w, w + 16, ...: the KB speakers' dcos[r,k] and cos[r,k] are one broadcast load each per
// row and wave, E^_r one 1-KB coalesced load, read once for KB speakers), the waves' partials added
// in LDS in wave order -- every speaker's sums in the same order for any KB.  Writes this shard's
// dC^_k and beta_k to the reduce buffer, and workgroup 0 the shard's loss / dw / db partials
// (r05: KB = 1 ran 256 workgroups that each streamed all of E^ from L2, 84 MB at c5's rank shape,
// 7.5-9.4 us; ge2e_cols_kernel<true> before it ran (N, D / 64) workgroups, 11 us; KB = 2 / 4 with
// 16-B broadcast loads measured 10.2 / 11.8 us: the product launches KB = 1).
template <int KB>
__global__ __launch_bounds__(1024) void ge2e_cols_partial_kernel(int Bl, int N, int D, int ldc,
                                                                 const float* __restrict__ Ehat,
                                                                 const float* __restrict__ cos,
                                                                 const float* __restrict__ dcos,
                                                                 const float* __restrict__ per,
                                                                 const float* __restrict__ dwdb_rows,
                                                                 float* __restrict__ loss, float* __restrict__ dwdb,
                                                                 float* __restrict__ red_dchat,
                                                                 float* __restrict__ red_beta) {
  constexpr int NW = 16;
  __shared__ __attribute__((aligned(16))) float4 part[KB][NW][64];
  __shared__ float bpart[KB][NW];
  __shared__ float red3[3][NW];
  const int k0 = blockIdx.x * KB, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool dok = 4 * lane < D;
  float4 acc[KB];
  float bsum[KB];
#pragma unroll
  for (int j = 0; j < KB; ++j) {
    acc[j] = float4{0.f, 0.f, 0.f, 0.f};
    bsum[j] = 0.f;
  }
  // RB rows per wave in flight at once (loads first, then the FMAs): a c5 rank's 320 rows are a few
  // batches, not one memory latency per 4 rows
  constexpr int RB = KB == 1 ? 16 : KB == 2 ? 10 : 6;
  for (int rb = w; rb < Bl; rb += NW * RB) {
    float dc[RB][KB], cv[RB][KB];
    float4 e[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int r = rb + NW * u;
      const bool ok = r < Bl;
      const long rr = ok ? r : 0;
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        dc[u][j] = ok ? dcos[rr * ldc + k0 + j] : 0.f;
        cv[u][j] = cos[rr * ldc + k0 + j];
      }
      e[u] = dok ? *reinterpret_cast<const float4*>(Ehat + rr * D + 4 * lane) : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < RB; ++u)
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        acc[j].x += dc[u][j] * e[u].x;
        acc[j].y += dc[u][j] * e[u].y;
        acc[j].z += dc[u][j] * e[u].z;
        acc[j].w += dc[u][j] * e[u].w;
        bsum[j] += dc[u][j] * cv[u][j];
      }
  }
#pragma unroll
  for (int j = 0; j < KB; ++j) {
    part[j][w][lane] = acc[j];
    if (lane == 0) bpart[j][w] = bsum[j];
  }
  __syncthreads();
  if (w < KB) {  // wave j sums speaker k0 + j's partials in wave order
    const int k = k0 + w;
    float4 t = part[w][0][lane];
#pragma unroll
    for (int i = 1; i < NW; ++i) {
      const float4 v = part[w][i][lane];
      t = float4{t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w};
    }
    if (k < N) {
      if (dok) *reinterpret_cast<float4*>(red_dchat + (long)k * D + 4 * lane) = t;
      if (lane == 0) {
        float b = 0.f;
#pragma unroll
        for (int i = 0; i < NW; ++i) b += bpart[w][i];
        red_beta[k] = b;
      }
    }
  }
  const int k = blockIdx.x;
  if (k == 0) {  // loss = sum per, dw, db: fixed-order block sums (block-uniform branch)
    float l = 0.f, a = 0.f, b = 0.f;
    for (int i = tid; i < Bl; i += 64 * NW) {
      l += per[i];
      a += dwdb_rows[i];
      b += dwdb_rows[Bl + i];
    }
    l = wave_sum(l);
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      red3[0][w] = l;
      red3[1][w] = a;
      red3[2][w] = b;
    }
    __syncthreads();
    if (tid == 0) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
      for (int i = 0; i < NW; ++i) {
        s0 += red3[0][i];
        s1 += red3[1][i];
        s2 += red3[2][i];
      }
      loss[0] = s0;
      dwdb[0] = s1;
      dwdb[1] = s2;
    }
  }
}

// can the fused 3-launch path run this shape?
extern "C" int sv_ge2e_train_ok(int N, int M, int D) {
  return N > 0 && N <= GF_NMAX && M >= 2 && M <= GF_MMAX && D > 0 && D <= GF_DMAX && D % 4 == 0;
}

// fused forward + backward of GE2ELoss for one GPU holding all N speakers (gloss = 1, the
// training step's): loss, per [N,M], dE [N,M,D], dwdb [2] = (dL/dw, dL/db)
extern "C" int sv_ge2e_train(const float* E, int N, int M, int D, const float* w, const float* b, float* loss,
                             float* per, float* dE, float* dwdb, float* workspace, hipStream_t stream) {
  if (!E || !w || !b || !loss || !per || !dE || !dwdb || !workspace) return SV_EARG;
  if (!sv_ge2e_train_ok(N, M, D)) return SV_ESHAPE;
  if (((uintptr_t)E | (uintptr_t)workspace) & 15) return SV_EALIGN;
  const Ge2eWs ws = carve(workspace, N, M, D, N);
  const int Bl = N * M, Np = (N + 3) & ~3;
  hipLaunchKernelGGL(ge2e_prep_kernel, dim3(N), dim3(256), 0, stream, E, M, D, ws.Chat, ws.Cn, ws.Ehat, ws.Uhat,
                     ws.En, ws.Un, ws.rawd, nullptr);
  SV_LAUNCH_CHECK();
  launch_rows(Bl, M, N, D, Np, 0, ws, w, b, per, stream);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_cols_kernel<false>, dim3(N, (D + 63) / 64), dim3(64 * GF_COLW), 0, stream, Bl, M, N, D, Np, ws.Chat, ws.Cn,
                     ws.Ehat, ws.Uhat, ws.En, ws.Un, ws.rawd, ws.cos, ws.dcos, ws.alpha, ws.dcd, ws.G1, per,
                     ws.dwdb_rows, dE, loss, dwdb, nullptr, nullptr);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// ---- the fused kernels in the speaker-sharded form (data parallel, sharded_ge2e.py) ----
// shard_prep: this shard's per-speaker sums (for the all-gather) and its rows' E^, U^, norms and
// diagonal cosines.  shard_rows: every speaker's C^ from the gathered sums, this shard's rows of
// the similarity matrix against all N (global speaker of local row r: spk_offset + r / M), the
// softmax and row backward, then per speaker k the shard's dC^_k and beta_k into the reduce
// buffer red [Np*D + N] (the caller SUM-all-reduces it) and the shard's loss / (dw, db)
// partials.  shard_finalize: this shard's dE from the reduced buffer.  The workspace carries the
// state between the three calls (sv_ge2e_workspace_size(N_local, M, D, N)).
extern "C" int sv_ge2e_shard_prep(const float* E, int N_local, int M, int D, float* ssum_local, float* workspace,
                                  hipStream_t stream) {
  if (!E || !ssum_local || !workspace || N_local <= 0) return SV_EARG;
  if (!sv_ge2e_train_ok(N_local, M, D)) return SV_ESHAPE;
  if (((uintptr_t)E | (uintptr_t)workspace | (uintptr_t)ssum_local) & 15) return SV_EALIGN;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N_local);
  hipLaunchKernelGGL(ge2e_prep_kernel, dim3(N_local), dim3(256), 0, stream, E, M, D, nullptr, nullptr, ws.Ehat, ws.Uhat,
                     ws.En, ws.Un, ws.rawd, ssum_local);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_shard_rows(int N_local, int M, int D, int spk_offset, int N, const float* ssum_all,
                                  const float* w, const float* b, float* per, float* red, float* loss_local,
                                  float* dwdb_local, float* workspace, hipStream_t stream) {
  if (!ssum_all || !w || !b || !per || !red || !loss_local || !dwdb_local || !workspace) return SV_EARG;
  if (!sv_ge2e_train_ok(N, M, D) || N_local <= 0 || spk_offset < 0 || spk_offset + N_local > N) return SV_ESHAPE;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N);
  const int Bl = N_local * M, Np = (N + 3) & ~3;
  if (rows_fuse_centroids(N, D) && Np == N) {  // (C^ formed inside the rows kernel)
    launch_rows(Bl, M, N, D, Np, spk_offset, ws, w, b, per, stream, ssum_all);
  } else {
    hipLaunchKernelGGL(ge2e_centroid_kernel, dim3(Np), dim3(256), 0, stream, ssum_all, N, M, D, ws.Chat, ws.Cn);
    SV_LAUNCH_CHECK();
    launch_rows(Bl, M, N, D, Np, spk_offset, ws, w, b, per, stream);
  }
  SV_LAUNCH_CHECK();
  // the padding rows of dC^ (speakers N .. Np-1) stay zero through the all-reduce
  if (Np > N) {
    hipError_t e = sv_memset0(red + (size_t)N * D, (size_t)(Np - N) * D * sizeof(float), stream);
    if (e != hipSuccess) return (int)e;
  }
  if (D <= 256)
    hipLaunchKernelGGL(ge2e_cols_partial_kernel<1>, dim3(N),
                       dim3(1024), 0, stream, Bl, N, D, Np, ws.Ehat, ws.cos, ws.dcos, per, ws.dwdb_rows, loss_local,
                       dwdb_local, red, red + (size_t)Np * D);
  else
    hipLaunchKernelGGL(ge2e_cols_kernel<true>, dim3(N, (D + 63) / 64), dim3(64 * GF_COLW), 0, stream, Bl, M, N, D, Np,
                       ws.Chat, ws.Cn, ws.Ehat, ws.Uhat, ws.En, ws.Un, ws.rawd, ws.cos, ws.dcos, ws.alpha, ws.dcd,
                       ws.G1, per, ws.dwdb_rows, nullptr, loss_local, dwdb_local, red, red + (size_t)Np * D);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_shard_finalize(int N_local, int M, int D, int spk_offset, int N, const float* red, float* dE,
                                      float* workspace, hipStream_t stream) {
  if (!red || !dE || !workspace || N_local <= 0 || M < 2 || D <= 0) return SV_EARG;
  const Ge2eWs ws = carve(workspace, N_local, M, D, N);
  const int Np = (N + 3) & ~3;
  launch_finalize(N_local, M, D, spk_offset, red, red + (size_t)Np * D, ws, ws.dcd, dE, stream);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// ============================================================================
// stand-alone forms of the reference helpers (utils.py): get_centroids, get_cossim
// with arbitrary (e.g. enrollment) centroids, calc_loss on a given similarity matrix.
// ============================================================================
__global__ void ge2e_scale_kernel(float* __restrict__ x, long n, float s) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= s;
}

// cos[r, k] += 1e-6 for all k; cos[r, s(r)] = rawd[r] + 1e-6 when s(r) < Nc
__global__ __launch_bounds__(256) void ge2e_cossim_fix_kernel(float* __restrict__ cos, const float* __restrict__ rawd,
                                                              int Bl, int M, int Nc) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int j = r / M;
  float* c = cos + (long)r * Nc;
  for (int k = lane; k < Nc; k += 64) c[k] = (k == j ? rawd[r] : c[k]) + EPS_SIM;
}

// calc_loss (utils.py:126-132) on S [N, M, K]: per[j,i] = log(sum_k e^S + 1e-6) - S[j,i,j]
__global__ __launch_bounds__(256) void ge2e_calc_loss_kernel(const float* __restrict__ S, int Bl, int M, int K,
                                                             float* __restrict__ per) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const float* s = S + (long)r * K;
  float mx = -INFINITY;
  for (int k = lane; k < K; k += 64) mx = fmaxf(mx, s[k]);
  mx = fmaxf(wave_max(mx), 0.f);
  float z = 0.f;
  for (int k = lane; k < K; k += 64) z += expf(s[k] - mx);
  z = wave_sum(z);
  if (lane == 0) per[r] = mx + logf(z + EPS_LOG * expf(-mx)) - s[r / M];
}

extern "C" int sv_ge2e_centroids(const float* E, int N, int M, int D, float* C, hipStream_t stream) {
  if (!E || !C || N <= 0 || M <= 0 || D <= 0) return SV_EARG;
  hipLaunchKernelGGL(ge2e_sums_kernel, dim3(N), dim3(256), 0, stream, E, M, D, C);
  SV_LAUNCH_CHECK();
  const long n = (long)N * D;
  hipLaunchKernelGGL(ge2e_scale_kernel, dim3((int)std::min<long>((n + 255) / 256, 1024)), dim3(256), 0, stream, C, n,
                     1.0f / (float)M);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" size_t sv_ge2e_cossim_workspace(int N, int M, int D, int Nc) {
  const size_t Bl = (size_t)N * M;
  size_t n = al((size_t)N * D) + 2 * al(Bl * D) + 3 * al(Bl) + al((size_t)Nc * D) + al(Nc);
  return n * sizeof(float) + sv_gemm_f32_workspace((int)Bl, Nc, D);
}

extern "C" int sv_ge2e_cossim(const float* E, int N, int M, int D, const float* C, int Nc, float* cos,
                              float* workspace, hipStream_t stream) {
  if (!E || !C || !cos || !workspace || N <= 0 || M < 2 || D <= 0 || D % 4 || Nc <= 0) return SV_EARG;
  const int Bl = N * M;
  float* p = workspace;
  float* ssum = p; p += al((size_t)N * D);
  float* Ehat = p; p += al((size_t)Bl * D);
  float* Uhat = p; p += al((size_t)Bl * D);
  float* En = p; p += al(Bl);
  float* Un = p; p += al(Bl);
  float* rawd = p; p += al(Bl);
  float* Chat = p; p += al((size_t)Nc * D);
  float* Cn = p; p += al(Nc);
  float* gws = p;
  hipLaunchKernelGGL(ge2e_sums_kernel, dim3(N), dim3(256), 0, stream, E, M, D, ssum);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_rowprep_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, E, ssum, Bl, M, D, 0, Ehat, Uhat,
                     En, Un, rawd);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_centroid_kernel, dim3(Nc), dim3(256), 0, stream, C, Nc, 1, D, Chat, Cn);
  SV_LAUNCH_CHECK();
  int rc = gemm_f32(1, 1, Bl, Nc, D, Ehat, D, Chat, D, cos, Nc, nullptr, nullptr, 0.f, gws, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(ge2e_cossim_fix_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, cos, rawd, Bl, M, Nc);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_calc_loss(const float* S, int N, int M, int K, float* per, float* loss, hipStream_t stream) {
  if (!S || !per || N <= 0 || M <= 0 || K < N) return SV_EARG;
  const int Bl = N * M;
  hipLaunchKernelGGL(ge2e_calc_loss_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, S, Bl, M, K, per);
  SV_LAUNCH_CHECK();
  if (loss) {
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, stream, per, Bl, loss);
    SV_LAUNCH_CHECK();
  }
  return SV_OK;
}

// ---------------------------------------------------------------------------
// Backward passes of the stand-alone helpers (the autograd graphs of utils.py:28, :72-115,
// :126-132), so a loss composed from them as in speech_embedder_net.py:45-48 trains.
// ---------------------------------------------------------------------------
// get_centroids: E.mean(1) -> dE[j,i,:] = dC[j,:] / M  (mean's backward divides by M)
__global__ void ge2e_centroids_bwd_kernel(const float* __restrict__ dC, int N, int M, int D, float* __restrict__ dE) {
  const long total = (long)N * M * D;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int d = (int)(e % D);
    const long j = e / ((long)M * D);
    dE[e] = dC[j * D + d] / (float)M;
  }
}

// get_cossim row pass, one wave per row r = (j, i): the upstream dcos row with the diagonal k = j
// taken out (the index_put overwrote cos[j, :, j], so C_j gets nothing from it) -> dcoff, its
// diagonal value -> dcd, the raw off-diagonal cosines (cosr, from the MFMA GEMM) with the
// diagonal replaced by the leave-one-out one -> alpha_r = sum_k dcos[r,k] cos_raw[r,k]
__global__ __launch_bounds__(256) void ge2e_cossim_bwd_rows_kernel(const float* __restrict__ dcos,
                                                                   const float* __restrict__ cosr,
                                                                   const float* __restrict__ rawd, int Bl, int M, int Nc,
                                                                   int ldc, float* __restrict__ dcoff,
                                                                   float* __restrict__ dcd, float* __restrict__ alpha) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int j = r / M;
  const float* g = dcos + (long)r * Nc;
  const float* c = cosr + (long)r * ldc;
  float* o = dcoff + (long)r * ldc;
  float a = 0.f;
  for (int k = lane; k < ldc; k += 64) {
    const float gk = k < Nc ? g[k] : 0.f;
    a += gk * (k == j ? rawd[r] : c[k]);
    o[k] = k == j ? 0.f : gk;
  }
  a = wave_sum(a);
  if (lane == 0) {
    alpha[r] = a;
    dcd[r] = g[j];
  }
}

// get_cossim, dE for one speaker per block (the finalize step without the centroid term):
//   dU_r = dcd_r (E^_r - raw_r U^_r [|U|>eps]) / max(|U_r|, eps)
//   dE_r = (G1_r + dcd_r U^_r - alpha_r E^_r [|E|>eps]) / max(|E_r|, eps) + (sum_i' dU_ji' - dU_r) / (M - 1)
__global__ __launch_bounds__(256) void ge2e_cossim_bwd_de_kernel(
    int M, int D, const float* __restrict__ Ehat, const float* __restrict__ Uhat, const float* __restrict__ En,
    const float* __restrict__ Un, const float* __restrict__ rawd, const float* __restrict__ dcd,
    const float* __restrict__ alpha, const float* __restrict__ G1, float* __restrict__ dE) {
  const int j = blockIdx.x;
  const float invm1 = 1.0f / (float)(M - 1);
  for (int d = threadIdx.x; d < D; d += 256) {
    float sumdU = 0.f;
    for (int i = 0; i < M; ++i) {
      const int r = j * M + i;
      const float iu = 1.0f / fmaxf(Un[r], EPS_COS);
      const float pu = Un[r] > EPS_COS ? 1.f : 0.f;
      sumdU += dcd[r] * (Ehat[(long)r * D + d] - rawd[r] * Uhat[(long)r * D + d] * pu) * iu;
    }
    for (int i = 0; i < M; ++i) {
      const int r = j * M + i;
      const long rd = (long)r * D + d;
      const float iu = 1.0f / fmaxf(Un[r], EPS_COS);
      const float pu = Un[r] > EPS_COS ? 1.f : 0.f;
      const float dU = dcd[r] * (Ehat[rd] - rawd[r] * Uhat[rd] * pu) * iu;
      const float ie = 1.0f / fmaxf(En[r], EPS_COS);
      const float pe = En[r] > EPS_COS ? 1.f : 0.f;
      dE[rd] = (G1[rd] + dcd[r] * Uhat[rd] - alpha[r] * Ehat[rd] * pe) * ie + (sumdU - dU) * invm1;
    }
  }
}

// get_cossim, dC_k = (dChat_k - beta_k C^_k [|C|>eps]) / max(|C_k|, eps), one centroid per block
__global__ __launch_bounds__(256) void ge2e_cossim_bwd_dc_kernel(int D, const float* __restrict__ dchat,
                                                                 const float* __restrict__ beta,
                                                                 const float* __restrict__ Chat,
                                                                 const float* __restrict__ Cn, float* __restrict__ dC) {
  const int k = blockIdx.x;
  const float cn = Cn[k];
  const float icn = 1.0f / fmaxf(cn, EPS_COS);
  const float pc = cn > EPS_COS ? 1.f : 0.f;
  for (int d = threadIdx.x; d < D; d += 256) {
    const long cd = (long)k * D + d;
    dC[cd] = (dchat[cd] - beta[k] * Chat[cd] * pc) * icn;
  }
}

// calc_loss backward, one wave per row: dS_k = g_r (e^{S_k - mx} / (z + 1e-6 e^{-mx}) - [k == j]),
// g_r = gloss + gper_r, with the forward's max shift (ge2e_calc_loss_kernel)
__global__ __launch_bounds__(256) void ge2e_calc_loss_bwd_kernel(const float* __restrict__ S, int Bl, int M, int K,
                                                                 const float* __restrict__ gloss,
                                                                 const float* __restrict__ gper, float* __restrict__ dS) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= Bl) return;
  const int j = r / M;
  const float* s = S + (long)r * K;
  float mx = -INFINITY;
  for (int k = lane; k < K; k += 64) mx = fmaxf(mx, s[k]);
  mx = fmaxf(wave_max(mx), 0.f);
  float z = 0.f;
  for (int k = lane; k < K; k += 64) z += expf(s[k] - mx);
  z = wave_sum(z);
  const float inv = 1.0f / (z + EPS_LOG * expf(-mx));
  const float g = (gloss ? *gloss : 0.f) + (gper ? gper[r] : 0.f);
  for (int k = lane; k < K; k += 64) dS[(long)r * K + k] = g * (expf(s[k] - mx) * inv - (k == j ? 1.f : 0.f));
}

extern "C" int sv_ge2e_centroids_bwd(const float* dC, int N, int M, int D, float* dE, hipStream_t stream) {
  if (!dC || !dE || N <= 0 || M <= 0 || D <= 0) return SV_EARG;
  const long n = (long)N * M * D;
  hipLaunchKernelGGL(ge2e_centroids_bwd_kernel, dim3((int)std::min<long>((n + 255) / 256, 4096)), dim3(256), 0, stream,
                     dC, N, M, D, dE);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

namespace {
struct CosBwdWs {
  float *ssum, *Ehat, *Uhat, *En, *Un, *rawd, *alpha, *dcd, *Chat, *Cn, *cosr, *dcoff, *G1, *dchat, *betap, *beta, *gemm;
  size_t total;
};
CosBwdWs carve_cos_bwd(float* base, int N, int M, int D, int Nc) {
  CosBwdWs w;
  const size_t Bl = (size_t)N * M;
  const int Ncp = (Nc + 3) & ~3;
  size_t off = 0;
  auto take = [&](size_t n) {
    float* p = base ? base + off : nullptr;
    off += al(n);
    return p;
  };
  w.ssum = take((size_t)N * D);
  w.Ehat = take(Bl * D);
  w.Uhat = take(Bl * D);
  w.En = take(Bl);
  w.Un = take(Bl);
  w.rawd = take(Bl);
  w.alpha = take(Bl);
  w.dcd = take(Bl);
  w.Chat = take((size_t)Ncp * D);
  w.Cn = take(Ncp);
  w.cosr = take(Bl * Ncp);
  w.dcoff = take(Bl * Ncp);
  w.G1 = take(Bl * D);
  w.dchat = take((size_t)Ncp * D);
  w.betap = take(((Bl + 63) / 64) * (size_t)Ncp);
  w.beta = take(Ncp);
  size_t g = sv_gemm_f32_workspace((int)Bl, Ncp, D);
  g = std::max(g, sv_gemm_f32_workspace((int)Bl, D, Ncp));
  g = std::max(g, sv_gemm_f32_workspace(Ncp, D, (int)Bl));
  w.gemm = take((g + 3) / 4);
  w.total = off * sizeof(float);
  return w;
}
}  // namespace

extern "C" size_t sv_ge2e_cossim_bwd_workspace(int N, int M, int D, int Nc) {
  return carve_cos_bwd(nullptr, N, M, D, Nc).total;
}

extern "C" int sv_ge2e_cossim_bwd(const float* E, int N, int M, int D, const float* C, int Nc, const float* dcos,
                                  float* dE, float* dC, float* workspace, hipStream_t stream) {
  if (!E || !C || !dcos || !dE || !dC || !workspace || N <= 0 || M < 2 || D <= 0 || D % 4 || Nc < N) return SV_EARG;
  const int Bl = N * M, Ncp = (Nc + 3) & ~3;
  const CosBwdWs ws = carve_cos_bwd(workspace, N, M, D, Nc);
  hipLaunchKernelGGL(ge2e_sums_kernel, dim3(N), dim3(256), 0, stream, E, M, D, ws.ssum);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_rowprep_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, E, ws.ssum, Bl, M, D, 0, ws.Ehat,
                     ws.Uhat, ws.En, ws.Un, ws.rawd);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_centroid_kernel, dim3(Ncp), dim3(256), 0, stream, C, Nc, 1, D, ws.Chat, ws.Cn);
  SV_LAUNCH_CHECK();
  // the raw cosines E^ C^T (padding columns zero)
  int rc = gemm_f32(1, 1, Bl, Ncp, D, ws.Ehat, D, ws.Chat, D, ws.cosr, Ncp, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(ge2e_cossim_bwd_rows_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, dcos, ws.cosr, ws.rawd, Bl,
                     M, Nc, Ncp, ws.dcoff, ws.dcd, ws.alpha);
  SV_LAUNCH_CHECK();
  // G1 = dcoff C^ ([Bl, Ncp] x [Ncp, D]);  dChat = dcoff^T E^ ([Ncp, Bl] x [Bl, D])
  rc = gemm_f32(1, 0, Bl, D, Ncp, ws.dcoff, Ncp, ws.Chat, D, ws.G1, D, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  rc = gemm_f32(0, 0, Ncp, D, Bl, ws.dcoff, Ncp, ws.Ehat, D, ws.dchat, D, nullptr, nullptr, 0.f, ws.gemm, stream);
  if (rc) return rc;
  const int nchunk = (Bl + 63) / 64;
  hipLaunchKernelGGL(ge2e_beta_partial_kernel, dim3((Nc + 63) / 64, nchunk), dim3(256), 0, stream, ws.dcoff, ws.cosr,
                     Bl, Nc, Ncp, ws.betap);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_beta_final_kernel, dim3((Nc + 255) / 256), dim3(256), 0, stream, ws.betap, nchunk, Nc,
                     ws.beta);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_cossim_bwd_de_kernel, dim3(N), dim3(256), 0, stream, M, D, ws.Ehat, ws.Uhat, ws.En, ws.Un,
                     ws.rawd, ws.dcd, ws.alpha, ws.G1, dE);
  SV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ge2e_cossim_bwd_dc_kernel, dim3(Nc), dim3(256), 0, stream, D, ws.dchat, ws.beta, ws.Chat, ws.Cn,
                     dC);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

extern "C" int sv_ge2e_calc_loss_bwd(const float* S, int N, int M, int K, const float* gloss, const float* gper,
                                     float* dS, hipStream_t stream) {
  if (!S || !dS || N <= 0 || M <= 0 || K < N) return SV_EARG;
  const int Bl = N * M;
  hipLaunchKernelGGL(ge2e_calc_loss_bwd_kernel, dim3((Bl + 3) / 4), dim3(256), 0, stream, S, Bl, M, K, gloss, gper, dS);
  SV_LAUNCH_CHECK();
  return SV_OK;
}

// ============================================================================
// EER threshold sweep (train_speech_embedder.py:134-149): for each threshold, the number of
// similarities above it (all entries and the diagonal k == j).  One block per threshold;
// integer counts, so the result is exact.
// ============================================================================
__global__ __launch_bounds__(256) void eer_counts_kernel(const float* __restrict__ S, int N, int M2, int Nc,
                                                         const float* __restrict__ thr, float* __restrict__ cnt_all,
                                                         float* __restrict__ cnt_diag) {
  __shared__ int red[2][4];
  const float th = thr[blockIdx.x];
  const long total = (long)N * M2 * Nc;
  int a = 0, d = 0;
  for (long e = threadIdx.x; e < total; e += 256) {
    const int k = (int)(e % Nc);
    const int j = (int)(e / ((long)M2 * Nc));
    const int over = S[e] > th;
    a += over;
    d += (over && k == j);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    d += __shfl_xor(d, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt_all[blockIdx.x] = (float)(red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    cnt_diag[blockIdx.x] = (float)(red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

extern "C" int sv_eer_counts(const float* S, int N, int M2, int Nc, const float* thresholds, int n_thr,
                             float* cnt_all, float* cnt_diag, hipStream_t stream) {
  if (!S || !thresholds || !cnt_all || !cnt_diag || N <= 0 || M2 <= 0 || Nc < N || n_thr <= 0) return SV_EARG;
  hipLaunchKernelGGL(eer_counts_kernel, dim3(n_thr), dim3(256), 0, stream, S, N, M2, Nc, thresholds, cnt_all, cnt_diag);
  SV_LAUNCH_CHECK();
  return SV_OK;
}
