// Large-batch d-vector inference (dvector_create.py:96-101: every 24-frame window of a file through
// SpeechEmbedder.forward, speech_embedder_net.py:27-33), bf16 operands / fp32 accumulation and state
// as the c3 forward.  At thousands of windows the recurrence is a sequence of large GEMMs
// (B = 16384: 77 GFLOP of recurrent products per step and layer), so instead of W-stationary
// persistent workgroups (whose grid has to be co-resident: at most ~640 rows) each timestep of each
// layer is ONE launch of the 256 x 256 8-phase bf16 GEMM (sv_gemm256.h, gemm_bf16_8q_kernel's
// schedule) over the concatenated contraction [x_t | h_{t-1}] . [W_ih | W_hh]^T with the LSTM cell
// in its epilogue:
//   * W rows interleaved by unit (row 4 j + q = gate q of unit j), so the 8-phase accumulator of a
//     lane -- acc[mt][nt] = C[row 16 mt + (lane & 15)][cols 16 nt + 4 (lane >> 4) .. + 3] -- holds
//     the four gates i, f, g, o of ONE (row, unit) in one f32x4: the cell needs no exchange;
//   * the x part of K first; at its end the accumulators become bf16(x W_ih^T + b_ih + b_hh) (the
//     c3 path's K1 rounding of the input projection), then the h part adds h_{t-1} W_hh^T;
//   * the cell state c stays in a fragment-order buffer (each lane's 32 values as 8 x 16 B,
//     coalesced), h_t goes out as bf16 rows through LDS (16-B stores): the next step's A operand
//     and the next layer's x operand; the last layer's h_{T-1} also in fp32 (the projection's input).
// No K1 GEMM and no x-projection round trip through HBM.
#include "sv_gemm256.h"
#include "../../include/sv_ge2e.h"

namespace {
struct DvecStep {
  const bf16_t* ax;  // [B][ldx] layer input at step t (x padded to Kx, or the lower layer's h_t)
  long ldx;
  int nkx;           // k-tiles of the x part
  const bf16_t* ah;  // [B][H] h_{t-1} (NULL at t = 0: no h part)
  const bf16_t* w;   // [4H][Kx + H] interleaved W
  long ldw;
  const float* bsum;  // [4H] interleaved b_ih + b_hh
  float* cst;         // fragment-order cell state
  bf16_t* hout;       // [B][H] h_t
  float* hlast;       // [B][H] fp32 h_t (last step of the last layer) or NULL
  int H;
  int first;  // t == 0: c_{t-1} = 0
};
}  // namespace

// LAST: the last step of the last layer, which also writes h_{T-1} in fp32 (p.hlast)
template <bool LAST>
__global__ __launch_bounds__(512, 1) void lstm_dvec_step_bf16_kernel(const DvecStep p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int N = 4 * p.H, tiles_n = N / G256_BM;
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int nkh = p.ah ? p.H / G256_BK : 0;
  const int nk = p.nkx + nkh;
  const int wr = w >> 2, wc = w & 3;
  G256Stage sx, sh, sb;
  sx.init(p.ax, p.ldx, tm * G256_BM, 0, tid);
  if (p.ah) sh.init(p.ah, p.H, tm * G256_BM, 0, tid);
  sb.init(p.w, p.ldw, tn * G256_BM, 0, tid);
  constexpr int OPB = G256_BM * G256_BK * 2;
  auto stage = [&](int kt) { return smem + (kt & 1) * 2 * OPB; };
  auto fill_a = [&](int kt, int i) {
    const bf16_t* src = kt < p.nkx ? sx.src[i] + kt * G256_BK : sh.src[i] + (kt - p.nkx) * G256_BK;
    __builtin_amdgcn_global_load_lds((glb_vptr_t)src, (lds_vptr_t)(stage(kt) + (w * 64 + 512 * i) * 16), 16, 0, 0);
  };
  auto fill_b = [&](int kt, int i) {
    __builtin_amdgcn_global_load_lds((glb_vptr_t)(sb.src[i] + kt * G256_BK),
                                     (lds_vptr_t)(stage(kt) + OPB + (w * 64 + 512 * i) * 16), 16, 0, 0);
  };
  auto read_a = [&](const char* As, int mt, int ks) -> bf16x8_t {
    const int row = wr * 128 + 16 * mt + fr;
    return *reinterpret_cast<const bf16x8_t*>(As + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
  };
  auto read_b = [&](const char* Bs, int nt, int ks) -> bf16x8_t {
    const int row = wc * 64 + 16 * nt + fr;
    return *reinterpret_cast<const bf16x8_t*>(Bs + row * 128 + g256_phys_slot(row, 4 * ks + fq) * 16);
  };
  g8_f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = g8_f32x4{0.f, 0.f, 0.f, 0.f};
  // the biases of this lane's 16 gate columns, loaded before the fills (a load inside the k-loop
  // would wait, in the in-order vmcnt, for every fill in flight)
  g8_f32x4 bs[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
    bs[nt] = *reinterpret_cast<const g8_f32x4*>(p.bsum + tn * G256_BM + wc * 64 + 16 * nt + 4 * fq);
  // the 8-phase schedule of gemm_bf16_8q_kernel (sv_gemm256.h: fills two per phase, counted waits,
  // the two wave groups one barrier apart)
#pragma unroll
  for (int i = 0; i < 4; ++i) fill_b(0, i);
#pragma unroll
  for (int i = 0; i < 4; ++i) fill_a(0, i);
  if (nk > 1) {
    fill_a(1, 0);
    fill_a(1, 2);
    fill_b(1, 0);
    fill_b(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (wr == 1) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  bf16x8_t a[4][2], b0[2][2], b1[2][2];
  auto mma = [&](int mh, int nh, const bf16x8_t (&bq)[2][2]) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 * mh + i][2 * nh + j] = mfma16_bf16(bq[j][ks], a[i][ks], acc[4 * mh + i][2 * nh + j]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int kt = 0; kt < nk; ++kt) {
    const char* As = stage(kt);
    const char* Bs = As + OPB;
    const bool m1 = kt + 1 < nk, m2 = kt + 2 < nk;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b0[j][ks] = read_b(Bs, j, ks);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, i, ks);
    if (m1) {
      fill_b(kt + 1, 2);
      fill_b(kt + 1, 3);
    }
    mma(0, 0, b0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) b1[j][ks] = read_b(Bs, 2 + j, ks);
    if (m1)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (m1) fill_a(kt + 1, 1);
    if (m2) fill_a(kt + 2, 0);
    mma(0, 1, b1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a[i][ks] = read_a(As, 4 + i, ks);
    if (m1) fill_a(kt + 1, 3);
    if (m2) fill_a(kt + 2, 2);
    mma(1, 1, b1);
    if (m2)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (m1)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (m2) {
      fill_b(kt + 2, 0);
      fill_b(kt + 2, 1);
    }
    mma(1, 0, b0);
    if (kt + 1 == p.nkx) {
      // the x part is complete: bf16(x W_ih^T + (b_ih + b_hh)), as the c3 path's K1 stores it
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          const g8_f32x4 v = acc[mt][nt] + bs[nt];
          acc[mt][nt] = g8_f32x4{round_bf(v[0]), round_bf(v[1]), round_bf(v[2]), round_bf(v[3])};
        }
      }
    }
  }
  if (wr == 0) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- the cell: lane (fr, fq), accumulator (mt, nt) = gates i, f, g, o of row 16 mt + fr, unit
  // 16 wc + 4 nt + fq of this tile's 64 units; c_{t-1} / c_t in the fragment-order state
  float4* cw = reinterpret_cast<float4*>(p.cst) + ((long)(id * 8 + w) * 8) * 64 + lane;  // + mt * 64
  char* tile = smem + w * 4096;  // [128 rows][16 units] bf16, after every wave's last stage read
  __syncthreads();
  const int ug = tn * 64 + wc * 16;  // first unit of this wave's 16
  // all eight c_{t-1} loads in flight at once, unconditionally (a load per branch waited for each;
  // at t = 0 the state is not yet written and the loaded values are discarded)
  float4 cps[8];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) cps[mt] = cw[mt * 64];
  const bool first = p.first;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const float4 cp = first ? float4{0.f, 0.f, 0.f, 0.f} : cps[mt];
    float cn[4], hn[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float pv[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
      const float zx[4] = {0.f, 0.f, 0.f, 0.f};
      float av[4];
      const float cprev = nt == 0 ? cp.x : nt == 1 ? cp.y : nt == 2 ? cp.z : cp.w;
      cn[nt] = lstm_cell_fwd(pv, zx, cprev, av, hn[nt]);
      *reinterpret_cast<bf16_t*>(tile + (16 * mt + fr) * 32 + (4 * nt + fq) * 2) = to_bf(hn[nt]);
      if constexpr (LAST) p.hlast[((long)tm * G256_BM + wr * 128 + 16 * mt + fr) * p.H + ug + 4 * nt + fq] = hn[nt];
    }
    cw[mt * 64] = float4{cn[0], cn[1], cn[2], cn[3]};
  }
  // h_t rows: 128 x 32 B per wave = 4 KB, 16 B per lane per store (the same wave reads its tile)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 64 + lane, row = q >> 1, hf = q & 1;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + row * 32 + hf * 16);
    *reinterpret_cast<uint4*>(p.hout + ((long)tm * G256_BM + wr * 128 + row) * p.H + ug + 8 * hf) = v;
  }
}

// ---- host side ----
namespace {
constexpr int DV_KX0 = 64;  // layer 0's x part: F features padded to one k-tile

// W_cat [4H][Kx + H] bf16, row 4 j + q = [W_ih[q H + j][0 .. F) (zero past F) | W_hh[q H + j]]
__global__ void dvec_weights_kernel(const float* __restrict__ w_ih, const float* __restrict__ w_hh, int F, int Kx,
                                    int H, bf16_t* __restrict__ wcat, const float* __restrict__ b_ih,
                                    const float* __restrict__ b_hh, float* __restrict__ bsum) {
  const int r = blockIdx.x, j = r >> 2, q = r & 3, src = q * H + j;
  const int ld = Kx + H;
  for (int k = threadIdx.x; k < ld; k += blockDim.x) {
    const float v = k < Kx ? (k < F ? w_ih[(long)src * F + k] : 0.f) : w_hh[(long)src * H + (k - Kx)];
    wcat[(long)r * ld + k] = to_bf(v);
  }
  if (threadIdx.x == 0) bsum[r] = (b_ih ? b_ih[src] : 0.f) + (b_hh ? b_hh[src] : 0.f);
}
// x [B][T][F] fp32 (batch-first windows) -> xpad [T][B][Kx] bf16 (zeros past F and past B)
__global__ void dvec_x_kernel(const float* __restrict__ x, int B, int Bp, int T, int F, int Kx,
                              bf16_t* __restrict__ xpad) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)T * Bp * Kx;
  if (i >= n) return;
  const int k = (int)(i % Kx);
  const long tb = i / Kx;
  const int b = (int)(tb % Bp), t = (int)(tb / Bp);
  xpad[i] = (b < B && k < F) ? to_bf(x[((long)b * T + t) * F + k]) : (bf16_t)0;
}
size_t align256(size_t n) { return (n + 255) & ~size_t(255); }
}  // namespace

extern "C" size_t sv_dvector_bf16_workspace(int B, int T, int F, int H, int L, int P) {
  const size_t Bp = ((size_t)B + 255) / 256 * 256;
  size_t n = align256(Bp * T * DV_KX0 * 2);                                        // xpad
  n += 2 * align256((size_t)(T + 1) * Bp * H * 2);                                 // h ping-pong [T + 1][Bp][H]
  n += align256(Bp * H * 4);                                                       // cell state
  n += align256(Bp * H * 4);                                                       // h_{T-1} fp32
  n += (size_t)L * (align256((size_t)4 * H * (H + (size_t)H) * 2) + align256((size_t)4 * H * 4));  // W_cat, bsum
  n += align256((size_t)B * P * 4) + align256((size_t)B * 4) + align256(sv_proj_norm_workspace(B, H, P));
  (void)F;
  return n;
}

// embeddings of B windows x [B][T][F] (fp32, batch-first; F <= 64, H % 64 == 0, 4H % 256 == 0):
// layers[l] = (w_ih [4H][F_l], w_hh [4H][H], b_ih, b_hh) fp32; projection w_p [P][H], b_p [P];
// emb [B][P] = normalize(h_{T-1} w_p^T + b_p).  workspace: sv_dvector_bf16_workspace bytes.
extern "C" int sv_dvector_embed_bf16(int B, int T, int F, int H, int L, const float* x, const float* const* w_ih,
                                     const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                                     const float* w_p, const float* b_p, int P, float* emb, void* workspace,
                                     hipStream_t stream) {
  if (B <= 0 || T <= 0 || L <= 0 || F <= 0 || F > DV_KX0 || H % G256_BK || (4 * H) % G256_BM || !x || !w_ih ||
      !w_hh || !w_p || !emb || !workspace)
    return SV_EARG;
  if ((uintptr_t)workspace & 255) return SV_EALIGN;
  const int Bp = (B + 255) / 256 * 256;
  char* ws = static_cast<char*>(workspace);
  bf16_t* xpad = reinterpret_cast<bf16_t*>(ws);
  ws += align256((size_t)Bp * T * DV_KX0 * 2);
  bf16_t* hbuf[2];
  for (int i = 0; i < 2; ++i) {
    hbuf[i] = reinterpret_cast<bf16_t*>(ws);
    ws += align256((size_t)(T + 1) * Bp * H * 2);
  }
  float* cst = reinterpret_cast<float*>(ws);
  ws += align256((size_t)Bp * H * 4);
  float* hlast = reinterpret_cast<float*>(ws);
  ws += align256((size_t)Bp * H * 4);
  hipLaunchKernelGGL(dvec_x_kernel, dim3((unsigned)(((long)T * Bp * DV_KX0 + 255) / 256)), dim3(256), 0, stream, x, B,
                     Bp, T, F, DV_KX0, xpad);
  SV_LAUNCH_CHECK();
  const size_t lds = G256_LDS;
  const int grid = (Bp / G256_BM) * (4 * H / G256_BM);
  for (int l = 0; l < L; ++l) {
    if (!w_ih[l] || !w_hh[l]) return SV_EARG;
    const int Fl = l == 0 ? F : H, Kx = l == 0 ? DV_KX0 : H;
    bf16_t* wcat = reinterpret_cast<bf16_t*>(ws);
    ws += align256((size_t)4 * H * (H + (size_t)H) * 2);
    float* bsum = reinterpret_cast<float*>(ws);
    ws += align256((size_t)4 * H * 4);
    hipLaunchKernelGGL(dvec_weights_kernel, dim3(4 * H), dim3(256), 0, stream, w_ih[l], w_hh[l], Fl, Kx, H, wcat,
                       b_ih ? b_ih[l] : nullptr, b_hh ? b_hh[l] : nullptr, bsum);
    SV_LAUNCH_CHECK();
    bf16_t* hin = hbuf[(l + 1) & 1];  // the layer below's h_1 .. h_T (slots 1 .. T)
    bf16_t* hl = hbuf[l & 1];         // this layer's h_t in slot t + 1
    for (int t = 0; t < T; ++t) {
      DvecStep s{};
      s.ax = l == 0 ? xpad + (size_t)t * Bp * DV_KX0 : hin + (size_t)(t + 1) * Bp * H;
      s.ldx = Kx;
      s.nkx = Kx / G256_BK;
      s.ah = t > 0 ? hl + (size_t)t * Bp * H : nullptr;
      s.w = wcat;
      s.ldw = Kx + H;
      s.bsum = bsum;
      s.cst = cst;
      s.hout = hl + (size_t)(t + 1) * Bp * H;
      s.hlast = (l == L - 1 && t == T - 1) ? hlast : nullptr;
      s.H = H;
      s.first = t == 0;
      if (s.hlast)
        hipLaunchKernelGGL(lstm_dvec_step_bf16_kernel<true>, dim3(grid), dim3(512), lds, stream, s);
      else
        hipLaunchKernelGGL(lstm_dvec_step_bf16_kernel<false>, dim3(grid), dim3(512), lds, stream, s);
      SV_LAUNCH_CHECK();
    }
  }
  // projection + L2 norm of h_{T-1} (fp32), the training path's sv_proj_norm_fwd
  float* y = reinterpret_cast<float*>(ws);
  ws += align256((size_t)B * P * 4);
  float* ynorm = reinterpret_cast<float*>(ws);
  ws += align256((size_t)B * 4);
  return sv_proj_norm_fwd(hlast, B, H, P, w_p, b_p, y, emb, ynorm, reinterpret_cast<float*>(ws), stream);
}
