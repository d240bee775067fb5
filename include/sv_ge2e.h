/* C ABI of libsv_ge2e.so -- the MI355X (gfx950) GE2E speaker-embedding training path.
 *
 * The reference (hwidong-na/PyTorch_Speaker_Verification) is pure Python over PyTorch and
 * has no FFI of its own; each entry point below replaces the device work PyTorch launches
 * implicitly at the cited reference line (SURVEY.md §2 "implicit op" table, §8 b).
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-owned, contiguous, row-major DEVICE buffer (fp32), 16-byte
 *     aligned; scalars such as w, b, gloss are device pointers to one float (no host sync);
 *   - nothing is allocated, no global state is kept, no pointer is retained after return;
 *     scratch comes from a caller workspace of the size the matching *_workspace* returns;
 *     modes are explicit arguments (`products`, `schedule`; the library reads no environment
 *     variables), cross-workgroup counters live in a caller sync block (sv_sync_size), so calls
 *     with distinct buffers may run concurrently;
 *   - every launch goes to `stream` (pass the current stream of the tensor's device: the
 *     *_bwd functions are called from the autograd engine's worker thread);
 *   - return 0 on success, a hipError_t (> 0) from a failed launch, or a negative
 *     argument error (SV_EARG -1, SV_EALIGN -2, SV_ESHAPE -3).  Functions are reentrant.
 */
#ifndef SV_GE2E_H
#define SV_GE2E_H

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SV_ABI_VERSION 11
int sv_abi_version(void);

/* ---- fp32 product modes (`products` argument of sv_gemm_f32 / sv_lstm_stack_fwd / _bwd; every
 * other fp32 entry point runs mode 0):
 *   0 exact fp32 MFMA products (v_mfma_f32_32x32x2_f32);
 *   1 "bf16x6": each fp32 operand split into three bf16 terms, six bf16 MFMA products per fp32
 *     product, fp32 accumulation -- products carried to ~2^-25 relative, measured GEMM error vs
 *     fp64 at or below the exact-MFMA path's (scripts/emu_check.py) -- on the NT GEMMs and K2;
 *   2 / 3 diagnostics (split at LDS store / in registers everywhere). */
#define SV_F32_EXACT 0
#define SV_F32_BF16X6 1

/* ---- schedule flags (`schedule` argument of the stack entry points; 0 = the measured default).
 * fp32 (sv_lstm_stack_fwd / _bwd): the W-stationary persistent recurrences (one launch per layer,
 * W_hh in registers, H = 768) under SV_SCHED_AUTO where their grid fills >= 3/4 of the device and
 * under SV_SCHED_PERSIST wherever it fits; SV_SCHED_PER_STEP keeps the layer-pipelined per-step
 * kernels (K2 / K3).  The two agree to fp32 rounding (different summation order).
 * bf16 (sv_lstm_stack_fwd_bf16 / _bwd_bf16):
 *   SV_SCHED_AUTO       the layer wavefront (all layers in one launch) where every layer's grid
 *                       fits co-resident, else one persistent recurrence launch per layer at
 *                       H = 768, else per-step launches;
 *   SV_SCHED_PER_LAYER  never the layer wavefront (it sums the upper layers' products in another
 *                       order: results agree at bf16 level, not bit for bit);
 *   SV_SCHED_PER_STEP   per-step launches, layer-pipelined over the side streams (bit-identical
 *                       to the persistent per-layer schedule);
 *   SV_SCHED_PERSIST    persistent per-layer recurrences for any H they support (64, 96, 768),
 *                       not only H = 768.
 * Both precisions:
 *   SV_SCHED_NO_EVENTS  (ABI v9) the stack backward's persistent / wavefront schedules record no
 *                       per-layer completion events into `ev` (set it when nothing waits on them,
 *                       i.e. no data-parallel gradient buckets: each event record leaves the GPU
 *                       idle for ~6 us between two kernels); the per-step schedule, whose side
 *                       streams synchronise through the events, ignores it.
 * bf16 stack backward only:
 *   SV_SCHED_WT_READY   (ABI v10) the workspace already holds the bf16 weight transposes, written by
 *                       sv_lstm_weights_bf16 (below) from the same weights into the same workspace:
 *                       no transpose launch (the fp32 backward ignores it).
 *   SV_SCHED_CNT_READY  (ABI v11) the sync block's backward counter channels are still as the last
 *                       bf16 stack forward on it left them (it zeroes them) -- no backward has run
 *                       on the block since: the persistent / wavefront backward launches no
 *                       counter zeroing (the caller tracks this; passing it wrongly makes the
 *                       hand-off waits pass early). */
#define SV_SCHED_AUTO 0
#define SV_SCHED_PER_LAYER 1
#define SV_SCHED_PER_STEP 2
#define SV_SCHED_PERSIST 4
#define SV_SCHED_NO_EVENTS 8
#define SV_SCHED_WT_READY 16
#define SV_SCHED_CNT_READY 32
#define SV_SCHED_MASK 63

/* ---- dense fp32 MFMA GEMM (used by every op below; exported for tests) -----------------
 * C[M,N] = op(A) op(B) (+ bias0[n] + bias1[n]) (+ beta C).
 * a_kcontig: A element (m,k) at A[m*lda+k], else at A[k*lda+m].
 * b_kcontig: B element (k,n) at B[n*ldb+k], else at B[k*ldb+n].  */
size_t sv_gemm_f32_workspace(int M, int N, int K);
int sv_gemm_f32(int a_kcontig, int b_kcontig, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                float* C, long ldc, const float* bias0, const float* bias1, float beta, float* workspace,
                int products, hipStream_t stream);

/* column sums of X[R,C] (deterministic two-level reduction) */
size_t sv_colsum_workspace(int R, int C);
int sv_colsum(const float* X, int R, int C, float* out, float* workspace, hipStream_t stream);

/* ---- SpeechEmbedder LSTM stack (replaces nn.LSTM fwd, speech_embedder_net.py:19,28, and its
 * autograd backward via train_speech_embedder.py:62).  Time-major layouts:
 *   x_tm [T,B,F], gates [T,B,4H] (activated i,f,g,o), c_tm [T,B,H], h_tm [T+1,B,H] (h_tm[0]=0). */
int sv_frames_to_time_major(const float* x, float* x_tm, int B, int T, int F, hipStream_t stream);
/* dst[c*ld_dst + r] = src[r*ld_src + c] for an R x C matrix */
int sv_transpose(const float* src, long ld_src, int R, int C, float* dst, long ld_dst, hipStream_t stream);
/* Transposed layouts use column blocks of Bp = (B + 3) & ~3 (padding columns zero).
 * hT [H, (T+1)Bp] (may be NULL): h_t^T as column block t+1, block 0 = 0 -- the k-contiguous
 * operand of the weight-gradient GEMMs (block t = h_{t-1}) and of the next layer's dW_ih. */
int sv_lstm_layer_fwd(const float* x_tm, int T, int B, int F, int H, const float* w_ih, const float* w_hh,
                      const float* b_ih, const float* b_hh, float* gates, float* c_tm, float* h_tm, float* hT,
                      hipStream_t stream);
/* one forward recurrent step (K2): on entry gates_t [B,4H] = x_t W_ih^T + b_ih + b_hh, on exit the
 * activated gates; h_prev / c_prev may be NULL (t = 0). */
int sv_lstm_step_fwd(const float* h_prev, const float* w_hh, float* gates_t, const float* c_prev, float* c_t,
                     float* h_t, int B, int H, hipStream_t stream);
/* one backward recurrent step (K3): dg_t [B,4H] = dL/d(gates_t) from dg_next [B,4H] (NULL at
 * t = T-1), W_hh^T [H,4H], dh_up [B,H] (may be NULL), dcf_next = dc_{t+1} f_{t+1} (may be NULL),
 * the activated gates, c_t, c_{t-1} (NULL at t = 0); writes dcf_t = dc_t f_t. */
int sv_lstm_step_bwd(const float* dg_next, const float* w_hhT, const float* dh_up, const float* dcf_next,
                     const float* acts_t, const float* c_t, const float* c_prev, float* dg_t, float* dcf_t, int B,
                     int H, hipStream_t stream);
/* Whole stack.  Per-step schedule: layer-pipelined over streams, layer l on side[l] in chunks of
 * `chunk` timesteps (chunk input-projection GEMM, then its steps), waiting only for layer l-1's
 * same chunk, so the layers' kernels overlap.  Persistent schedule (`schedule`, above): per layer on
 * `main`, the whole-T input projection, then one persistent recurrence launch (needs `sync`, the
 * caller's sync block below; probe (may be NULL): 2*L caller events recorded around layer l's
 * launch, probe[2l] before, [2l+1] after).  Per-layer pointers come in host arrays of length L
 * (layer 0 input width F, others H); ev = L*ceil(T/chunk)+1 caller-created events.  Starts after
 * and joins back into `main` (all work ordered before the next op on `main`). */
int sv_lstm_stack_fwd(int L, int T, int B, int F, int H, const float* x_tm, const float* const* w_ih,
                      const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                      float* const* gates, float* const* c_tm, float* const* h_tm, float* const* hT, int chunk,
                      hipStream_t main, const hipStream_t* side, hipEvent_t* ev, int products, int schedule,
                      unsigned* sync, hipEvent_t* probe);
/* 1 if the fp32 stack functions take the persistent recurrences for this batch under `schedule`
 * on the current device */
int sv_lstm_f32_persist_ok(int B, int H, int schedule);
size_t sv_lstm_layer_bwd_workspace(int T, int B, int F, int H);
/* Whole-stack backward (top layer first).  Per-step schedule, layer-pipelined over streams: each
 * layer's reverse chunks of steps on side[l], then (l > 0) the chunk's dx = dG W_ih GEMM that feeds
 * layer l-1; then the layer's whole-T dW_hh / dW_ih GEMMs and bias row sums on side[l].  side: L
 * streams.  Persistent schedule (`schedule`, `sync` as sv_lstm_stack_fwd): per layer on `main`, one
 * persistent recurrence launch (probe[2l] / [2l+1] around it; kstamp unused), then the whole-T dx,
 * dW GEMMs and row sums; ev[L*nch + l] recorded after layer l's gradients.
 * xT/ld_xT: per-layer transposed inputs; dx[l] [T,B,H] for l > 0;
 * ev = L*ceil(T/chunk) + L + 1 caller events (ev[L*nch + l] = layer l's gradients done);
 * joins back into `main`.  probe (may be NULL): 2*L*ceil(T/chunk) caller events recorded on the
 * layer's stream around ONE recurrent-step (K3) launch of each chunk (its second),
 * probe[2(l nch + c)] before, [+1] after (stream view: includes any wait for CUs); kstamp (may be
 * NULL): 2*L*T u64, each pair preset by the caller to {UINT64_MAX, 0}, which K3 launch (l, t)
 * sets to its first-workgroup start / last-workgroup end on the GPU's 100 MHz real-time clock
 * (the kernel's own execution span, as a profiler measures it) -- the bench's in-step roofline. */
size_t sv_lstm_stack_bwd_workspace(int L, int T, int B, int F, int H);
int sv_lstm_stack_bwd(int L, int T, int B, int F, int H, const float* const* xT, const long* ld_xT,
                      const float* const* w_ih, const float* const* w_hh, const float* const* gates,
                      const float* const* c_tm, const float* const* hT, const float* dh_last, float* const* dgates,
                      float* const* dgT, float* const* dx, float* const* dw_ih, float* const* dw_hh,
                      float* const* db_ih, float* const* db_hh, float* workspace, int chunk, hipStream_t main,
                      const hipStream_t* side, hipEvent_t* ev, int products, hipEvent_t* probe,
                      unsigned long long* kstamp, int schedule, unsigned* sync);
/* xT: the layer input transposed, [F, >= T*Bp] with row stride ld_xT (layer 0: the frames;
 * layer l > 0: hT of layer l-1 offset by Bp columns).  hT: this layer's [H, (T+1)Bp] from the fwd.
 * dh_up: gradient w.r.t. this layer's outputs; dh_up_full=1 -> [T,B,H], 0 -> [B,H] for t=T-1 only.
 * Outputs dgates [T,B,4H], dgT [4H, T*Bp] (its transpose), dx_tm [T,B,F] (may be NULL),
 * dw_ih [4H,F], dw_hh [4H,H], db_ih [4H] and db_hh [4H] (may be NULL; both = sum dgates). */
int sv_lstm_layer_bwd(int T, int B, int F, int H, const float* xT, long ld_xT, const float* w_ih, const float* w_hh,
                      const float* gates, const float* c_tm, const float* hT, const float* dh_up, int dh_up_full,
                      float* dgates, float* dgT, float* dx_tm, float* dw_ih, float* dw_hh, float* db_ih,
                      float* db_hh, float* workspace, hipStream_t stream);

/* ---- projection + L2 norm (speech_embedder_net.py:30-32) --------------------------------- */
size_t sv_proj_norm_workspace(int B, int H, int P);
int sv_proj_norm_fwd(const float* h_last, int B, int H, int P, const float* w_p, const float* b_p, float* y,
                     float* emb, float* ynorm, float* workspace, hipStream_t stream);
int sv_proj_norm_bwd(const float* demb, const float* emb, const float* ynorm, const float* h_last, int B, int H, int P,
                     const float* w_p, float* dw_p, float* db_p, float* dh_last, float* workspace,
                     hipStream_t stream);

/* ---- GE2E loss (speech_embedder_net.py:43-49; utils.py:27-132) -----------------------------
 * E is the local block [N_local, M, D] of a batch of N speakers; its first speaker is global
 * speaker spk_offset.  ssum_all [N,D] = per-speaker sums (all-gathered when sharded).
 * D % 4 == 0 and M >= 2.  dchat buffers are [Np, D] with Np = (N + 3) & ~3.
 * The workspace carries state from fwd to bwd: keep it alive and untouched in between. */
size_t sv_ge2e_workspace_size(int N_local, int M, int D, int N);
int sv_ge2e_speaker_sums(const float* E, int N_local, int M, int D, float* ssum_local, hipStream_t stream);
int sv_ge2e_fwd_rows(const float* E, int N_local, int M, int D, int spk_offset, int N, const float* ssum_all,
                     const float* w, const float* b, float* per, float* loss_local, float* workspace,
                     hipStream_t stream);
int sv_ge2e_fwd(const float* E, int N, int M, int D, const float* w, const float* b, float* loss, float* per,
                float* workspace, float* ssum, hipStream_t stream);
/* dchat_partial [Np,D] and beta_partial [N]: this shard's contribution (sum over ranks before
 * finalize); dwdb [2] = this shard's (dL/dw, dL/db).  gloss = upstream dL (NULL -> 1). */
int sv_ge2e_bwd_rows(int N_local, int M, int D, int spk_offset, int N, const float* w, const float* b,
                     const float* gloss, float* dchat_partial, float* beta_partial, float* dwdb, float* workspace,
                     hipStream_t stream);
int sv_ge2e_bwd_finalize(int N_local, int M, int D, int spk_offset, int N, const float* dchat, const float* beta,
                         float* dE, float* workspace, hipStream_t stream);
int sv_ge2e_bwd(int N, int M, int D, const float* w, const float* b, const float* gloss, float* dE, float* dwdb,
                float* dchat, float* beta, float* workspace, hipStream_t stream);

/* fused single-GPU training form (all N speakers local, gloss = 1): forward + closed-form
 * backward in three launches (per-speaker prep; a wave per row with the centroids staged in LDS,
 * fp32, in one tile up to 128 speakers and two tiles of 128 above: cosines, shuffle softmax, row
 * backward; a workgroup per (speaker, 64-wide d slice): centroid gradients and the speaker's dE).
 * Needs N <= 256, 2 <= M <= 16, D <= 256, D % 4 == 0 (sv_ge2e_train_ok);
 * workspace: sv_ge2e_workspace_size(N, M, D, N). */
int sv_ge2e_train_ok(int N, int M, int D);
int sv_ge2e_train(const float* E, int N, int M, int D, const float* w, const float* b, float* loss, float* per,
                  float* dE, float* dwdb, float* workspace, hipStream_t stream);

/* the fused kernels in the speaker-sharded form (data parallel; same shape limits as
 * sv_ge2e_train_ok(N, M, D) for the GLOBAL N):
 *   sv_ge2e_shard_prep      this shard's per-speaker sums ssum_local [N_local, D] (all-gather them
 *                           into ssum_all [N, D]) and its rows' normalised state (workspace);
 *   sv_ge2e_shard_rows      rows against all N centroids, softmax, row backward, then this shard's
 *                           contribution to red [Np*D + N] (dC^ before the norm Jacobian, beta;
 *                           SUM-all-reduce it) and its loss / (dw, db) partials;
 *   sv_ge2e_shard_finalize  this shard's dE from the reduced red.
 * workspace: sv_ge2e_workspace_size(N_local, M, D, N), kept across the three calls. */
int sv_ge2e_shard_prep(const float* E, int N_local, int M, int D, float* ssum_local, float* workspace,
                       hipStream_t stream);
int sv_ge2e_shard_rows(int N_local, int M, int D, int spk_offset, int N, const float* ssum_all, const float* w,
                       const float* b, float* per, float* red, float* loss_local, float* dwdb_local, float* workspace,
                       hipStream_t stream);
int sv_ge2e_shard_finalize(int N_local, int M, int D, int spk_offset, int N, const float* red, float* dE,
                           float* workspace, hipStream_t stream);

/* stand-alone helpers (utils.py): C = E.mean(1) [N,D]; cos [N,M,Nc] = get_cossim(E, C) with the
 * diagonal from E's own leave-one-out centroids (utils.py:75,91,113), +1e-6; calc_loss on S [N,M,K]. */
int sv_ge2e_centroids(const float* E, int N, int M, int D, float* C, hipStream_t stream);
size_t sv_ge2e_cossim_workspace(int N, int M, int D, int Nc);
int sv_ge2e_cossim(const float* E, int N, int M, int D, const float* C, int Nc, float* cos, float* workspace,
                   hipStream_t stream);
int sv_ge2e_calc_loss(const float* S, int N, int M, int K, float* per, float* loss, hipStream_t stream);
/* their backward passes (the autograd of utils.py:28, :72-115, :126-132):
 *   dE = dC / M broadcast over the M utterances;
 *   cossim: dE [N,M,D], dC [Nc,D] from dcos [N,M,Nc] -- gradient through the cosines against C_k
 *   (k != j) and, on the diagonal, through E's own leave-one-out centroid U_ji = (sum_i' E_ji' -
 *   E_ji) / (M - 1), as index_put's backward routes it (the overwritten entries give C nothing);
 *   calc_loss: dS [N,M,K] from gloss (device scalar, NULL = 0) and gper [N,M] (NULL = 0):
 *   dS_jik = (gloss + gper_ji) (e^{S_jik} / (sum_k e^{S_jik} + 1e-6) - [k == j]). */
int sv_ge2e_centroids_bwd(const float* dC, int N, int M, int D, float* dE, hipStream_t stream);
size_t sv_ge2e_cossim_bwd_workspace(int N, int M, int D, int Nc);
int sv_ge2e_cossim_bwd(const float* E, int N, int M, int D, const float* C, int Nc, const float* dcos, float* dE,
                       float* dC, float* workspace, hipStream_t stream);
int sv_ge2e_calc_loss_bwd(const float* S, int N, int M, int K, const float* gloss, const float* gper, float* dS,
                          hipStream_t stream);
/* EER sweep (train_speech_embedder.py:134-149): per threshold, #{S > thr} over all of S [N,M2,Nc]
 * and over its diagonal k == j (exact integer counts, returned as float). */
int sv_eer_counts(const float* S, int N, int M2, int Nc, const float* thresholds, int n_thr, float* cnt_all,
                  float* cnt_diag, hipStream_t stream);

/* ---- bf16 mixed-precision variant (BASELINE config c3) ---------------------------------------
 * GEMM operands (weights, h, dgates) in bf16 (RNE casts), bf16 MFMA with fp32 accumulation;
 * the stored x-projection (K1 output incl. biases) and the saved activated gates are bf16 (ABI
 * v3: `gates` is sv_bf16 [T,B,4H] -- in: bf16(x W_ih^T + b_ih + b_hh), out: bf16 activations;
 * the cell update itself runs on the fp32 sums and fp32 activations); cell state, biases,
 * gradients and outputs fp32.  Same layouts as the fp32 entry points, except transposed layouts
 * use column blocks of Bp = (B + 7) & ~7 and F, H, K and every bf16 leading dimension must be
 * multiples of 8.  sv_bf16 = raw bf16 bits. */
typedef unsigned short sv_bf16;
size_t sv_gemm_bf16_workspace(int M, int N, int K);
/* C[M,N] (fp32) = A[M,K] . B[N,K]^T (+ bias0 + bias1) (+ beta C); both operands k-contiguous */
int sv_gemm_bf16(int M, int N, int K, const sv_bf16* A, long lda, const sv_bf16* B, long ldb, float* C, long ldc,
                 const float* bias0, const float* bias1, float beta, float* workspace, hipStream_t stream);
/* C[M,N] (bf16) = bf16(A[M,K] . B[N,K]^T + bias0 + bias1): fp32 accumulation, one rounding (the
 * x-projection store of the bf16 LSTM); ldc % 4 == 0 for the 256 x 256 kernel, else a slower one */
int sv_gemm_bf16_bf(int M, int N, int K, const sv_bf16* A, long lda, const sv_bf16* B, long ldb, sv_bf16* C,
                    long ldc, const float* bias0, const float* bias1, hipStream_t stream);
int sv_cast_bf16(const float* x, sv_bf16* y, long n, hipStream_t stream);
/* n <= 8 such casts in one launch (y[i] = bf16(x[i]), count[i] elements each; host arrays) */
int sv_cast_bf16_batch(int n, const float* const* x, sv_bf16* const* y, const long* count, hipStream_t stream);
int sv_transpose_cast_bf16(const float* src, long ld_src, int R, int C, sv_bf16* dst, long ld_dst,
                           hipStream_t stream);
/* (ABI v10) the bf16 stack's input in one launch: frames x [B,T,F] (F <= 64) -> x_bf [T,B,F] and,
 * if xT != NULL, xT [F][T*Bp] (column t*Bp + b = x[b,t,:], columns b in [B, Bp) zero) */
int sv_frames_to_bf16(const float* x, int B, int T, int F, sv_bf16* x_bf, sv_bf16* xT, int Bp, hipStream_t stream);
/* (ABI v10) every layer's bf16 weights in one launch, each fp32 weight read once: w_ih_bf[l] /
 * w_hh_bf[l] = bf16(w_ih[l]) / bf16(w_hh[l]) (row-major, the stack forward's operands) and, if
 * bwd_workspace != NULL (sv_lstm_bwd_workspace(SV_DTYPE_BF16, L, T, B, F, H) bytes), the bf16
 * transposes the stack backward reads, inside that workspace: pass it to sv_lstm_bwd with
 * SV_SCHED_WT_READY and the backward launches no transposes. */
int sv_lstm_weights_bf16(int L, int T, int B, int F, int H, const float* const* w_ih, const float* const* w_hh,
                         sv_bf16* const* w_ih_bf, sv_bf16* const* w_hh_bf, void* bwd_workspace, hipStream_t stream);
/* (ABI v11) sv_frames_to_bf16 (frames x [B,T,F] -> x_bf, xT) and sv_lstm_weights_bf16 in ONE launch:
 * the bf16 stack forward's whole operand preparation. */
int sv_lstm_prep_bf16(int L, int T, int B, int F, int H, const float* x, sv_bf16* x_bf, sv_bf16* xT, int Bp,
                      const float* const* w_ih, const float* const* w_hh, sv_bf16* const* w_ih_bf,
                      sv_bf16* const* w_hh_bf, void* bwd_workspace, hipStream_t stream);
/* x_bf [T,B,F]; writes gates (bf16), c_tm/h_tm (fp32) plus h_bf [T+1,B,H] and hT [H,(T+1)Bp] (bf16) */
int sv_lstm_layer_fwd_bf16(const sv_bf16* x_bf, int T, int B, int F, int H, const sv_bf16* w_ih_bf,
                           const sv_bf16* w_hh_bf, const float* b_ih, const float* b_hh, sv_bf16* gates, float* c_tm,
                           float* h_tm, sv_bf16* h_bf, sv_bf16* hT, hipStream_t stream);
/* stack forward in bf16 (as sv_lstm_stack_fwd; h_bf per layer [T+1,B,H]; of the fp32 h_tm only
 * slot T = h_{T-1}, the projection's input, is guaranteed -- the persistent schedules write no
 * other slot, the next layer and the backward read the bf16 copies) under `schedule`
 * (SV_SCHED_*).  sync: the caller's sync block (below; required when the persistent recurrences run).
 * probe (may be NULL): 2*L caller events recorded around each layer's persistent recurrence
 * launch (before / after; only when the persistent schedule runs) -- in-step kernel timing. */
int sv_lstm_stack_fwd_bf16(int L, int T, int B, int F, int H, const sv_bf16* x_bf, const sv_bf16* const* w_ih_bf,
                           const sv_bf16* const* w_hh_bf, const float* const* b_ih, const float* const* b_hh,
                           sv_bf16* const* gates, float* const* c_tm, float* const* h_tm, sv_bf16* const* h_bf,
                           sv_bf16* const* hT, int chunk, hipStream_t main, const hipStream_t* side,
                           hipEvent_t* ev, void* sync, hipEvent_t* probe, int schedule);
size_t sv_lstm_layer_bwd_bf16_workspace(int T, int B, int F, int H);
/* wihT_bf [F,4H], whhT_bf [H,4H]; dg_bf [T,B,4H] and dgT_bf [4H,T*Bp] are bf16 outputs */
int sv_lstm_layer_bwd_bf16(int T, int B, int F, int H, const sv_bf16* xT_bf, long ld_xT, const sv_bf16* wihT_bf,
                           const sv_bf16* whhT_bf, const sv_bf16* gates, const float* c_tm, const sv_bf16* hT_bf,
                           const float* dh_up, int dh_up_full, sv_bf16* dg_bf, sv_bf16* dgT_bf, float* dx_tm,
                           float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, float* workspace,
                           hipStream_t stream);

/* stack backward in bf16 under `schedule` (as sv_lstm_stack_bwd, L side streams; fp32 master
 * weights are transpose-cast per call; dg/dgT per layer bf16).  probe: as the bf16 stack
 * forward's, around each layer's persistent backward recurrence. */
size_t sv_lstm_stack_bwd_bf16_workspace(int L, int T, int B, int F, int H);
int sv_lstm_stack_bwd_bf16(int L, int T, int B, int F, int H, const sv_bf16* const* xT, const long* ld_xT,
                           const float* const* w_ih, const float* const* w_hh, const sv_bf16* const* gates,
                           const float* const* c_tm, const sv_bf16* const* hT, const float* dh_last,
                           sv_bf16* const* dg, sv_bf16* const* dgT, float* const* dx, float* const* dw_ih,
                           float* const* dw_hh, float* const* db_ih, float* const* db_hh, void* workspace, int chunk,
                           hipStream_t main, const hipStream_t* side, hipEvent_t* ev, void* sync, hipEvent_t* probe,
                           int schedule);

/* ---- dtype-enum form of the stack entry points (SURVEY.md §8 b: `lstm_fwd` = K1 + K2 and
 * `lstm_bwd` = K3 + K4 with a dtype argument; replaces the nn.LSTM forward / autograd backward at
 * speech_embedder_net.py:28 and train_speech_embedder.py:62).  One entry point per direction:
 *   SV_DTYPE_F32   -> sv_lstm_stack_fwd / _bwd: the `void` operands are float; h_bf is ignored
 *                     (pass NULL);
 *   SV_DTYPE_BF16  -> sv_lstm_stack_fwd_bf16 / _bwd_bf16: the `void` operands are sv_bf16
 *                     (x, w_ih, w_hh, gates, h_bf, hT; in the backward xT, gates, hT, dg, dgT);
 *                     `products` and `kstamp` are ignored (pass 0 / NULL).
 * Every other argument means what it means in the dtype-specific entry point; the backward takes
 * the fp32 master weights in both dtypes.  An unknown dtype returns SV_EARG. */
#define SV_DTYPE_F32 0
#define SV_DTYPE_BF16 1
int sv_lstm_fwd(int dtype, int L, int T, int B, int F, int H, const void* x, const void* const* w_ih,
                const void* const* w_hh, const float* const* b_ih, const float* const* b_hh, void* const* gates,
                float* const* c_tm, float* const* h_tm, void* const* h_bf, void* const* hT, int chunk,
                hipStream_t main, const hipStream_t* side, hipEvent_t* ev, int products, int schedule, void* sync,
                hipEvent_t* probe);
size_t sv_lstm_bwd_workspace(int dtype, int L, int T, int B, int F, int H);
int sv_lstm_bwd(int dtype, int L, int T, int B, int F, int H, const void* const* xT, const long* ld_xT,
                const float* const* w_ih, const float* const* w_hh, const void* const* gates, const float* const* c_tm,
                const void* const* hT, const float* dh_last, void* const* dg, void* const* dgT, float* const* dx,
                float* const* dw_ih, float* const* dw_hh, float* const* db_ih, float* const* db_hh, void* workspace,
                int chunk, hipStream_t main, const hipStream_t* side, hipEvent_t* ev, int products, hipEvent_t* probe,
                unsigned long long* kstamp, int schedule, void* sync);

/* ---- persistent recurrences (one launch per layer for all T; sv_persist.hip).  The bf16 stack
 * forward uses them (by default when H = 768: W_hh held in registers) when the grid is
 * co-resident on the device of `main` (sv_persist_fwd_ok answers for the current device); the
 * bf16 stack backward likewise (H in {64, 96, 768}; by default when H = 768), handing dG off
 * through a fragment-order scratch of sv_persist_bwd_scratch(T, B, H) bytes that
 * sv_lstm_stack_bwd_bf16_workspace includes.
 * Sync block: caller-owned device memory of sv_sync_size() bytes, zeroed once before first use;
 * it holds the recurrences' arrival counters and, in its first u32 word, a STICKY status:
 *   0 ok; bit 0 / bit 1 set = a forward / backward hand-off wait timed out (a co-residency
 *   failure: another kernel or process held the CUs).  A timed-out launch drains instead of
 *   hanging; every later wait on the same block returns at once; all outputs written since are
 *   invalid.  The caller reads the word (async copy) and clears it.
 * Calls that share one block must be ordered (one stream); distinct blocks may run concurrently.
 * sv_status_poison: x[0..n) := NaN if the block's status is set (stream-ordered, no host sync). */
size_t sv_sync_size(void);
int sv_persist_fwd_ok(int B, int H);
int sv_persist_bwd_ok(int B, int H);
/* the bf16 layer-wavefront schedule (all L layers in one forward and one backward launch) fits
 * B rows on the current device (L = 3, F = 40, H = 768: B <= 96 on 256 CUs) */
int sv_wave_ok(int L, int T, int B, int F, int H);
size_t sv_persist_bwd_scratch(int T, int B, int H);
int sv_status_poison(const void* sync, float* x, int n, hipStream_t stream);
/* (ABI v9) sv_status_poison's poisoning of x[0..n) (n may be 0) plus a report of the status word
 * to the host without a copy: one 8-byte store of ((seq << 32) | status) into host_slot_dev, the
 * device address (sv_host_device_ptr = hipHostGetDevicePointer) of a caller-owned, 8-byte aligned
 * slot of pinned host memory; the host knows step `seq` is done when the slot's high word equals
 * seq.  Replaces the device->pinned copy + event of the old check. */
int sv_status_report(const void* sync, float* x, int n, void* host_slot_dev, unsigned seq, hipStream_t stream);
int sv_host_device_ptr(void* host, void** dev);
/* data-parallel status agreement (a rank whose recurrence timed out must stop every rank's
 * update): sv_status_to_flag writes the status's forward / backward bits as 0/1 floats into
 * flag[0..1], two words of the gradient buffer that the SUM all-reduce carries; sv_status_merge
 * ORs the bits whose reduced flag is nonzero back into the block's status, so sv_clip_sgd_step
 * skips the update on every rank alike. */
int sv_status_to_flag(const void* sync, float* flag, hipStream_t stream);
int sv_status_merge(void* sync, const float* flag, hipStream_t stream);

/* ---- large-batch d-vector inference (dvector_create.py:96-101; SpeechEmbedder.forward of every
 * 24-frame window of a file, speech_embedder_net.py:27-33), bf16 GEMM operands / fp32 accumulation
 * and state as the c3 forward (the input projection rounded to bf16 with its biases).  One launch per
 * timestep and layer: the 256 x 256 bf16 GEMM over [x_t | h_{t-1}] . [W_ih | W_hh]^T with the LSTM
 * cell in its epilogue, so no co-residency requirement at any B.  x [B][T][F] fp32 (batch-first
 * windows; F <= 64), layer l's w_ih [4H][F_l] (F_0 = F, else H), w_hh [4H][H], b_ih / b_hh [4H]
 * (the arrays of b_ih / b_hh may be NULL), w_p [P][H], b_p [P] (may be NULL), all fp32 device
 * pointers; emb [B][P] = normalize(h_{T-1} w_p^T + b_p).  H % 64 == 0, 4H % 256 == 0; workspace
 * of sv_dvector_bf16_workspace bytes, 256-B aligned.  Replaces embedder_net(windows) at
 * dvector_create.py:100 for the bf16 precision of embed_windows (dvector.py). */
size_t sv_dvector_bf16_workspace(int B, int T, int F, int H, int L, int P);
int sv_dvector_embed_bf16(int B, int T, int F, int H, int L, const float* x, const float* const* w_ih,
                          const float* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                          const float* w_p, const float* b_p, int P, float* emb, void* workspace,
                          hipStream_t stream);

/* ---- clip_grad_norm_ + SGD step over one flat parameter group (train_speech_embedder.py:63-65)
 * p -= lr * min(1, max_norm / (|g|_2 + 1e-6)) * g; write_grad=1 also scales g in place.
 * sync (may be NULL): a persistent-recurrence sync block; if its status is set the step is
 * skipped (p and g untouched, total_norm_out = NaN): never a step on invalid gradients. */
size_t sv_clip_sgd_workspace(void);
int sv_clip_sgd_step(float* params, float* grads, long n, float max_norm, float lr, int write_grad,
                     float* total_norm_out, const void* sync, float* workspace, hipStream_t stream);
/* the reference's two parameter groups in one pair of launches (ABI v8): the network's
 * (clip_grad_norm_(net, 3.0), train_speech_embedder.py:63) and the GE2E loss's {w, b}
 * (clip_grad_norm_(ge2e, 1.0), :64), each exactly as sv_clip_sgd_step computes it (bit-identical);
 * total_norm_out (may be NULL): float[2]; workspace: sv_clip_sgd_workspace() * 2 bytes */
int sv_clip_sgd_step2(float* params0, float* grads0, long n0, float max_norm0, float* params1, float* grads1,
                      long n1, float max_norm1, float lr, int write_grad, float* total_norm_out, const void* sync,
                      float* workspace, hipStream_t stream);
/* (ABI v11) sv_clip_sgd_step2 with the training step's status report in its update launch: as
 * sv_status_report(sync, report_x, report_n, host_slot_dev, seq) after it, one launch fewer */
int sv_clip_sgd_step2_report(float* params0, float* grads0, long n0, float max_norm0, float* params1, float* grads1,
                             long n1, float max_norm1, float lr, int write_grad, float* total_norm_out,
                             const void* sync, float* workspace, float* report_x, int report_n, void* host_slot_dev,
                             unsigned seq, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SV_GE2E_H */
