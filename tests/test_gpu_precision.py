"""GPU: the mixed-precision configs (BASELINE c3 / c4 / c5: bf16 GEMM operands, bf16 storage of the
x-projection and saved activations, fp32 state, accumulation, gradients and loss) pinned to the
bf16 oracle (oracle/lstm_bf16.py, whose
fp32 mode is pinned to the reference's golden vectors), at the shapes the configs run per GPU:

  c4 per rank   N = 64 speakers over 8 GPUs -> 8 x M = 10 = 80 utterances, T = 160
  c3            N = 64 x M = 10 = 640 utterances at T = 24 (CPU oracle) and at its full T = 160
                (the same oracle run on the GPU's stock torch ops)
  c5 per rank   N = 256 over 8 GPUs -> 32 x 10 = 320 utterances, T = 180

Every tolerance is about 10x the deviation measured on MI355X (DESIGN.md §6 lists the measured
values; each check prints its MEASURED line).  Deviations are relative to the reference
quantity's max-abs (emb: absolute; loss: relative).  Weights use the portable recipe scaled x3 so
the embeddings are diverse (SURVEY §7 hard part 5)."""
import numpy as np
import pytest
import torch

import recipe
from conftest import model_dims
from oracle import lstm_bf16

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(name, value, tol):
    print(f"\nMEASURED {name} {value:.3e} (tol {tol:.1e})")
    assert value <= tol, (name, value, tol)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _hip_step(dims, sd, x, N, M, precision):
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(DEV)
    net.precision = precision
    emb = net(torch.tensor(x, device=DEV)).detach().cpu().numpy()
    tr = GE2ETrainer(net, GE2ELoss(DEV), lr=0.01)
    loss = float(tr.step(torch.tensor(x, device=DEV), N, M))
    tr.check()
    grads = {k: p.grad.detach().cpu().numpy().copy() for k, p in net.named_parameters()}
    params = {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()}
    return emb, loss, grads, params


def _compare(tag, dims, N, M, T, seed, tol, oracle_device="cpu"):
    sd = recipe.make_weights(seed, *dims, scale=3.0)
    x = recipe.make_frames(seed + 1, N * M, T, dims[0])
    emb, loss, grads, params = _hip_step(dims, sd, x, N, M, "bf16")
    r_loss, r_new, _, _, r_emb, r_grads, _, _ = lstm_bf16.train_step(sd, 10.0, -5.0, x, N, M, dims[2], bf16=True,
                                                                     device=oracle_device)
    r_emb = r_emb.detach().cpu()
    r_grads = {k: v.detach().cpu() for k, v in r_grads.items()}
    r_new = {k: v.detach().cpu() for k, v in r_new.items()}
    _check(f"{tag}.emb_abs", float(np.abs(emb - r_emb.numpy()).max()), tol["emb"])
    _check(f"{tag}.loss_rel", abs(loss - r_loss) / abs(r_loss), tol["loss"])
    # the trainer leaves the CLIPPED gradients in .grad (clip_grad_norm_ scales them in place)
    tot = float(np.sqrt(sum(float((r_grads[k].double() ** 2).sum()) for k in r_grads)))
    coef = min(1.0, 3.0 / (tot + 1e-6))
    g = max(_rel(grads[k], coef * r_grads[k].numpy()) for k in grads)
    _check(f"{tag}.grad_rel_max", g, tol["grad"])
    p = max(float(np.abs(params[k] - r_new[k].numpy()).max()) for k in params)
    _check(f"{tag}.param_abs", p, tol["param"])
    return emb, loss


def test_c4_rank_shape_bf16_against_oracle():
    """c4's per-rank shape (B = 80) on the persistent W-stationary kernels: against the bf16
    oracle, and the bf16-vs-fp32 gap of the oracle itself recorded beside it."""
    from pytorch_speaker_verification_amd._lib import lib
    dims, N, M, T = (40, 768, 3, 256), 8, 10, 160
    assert lib().sv_persist_fwd_ok(N * M, 768) and lib().sv_persist_bwd_ok(N * M, 768)
    # loss 2e-3: measured 2.9e-4 since the x-projection is stored in bf16 (the wavefront rounds it
    # inside its accumulator, so fp32-order flips of that rounding reach the loss at B = 80)
    _compare("c4_rank", dims, N, M, T, 4040, dict(emb=5e-3, loss=2e-3, grad=5e-2, param=2e-5))


def test_c3_shape_bf16_against_oracle():
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 24
    _compare("c3_T24", dims, N, M, T, 3030, dict(emb=5e-3, loss=5e-4, grad=5e-2, param=2e-5))


def test_c3_full_T160_bf16_against_oracle():
    """c3 exactly as benched: B = 640, T = 160 on the wide 32 x 64 persistent tiles
    (lstm_persist3_fwd/bwd_bf16_kernel, chosen for B > 320), against the bf16 oracle run on the
    GPU (its fp32 mode is pinned to the reference-generated golden step, test_oracle_bf16.py)."""
    from pytorch_speaker_verification_amd._lib import lib
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 160
    assert lib().sv_persist_fwd_ok(N * M, 768) and lib().sv_persist_bwd_ok(N * M, 768)
    _compare("c3_T160", dims, N, M, T, 3131, dict(emb=5e-3, loss=5e-4, grad=5e-2, param=2e-5), oracle_device=DEV)


def test_c5_rank_shape_bf16_against_oracle():
    dims, N, M, T = (40, 768, 3, 256), 32, 10, 180
    _compare("c5_rank", dims, N, M, T, 5050, dict(emb=5e-3, loss=5e-4, grad=5e-2, param=2e-5))


def test_bf16_vs_fp32_gap_matches_oracle_gap():
    """What bf16 operands cost: the HIP bf16-vs-fp32 gap equals the oracle's bf16-vs-fp32 gap
    (same inputs, c4 rank shape) to within the oracle tolerance -- the mixed-precision error is
    the rounding the config prescribes, nothing more."""
    dims, N, M, T = (40, 768, 3, 256), 8, 10, 160
    sd = recipe.make_weights(4041, *dims, scale=3.0)
    x = recipe.make_frames(4042, N * M, T, dims[0])
    e16, l16, _, _ = _hip_step(dims, sd, x, N, M, "bf16")
    e32, l32, _, _ = _hip_step(dims, sd, x, N, M, "f32")
    o16, _ = lstm_bf16.embedder_forward(sd, x, dims[2], bf16=True)
    o32, _ = lstm_bf16.embedder_forward(sd, x, dims[2], bf16=False)
    hip_gap = float(np.abs(e16 - e32).max())
    ora_gap = float((o16 - o32).abs().max())
    _check("c4_rank.hip_bf16_fp32_emb_gap", hip_gap, 2e-2)
    _check("c4_rank.gap_mismatch", abs(hip_gap - ora_gap), 3e-4)


def test_c5_two_rank_shape_bf16_row_chunks_against_oracle():
    """c5 split over 2 GPUs: 128 x 10 = 1280 rows per rank at T = 180, more than the co-resident
    persistent recurrences take (<= 672 rows), so the trainer runs the bf16 stack as two 640-row
    chunks on the persistent kernels and sums their weight gradients (trainer.bf16_row_chunks);
    against the bf16 oracle run on the GPU."""
    from pytorch_speaker_verification_amd.trainer import bf16_row_chunks
    dims, N, M, T = (40, 768, 3, 256), 128, 10, 180
    assert bf16_row_chunks(N * M, 768, T=T) == [(0, 640), (640, 1280)]
    assert bf16_row_chunks(640, 768) == [(0, 640)] and bf16_row_chunks(1280, 768, "per_step") == [(0, 1280)]
    # the layer wavefront: 80 rows whole, 160 rows as two halves, 320 rows on the persistent kernels
    assert bf16_row_chunks(80, 768) == [(0, 80)] and bf16_row_chunks(160, 768) == [(0, 80), (80, 160)]
    assert bf16_row_chunks(320, 768) == [(0, 320)]
    _compare("c5_2rank_chunked", dims, N, M, T, 5151, dict(emb=5e-3, loss=5e-4, grad=5e-2, param=2e-5),
             oracle_device=DEV)


def test_c4_four_rank_shape_bf16_wavefront_halves_against_oracle():
    """c4 split over 4 GPUs: 16 x 10 = 160 rows per rank at T = 160, run as two 80-row halves on the
    one-launch layer wavefront (trainer.bf16_row_chunks); against the bf16 oracle on the GPU."""
    from pytorch_speaker_verification_amd.trainer import bf16_row_chunks
    dims, N, M, T = (40, 768, 3, 256), 16, 10, 160
    assert bf16_row_chunks(N * M, 768, T=T) == [(0, 80), (80, 160)]
    _compare("c4_4rank_halves", dims, N, M, T, 4141, dict(emb=5e-3, loss=2e-3, grad=5e-2, param=2e-5),
             oracle_device=DEV)


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_input_gradient_through_embedder_function(precision):
    """loss.backward() with frames that require grad: EmbedderFunction returns dx [B,T,F] in both
    precisions (bf16: the per-layer kernels with the layer-0 dx = dG W_ih GEMM).  Against the bf16
    oracle's layer-0 dx (fp32 mode for f32) for d emb = a fixed random direction, c4 rank dims at
    T = 24."""
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims, B, T, seed = (40, 768, 3, 256), 80, 24, 5151
    sd = recipe.make_weights(seed, *dims, scale=3.0)
    x = recipe.make_frames(seed + 1, B, T, dims[0])
    g = np.random.default_rng(seed + 2).standard_normal((B, dims[3])).astype(np.float32)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(DEV)
    net.precision = precision
    xt = torch.tensor(x, device=DEV, requires_grad=True)
    emb = net(xt)
    emb.backward(torch.tensor(g, device=DEV))
    dx = xt.grad.detach().cpu().numpy()
    bf = precision == "bf16"
    r_emb, cache = lstm_bf16.embedder_forward(sd, x, dims[2], bf16=bf)
    r_dx = lstm_bf16.embedder_backward(sd, g, cache, dims[2], bf16=bf)["input"].numpy()
    assert dx.shape == r_dx.shape == (B, T, dims[0])
    _check(f"dx_{precision}.rel_vs_oracle", _rel(dx, r_dx), 5e-2 if bf else 1e-4)
