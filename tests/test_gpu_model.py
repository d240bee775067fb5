"""GPU parity of the full path (SpeechEmbedder + GE2ELoss + backward + clip/SGD) against
the reference's golden vectors (small dims and the full 40->768x3->256 net at c1) and,
at the full c2 size (N=64 x M=10, T=160), against stock PyTorch fp32 on the same GPU
(nn.LSTM via MIOpen; oracle/torch_port.py) plus size-independent properties."""
import numpy as np
import pytest
import torch

import recipe
from conftest import golden, model_dims
from oracle import torch_port

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(dims, sd_np):
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd_np[k]))
    return net.to(DEV), GE2ELoss(DEV)


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _check(name, value, tol):
    """Tolerances are ~10x the deviation measured on MI355X."""
    print(f"\nMEASURED {name} {value:.3e} (tol {tol:.1e})")
    assert value <= tol, (name, value, tol)


def test_small_net_autograd_path_matches_reference():
    """The drop-in path: module forward, loss.backward(), torch clip + SGD (user code)."""
    s = golden("net_small.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": ge2e.parameters()}], lr=0.01)
    losses = []
    for step in range(3):
        opt.zero_grad()
        emb = net(x).reshape(N, M, -1)
        if step == 0:
            np.testing.assert_allclose(emb.detach().cpu().numpy(), s["emb0"], atol=2e-5)
        loss = ge2e(emb)
        loss.backward()
        if step == 0:
            for k, p in net.named_parameters():
                assert _rel(p.grad.cpu().numpy(), s["grad." + k]) < 1e-4, k
            assert abs(ge2e.w.grad.item() - float(s["dw0"])) <= 1e-4 * max(1, abs(float(s["dw0"])))
        torch.nn.utils.clip_grad_norm_(net.parameters(), 3.0)
        torch.nn.utils.clip_grad_norm_(ge2e.parameters(), 1.0)
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, s["losses"], rtol=1e-4)
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), s["pf." + k], atol=2e-5)


def test_small_net_fused_trainer_matches_reference():
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    s = golden("net_small.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    losses = [float(tr.step(x, N, M)) for _ in range(3)]
    np.testing.assert_allclose(losses, s["losses"], rtol=1e-4)
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), s["pf." + k], atol=2e-5)
    np.testing.assert_allclose([ge2e.w.item(), ge2e.b.item()], s["wb_final"], atol=1e-5)


@pytest.mark.parametrize("schedule", ["auto", "persist"])
def test_full_dims_c1_matches_reference(schedule):
    """The reference's own full-dims step at c1 (B = 20, T = 160): under 'auto' the per-step
    kernels (the persistent grid would fill 24 of 256 CUs), under 'persist' the fp32
    W-stationary persistent recurrences (sv_persist_f32.hip) against the same golden."""
    s = golden("net_full_c1.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    net.schedule = schedule
    tag = "c1" if schedule == "auto" else "c1_persist"
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    emb = net(x).reshape(N, M, -1)
    _check(f"{tag}.emb_abs", float(np.abs(emb.detach().cpu().numpy() - s["emb"]).max()), 2e-6)
    loss = ge2e(emb)
    _check(f"{tag}.loss_rel", abs(loss.item() - float(s["loss"])) / abs(float(s["loss"])), 2e-6)
    loss.backward()
    gn, gh = 0.0, 0.0
    for k, p in net.named_parameters():
        g = p.grad.cpu().double()
        gn = max(gn, abs(g.norm().item() - float(s["gnorm." + k])) / float(s["gnorm." + k]))
        head = g.reshape(g.shape[0], -1)[:8, :8].numpy() if g.dim() == 2 else g[:64].numpy()
        ref = s["ghead." + k]
        gh = max(gh, float(np.abs(head - ref).max()) / max(np.abs(ref).max(), 1e-6))
    _check(f"{tag}.grad_norm_rel", gn, 2e-5)
    _check(f"{tag}.grad_head_rel", gh, 5e-5)


def _grad_checks(tag, net, s, tol_norm=2e-5, tol_head=5e-5):
    gn, gh = (0.0, ""), (0.0, "")
    for k, p in net.named_parameters():
        g = p.grad.cpu().double()
        gn = max(gn, (abs(g.norm().item() - float(s["gnorm." + k])) / float(s["gnorm." + k]), k))
        head = g.reshape(g.shape[0], -1)[:8, :8].numpy() if g.dim() == 2 else g[:64].numpy()
        ref = s["ghead." + k]
        gh = max(gh, (float(np.abs(head - ref).max()) / max(np.abs(ref).max(), 1e-6), k))
    print(f"\nMEASURED {tag}.worst grad_norm {gn[1]}, grad_head {gh[1]}")
    _check(f"{tag}.grad_norm_rel", gn[0], tol_norm)
    _check(f"{tag}.grad_head_rel", gh[0], tol_head)


@pytest.mark.parametrize("schedule", ["auto", "per_step"])
def test_full_size_c2_matches_reference(schedule):
    """The headline config c2 (N=64 x M=10, T=160, fp32) against the reference's own step
    (tests/golden/net_full_c2.npz, generated by running the reference): embeddings, loss, every
    parameter's gradient norm and 8x8 head through module forward + loss.backward(); 'auto' runs the
    fp32 persistent recurrences at this batch, 'per_step' the K2 / K3 kernels."""
    s = golden("net_full_c2.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    net.schedule = schedule
    tag = "c2_ref" if schedule == "auto" else "c2_ref_per_step"
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    emb = net(x).reshape(N, M, -1)
    _check(f"{tag}.emb_abs", float(np.abs(emb.detach().cpu().numpy().reshape(N * M, -1) - s["emb"].reshape(N * M, -1)).max()), 5e-6)
    loss = ge2e(emb)
    _check(f"{tag}.loss_rel", abs(loss.item() - float(s["loss"])) / abs(float(s["loss"])), 1e-5)
    loss.backward()
    _grad_checks(tag, net, s)
    # dL/dw = sum dS cos is a difference of two ~600-sized sums (dS sums to ~0 per row): it moves
    # with the embeddings' last-bit deviations.  Checked in two parts against the fp64 GE2E oracle:
    # the kernel on our embeddings, and the reference's dw against the oracle on ITS embeddings
    # moved by the same embedding deviation
    from oracle import ge2e_np
    e_ours = emb.detach().cpu().double().numpy()
    e_ref = s["emb"].reshape(N, M, -1).astype(np.float64)
    dw_ours64 = ge2e_np.ge2e_backward(e_ours, 10.0, -5.0)[1]
    dw_ref64 = ge2e_np.ge2e_backward(e_ref, 10.0, -5.0)[1]
    dw = ge2e.w.grad.item()
    _check(f"{tag}.dw_kernel_rel_vs_fp64_on_own_emb", abs(dw - dw_ours64) / max(1.0, abs(dw_ours64)), 1e-5)
    sens = abs(dw_ours64 - dw_ref64)
    print(f"\nMEASURED {tag}.dw ours {dw:.7f} ref {float(s['dw0']):.7f} fp64(own emb) {dw_ours64:.7f} "
          f"fp64(ref emb) {dw_ref64:.7f}")
    _check(f"{tag}.dw_abs_beyond_emb_sensitivity", max(0.0, abs(dw - float(s["dw0"])) - sens), 2e-5)


@pytest.mark.parametrize("schedule", ["auto", "per_step"])
def test_full_size_c2_fused_step_matches_reference(schedule):
    """The fused step bench.py times (GE2ETrainer.step: forward, GE2E, backward, clip 3.0 / 1.0,
    SGD) at c2 against the reference's parameters after its one clipped SGD step: 8x8 heads and
    every parameter's update norm |p1 - p0|, plus the loss and w, b."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    s = golden("net_full_c2.npz")
    dims = tuple(int(v) for v in s["dims"])
    sd = recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"]))
    net, ge2e = _build(dims, sd)
    net.schedule = schedule
    tag = "c2_ref_step" if schedule == "auto" else "c2_ref_step_per_step"
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    loss = float(tr.step(x, N, M))
    _check(f"{tag}.loss_rel", abs(loss - float(s["loss"])) / abs(float(s["loss"])), 1e-5)
    ph, dn = 0.0, (0.0, "")
    for k, v in net.state_dict().items():
        p32 = v.detach().cpu().numpy()
        p = p32.astype(np.float64)
        head = p.reshape(p.shape[0], -1)[:8, :8] if p.ndim == 2 else p[:64]
        ph = max(ph, float(np.abs(head - s["p1head." + k]).max()))
        ref = float(s["dpnorm." + k])
        # |p1 - p0| of a small update (the biases') is partly the fp32 rounding of p1 itself, in both
        # runs: allowed = 1e-4 relative + twice the norm of p1's ulps
        floor = 2.0 * float(np.linalg.norm(np.spacing(np.abs(p32)).astype(np.float64)))
        dn = max(dn, (abs(float(np.linalg.norm(p - sd[k].astype(np.float64))) - ref) / (1e-4 * ref + floor), k))
    _check(f"{tag}.param_head_abs", ph, 3e-7)
    print(f"\nMEASURED {tag}.update_norm worst {dn[1]}")
    _check(f"{tag}.update_norm_dev_over_allowed", dn[0], 1.0)
    # the trainer leaves the CLIPPED gradients in .grad (clip_grad_norm_ scales in place): against
    # the reference's gradient norms times its clip coefficient 3 / total norm
    tot = float(np.sqrt(sum(float(s["gnorm." + k]) ** 2 for k, _ in net.named_parameters())))
    coef = min(1.0, 3.0 / (tot + 1e-6))
    gn = max((abs(float(p.grad.double().norm()) - coef * float(s["gnorm." + k])) / (coef * float(s["gnorm." + k])), k)
             for k, p in net.named_parameters())
    print(f"\nMEASURED {tag}.clipped_grad_norm worst {gn[1]} (clip coefficient {coef:.6f})")
    _check(f"{tag}.clipped_grad_norm_rel", gn[0], 2e-5)
    _check(f"{tag}.wb_abs", float(np.abs(np.array([ge2e.w.item(), ge2e.b.item()]) - s["wb1"]).max()), 1e-5)


def test_c5_global_forward_matches_reference():
    """c5's global batch (N=256 x M=10, T=180, fp32) forward + GE2E loss on one GPU against the
    reference's own run (tests/golden/net_fwd_c5.npz): every 8th embedding row, every row's
    projection on 4 fixed directions, the per-embedding loss (the N=256 GE2E path) and the loss."""
    s = golden("net_fwd_c5.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    with torch.no_grad():
        emb = net(x)
        loss = ge2e(emb.reshape(N, M, -1))
        from pytorch_speaker_verification_amd.utils import calc_loss, get_centroids, get_cossim
        E = emb.reshape(N, M, -1)
        _, per = calc_loss(ge2e.w * get_cossim(E, get_centroids(E)) + ge2e.b)
    e = emb.cpu().numpy()
    _check("c5_ref.emb_rows_abs", float(np.abs(e[::8] - s["emb_rows"]).max()), 5e-6)
    _check("c5_ref.emb_proj_abs", float(np.abs(e.astype(np.float64) @ s["dirs"].T - s["emb_proj"]).max()), 2e-5)
    _check("c5_ref.per_abs", float(np.abs(per.cpu().numpy() - s["per"]).max()), 1e-4)
    _check("c5_ref.loss_rel", abs(loss.item() - float(s["loss"])) / abs(float(s["loss"])), 1e-5)


@pytest.mark.parametrize("schedule", ["auto", "per_step"])
def test_full_size_c2_against_torch_gpu(schedule):
    """c2 (N=64 x M=10, T=160) vs the stock-PyTorch fp32 port of the reference on the same GPU:
    'auto' runs the fp32 persistent recurrences at this batch, 'per_step' the K2 / K3 kernels."""
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 160
    sd = recipe.make_weights(2024, *dims, scale=3.0)
    net, ge2e = _build(dims, sd)
    net.schedule = schedule
    tag = "c2" if schedule == "auto" else "c2_per_step"
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.to(DEV)
    x = torch.tensor(recipe.make_frames(1236, N * M, T, dims[0]), device=DEV)
    emb = net(x).reshape(N, M, -1)
    emb_ref = port(x).reshape(N, M, -1)
    _check(f"{tag}.emb_rel_vs_miopen", _rel(emb.detach().cpu().numpy(), emb_ref.detach().cpu().numpy()), 1e-5)
    # unit-norm rows (size-independent property of the projection + L2 norm)
    np.testing.assert_allclose(emb.norm(dim=2).detach().cpu().numpy(), 1.0, atol=1e-5)
    loss = ge2e(emb)
    w = torch.tensor(10.0, device=DEV, requires_grad=True)
    b = torch.tensor(-5.0, device=DEV, requires_grad=True)
    loss_ref = torch_port.ge2e_loss(emb_ref, w, b)
    _check(f"{tag}.loss_rel_vs_miopen", abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()), 1e-6)
    loss.backward()
    loss_ref.backward()
    pr = dict(port.named_parameters())
    g = max(_rel(p.grad.cpu().numpy(), pr[k].grad.cpu().numpy()) for k, p in net.named_parameters())
    _check(f"{tag}.grad_rel_vs_miopen", g, 4e-5)
    _check(f"{tag}.dw_vs_miopen", abs(ge2e.w.grad.item() - w.grad.item()) / max(1, abs(w.grad.item())), 2.5e-5)


def test_dropin_loop_body_c2_against_torch_gpu():
    """A user-written loop of the reference's shape (train_speech_embedder.py:46-65: shuffled rows
    around the forward, zero_grad, forward, GE2E loss, loss.backward(), torch clip_grad_norm_ x2,
    SGD.step) -- bench.user_train_step -- on this package's modules imported the reference's way
    (dropin/) and on the stock-PyTorch port (MIOpen nn.LSTM) on the same GPU, at c2 (N = 64 x
    M = 10, T = 160), two steps from the same weights and the same row orders."""
    import os
    import sys
    import bench
    sys.path.append(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dropin"))
    from speech_embedder_net import GE2ELoss, SpeechEmbedder  # noqa: E402  (the dropin/ shim)
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 160
    sd = recipe.make_weights(2025, *dims, scale=1.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    torch_port.load_recipe_weights(net, sd)
    net = net.to(DEV)
    ge2e = GE2ELoss(DEV)
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.to(DEV)
    ge2e_ref = torch_port.GE2ELossPort(DEV)
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": ge2e.parameters()}], lr=0.01)
    opt_ref = torch.optim.SGD([{"params": port.parameters()}, {"params": ge2e_ref.parameters()}], lr=0.01)
    x = torch.tensor(recipe.make_frames(1237, N * M, T, dims[0]), device=DEV).reshape(N, M, T, dims[0])
    for step in range(2):
        loss = bench.user_train_step(net, ge2e, opt, x, N, M, torch.Generator().manual_seed(step))
        loss_ref = bench.user_train_step(port, ge2e_ref, opt_ref, x, N, M, torch.Generator().manual_seed(step))
        _check(f"dropin_loop_c2.step{step}.loss_rel_vs_miopen",
               abs(loss.item() - loss_ref.item()) / abs(loss_ref.item()), 1e-5)
    pr = dict(port.named_parameters())
    dp = max(float((p.detach() - pr[k].detach()).abs().max()) for k, p in net.named_parameters())
    _check("dropin_loop_c2.params_after_2_steps_vs_miopen", dp, 3e-6)
    _check("dropin_loop_c2.wb_vs_miopen", max(abs(ge2e.w.item() - ge2e_ref.w.item()),
                                              abs(ge2e.b.item() - ge2e_ref.b.item())), 1e-5)


def test_batch_permutation_invariance():
    """The reference permutes rows around the forward (train_speech_embedder.py:48-57);
    rows are independent, so perm -> embed -> unperm equals embed."""
    dims = (40, 128, 2, 64)
    net, _ = _build(dims, recipe.make_weights(3, *dims, scale=2.0))
    x = torch.tensor(recipe.make_frames(4, 24, 30, 40), device=DEV)
    perm = torch.randperm(24, generator=torch.Generator().manual_seed(0)).to(DEV)
    unperm = torch.empty_like(perm)
    unperm[perm] = torch.arange(24, device=DEV)
    a = net(x)
    bb = net(x[perm])[unperm]
    assert torch.equal(a, bb)


def test_ragged_batch_and_seq_sizes():
    """Non-multiple-of-tile batch / time / hidden sizes against the torch port."""
    for dims, B, T in [((40, 96, 1, 24), 7, 5), ((40, 200, 2, 36), 33, 3), ((40, 64, 3, 32), 1, 1)]:
        sd = recipe.make_weights(B * 13 + T, *dims, scale=2.0)
        net, _ = _build(dims, sd)
        port = torch_port.SpeechEmbedderPort(*dims)
        torch_port.load_recipe_weights(port, sd)
        x = torch.tensor(recipe.make_frames(B, B, T, dims[0]))
        e = net(x.to(DEV)).detach().cpu().numpy()
        er = port(x).detach().numpy()
        np.testing.assert_allclose(e, er, atol=5e-5)


def test_bf16_training_lowers_loss_c2():
    """Config c3 trains: a few fused bf16 steps at the full c2 size lower the loss (the
    per-step numerics are pinned to the bf16 oracle in test_gpu_precision.py)."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 160
    sd = recipe.make_weights(2025, *dims, scale=3.0)
    x = torch.tensor(recipe.make_frames(1237, N * M, T, dims[0]), device=DEV)
    net16b, ge16b = _build(dims, sd)
    net16b.precision = "bf16"
    tr = GE2ETrainer(net16b, ge16b, lr=0.01)
    losses = [float(tr.step(x, N, M)) for _ in range(4)]
    tr.check()
    assert losses[-1] < losses[0], losses


def test_c5_per_gpu_shape_f32():
    """BASELINE config c5's per-rank shape (N = 256 over 8 GPUs -> 32 x M = 10, T = 180) in
    fp32 against the stock-PyTorch port on the same GPU (the bf16 form is pinned to the bf16
    oracle in test_gpu_precision.py; the cross-rank exchange by test_gpu_dp / the gloo test)."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    dims, N, M, T = (40, 768, 3, 256), 32, 10, 180
    sd = recipe.make_weights(55, *dims, scale=3.0)
    xh = recipe.make_frames(1238, N * M, T, dims[0])
    net, ge = _build(dims, sd)
    tr = GE2ETrainer(net, ge, lr=0.01)
    loss = float(tr.step(torch.tensor(xh, device=DEV), N, M))
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.to(DEV)
    w = torch.nn.Parameter(torch.tensor(10.0, device=DEV))
    b = torch.nn.Parameter(torch.tensor(-5.0, device=DEV))
    opt = torch.optim.SGD([{"params": port.parameters()}, {"params": [w, b]}], lr=0.01)
    ref = float(torch_port.train_step(port, w, b, opt, torch.tensor(xh, device=DEV), N, M))
    _check("c5_rank.f32_loss_rel_vs_miopen", abs(loss - ref) / abs(ref), 1e-6)
    got = {k: v.detach() for k, v in net.state_dict().items()}
    d = max(float((got[k] - v.detach()).abs().max()) for k, v in port.state_dict().items())
    _check("c5_rank.f32_param_abs_vs_miopen", d, 3e-7)


@pytest.mark.parametrize("dims,N,M,T", [((40, 96, 2, 24), 3, 3, 5),     # B = 9: odd, below every tile
                                        ((40, 64, 3, 32), 2, 2, 1),     # T = 1, M = 2 (leave-one-out of one)
                                        ((40, 72, 2, 20), 5, 7, 37)])   # H = 72, D = 20, T > pipeline chunk
def test_ragged_training_step_against_torch_port(dims, N, M, T):
    """Fused trainer steps (fp32) at ragged sizes against the stock PyTorch port on the host:
    loss, and parameters after two clipped SGD steps."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    sd = recipe.make_weights(N * 31 + M * 7 + T, *dims, scale=2.0)
    x = recipe.make_frames(N + M + T, N * M, T, dims[0])
    net, ge2e = _build(dims, sd)
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    xd = torch.tensor(x, device=DEV)
    losses = [float(tr.step(xd, N, M)) for _ in range(2)]
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    w = torch.nn.Parameter(torch.tensor(10.0))
    b = torch.nn.Parameter(torch.tensor(-5.0))
    opt = torch.optim.SGD([{"params": port.parameters()}, {"params": [w, b]}], lr=0.01)
    ref = [float(torch_port.train_step(port, w, b, opt, torch.tensor(x), N, M)) for _ in range(2)]
    np.testing.assert_allclose(losses, ref, rtol=1e-4)
    got = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    for k, v in port.state_dict().items():
        np.testing.assert_allclose(got[k], v.numpy(), atol=5e-5, err_msg=k)
    np.testing.assert_allclose([ge2e.w.item(), ge2e.b.item()], [w.item(), b.item()], atol=1e-5)


@pytest.mark.parametrize("dims,N,M,T", [((40, 96, 2, 24), 3, 3, 5), ((40, 64, 3, 32), 2, 2, 1),
                                        ((40, 72, 2, 20), 5, 7, 37)])
def test_ragged_training_step_bf16(dims, N, M, T):
    """The bf16-operand step at the same ragged sizes (Bp padding to 8, partial k-tiles, T = 1,
    two pipeline chunks): loss within 1e-2 relative of the fp32 HIP step, finite updates."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    sd = recipe.make_weights(N * 31 + M * 7 + T, *dims, scale=2.0)
    xd = torch.tensor(recipe.make_frames(N + M + T, N * M, T, dims[0]), device=DEV)
    out = {}
    for prec in ("f32", "bf16"):
        net, ge2e = _build(dims, sd)
        net.precision = prec
        tr = GE2ETrainer(net, ge2e, lr=0.01)
        out[prec] = [float(tr.step(xd, N, M)) for _ in range(2)]
        assert all(torch.isfinite(p).all() for p in net.parameters())
    np.testing.assert_allclose(out["bf16"], out["f32"], rtol=1e-2)


@pytest.mark.parametrize("N,M,T", [(10, 10, 37),   # B = 100: a partial second row block, T > pipeline chunk
                                   (3, 3, 2)])     # B = 9, T = 2
def test_f32_persistent_ragged_against_torch_gpu(N, M, T):
    """The fp32 persistent recurrences (forced: schedule 'persist') at ragged batch sizes: one
    fused trainer step against the stock-PyTorch port on the same GPU (loss, parameters)."""
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(N * 13 + T, *dims, scale=3.0)
    xh = recipe.make_frames(N + 7 * T, N * M, T, dims[0])
    net, ge = _build(dims, sd)
    net.schedule = "persist"
    tr = GE2ETrainer(net, ge, lr=0.01)
    loss = float(tr.step(torch.tensor(xh, device=DEV), N, M))
    tr.check()
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.to(DEV)
    w = torch.nn.Parameter(torch.tensor(10.0, device=DEV))
    b = torch.nn.Parameter(torch.tensor(-5.0, device=DEV))
    opt = torch.optim.SGD([{"params": port.parameters()}, {"params": [w, b]}], lr=0.01)
    ref = float(torch_port.train_step(port, w, b, opt, torch.tensor(xh, device=DEV), N, M))
    _check(f"f32_persist_B{N * M}_T{T}.loss_rel_vs_miopen", abs(loss - ref) / abs(ref), 1e-5)
    got = {k: v.detach() for k, v in net.state_dict().items()}
    d = max(float((got[k] - v.detach()).abs().max()) for k, v in port.state_dict().items())
    _check(f"f32_persist_B{N * M}_T{T}.param_abs_vs_miopen", d, 1e-6)


def test_c5_global_step_matches_reference():
    """c5's global batch (N=256 x M=10, T=180) through a whole fp32 training step on one GPU
    (module forward, GE2E, loss.backward(): the per-step kernels at 2560 rows) against the
    reference's own step (tests/golden/net_full_c5.npz): embeddings, loss, every parameter's
    gradient norm and 8x8 head, dL/dw -- the c5 backward pinned to the reference itself, not only
    at the 320-row rank shape."""
    s = golden("net_full_c5.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    emb = net(x).reshape(N, M, -1)
    e = emb.detach().cpu().numpy().reshape(N * M, -1)
    _check("c5_step_ref.emb_rows_abs", float(np.abs(e[::8] - s["emb_rows"]).max()), 5e-6)
    _check("c5_step_ref.emb_proj_abs", float(np.abs(e.astype(np.float64) @ s["dirs"].T - s["emb_proj"]).max()), 2e-5)
    loss = ge2e(emb)
    _check("c5_step_ref.loss_rel", abs(loss.item() - float(s["loss"])) / abs(float(s["loss"])), 1e-5)
    loss.backward()
    _grad_checks("c5_step_ref", net, s)
    from oracle import ge2e_np
    dw64 = ge2e_np.ge2e_backward(emb.detach().cpu().double().numpy(), 10.0, -5.0)[1]
    _check("c5_step_ref.dw_kernel_rel_vs_fp64_on_own_emb", abs(ge2e.w.grad.item() - dw64) / max(1.0, abs(dw64)), 1e-5)


@pytest.mark.parametrize("cfg", ["c2", "c5"])
def test_bf16_path_against_reference_fp32(cfg):
    """The mixed-precision path (c3's numerics: bf16 GEMM operands and bf16 storage, fp32 state,
    accumulation, loss) on the inputs of the reference's own fp32 step (net_full_c2.npz: c2 =
    c3's shape; net_full_c5.npz: c5's global batch), with every deviation bounded against the
    REFERENCE's fp32 values, not the bf16 oracle: loss, embeddings, every parameter's gradient norm.
    The bounds are the mixed-precision tolerance stated in DESIGN §7, about 3-4x the gap measured on
    MI355X (r06: emb 9.4e-4 / 8.2e-4, loss 2.7e-5 / 3.4e-6, grad norms 4.0e-3 / 1.4e-3, dw 3.6e-3 /
    8.2e-4 at c2 / c5)."""
    s = golden(f"net_full_{cfg}.npz")
    dims = tuple(int(v) for v in s["dims"])
    net, ge2e = _build(dims, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    net.precision = "bf16"
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]), device=DEV)
    emb = net(x).reshape(N, M, -1)
    e = emb.detach().cpu().numpy().reshape(N * M, -1)
    ref_e = s["emb"].reshape(N * M, -1) if "emb" in s.files else s["emb_rows"]
    mine = e if "emb" in s.files else e[::8]
    _check(f"bf16_vs_ref_fp32.{cfg}.emb_abs", float(np.abs(mine - ref_e).max()), 3e-3)
    loss = ge2e(emb)
    _check(f"bf16_vs_ref_fp32.{cfg}.loss_rel", abs(loss.item() - float(s["loss"])) / abs(float(s["loss"])), 1e-4)
    loss.backward()
    gn = max((abs(float(p.grad.double().norm()) - float(s["gnorm." + k])) / float(s["gnorm." + k]), k)
             for k, p in net.named_parameters())
    print(f"\nMEASURED bf16_vs_ref_fp32.{cfg}.worst grad_norm {gn[1]}")
    _check(f"bf16_vs_ref_fp32.{cfg}.grad_norm_rel", gn[0], 1.5e-2)
    _check(f"bf16_vs_ref_fp32.{cfg}.dw_rel", abs(ge2e.w.grad.item() - float(s["dw0"])) / max(1.0, abs(float(s["dw0"]))),
           1.5e-2)
