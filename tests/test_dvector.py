"""d-vector helpers (dvector_create.py:38-73).  The reference script runs its whole pipeline at
import time (VAD + librosa + a checkpoint), so these are pinned by hand-computed known answers
rather than by the reference itself ("parity unpinned" beyond these cases)."""
import numpy as np
import pytest
import torch

from pytorch_speaker_verification_amd import dvector


def test_window_frames_counts_and_content():
    m = np.arange(40 * 60, dtype=np.float32).reshape(40, 60)
    w = dvector.window_frames(m)
    # starts 0,12,24 (24+24=48<60); 36+24=60 is not < 60 -> stops
    assert w.shape == (3, 24, 40)
    np.testing.assert_array_equal(w[1], m[:, 12:36].T)
    assert dvector.window_frames(np.zeros((40, 24))).shape == (0, 24, 40)


def test_partitions_known_answer():
    # window i ends at 0.12 i + 0.24; segment j closes at 0.401 j
    assert dvector.partitions(6) == [(0, 2), (2, 5), (5, 6)]
    assert dvector.partitions(1) == [(0, 1)]
    e = np.arange(12, dtype=np.float64).reshape(6, 2)
    np.testing.assert_allclose(dvector.align_embeddings(e), [[1, 2], [6, 7], [10, 11]])


@pytest.mark.gpu
def test_embed_windows_short_sequence_large_batch():
    """T = 24 windows, thousands at once (the inference point of the kernel design space),
    against the stock-PyTorch port."""
    import recipe
    from conftest import model_dims
    from oracle import torch_port
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(9, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.cuda()
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.cuda()
    x = recipe.make_frames(10, 3000, 24, 40)
    e = dvector.embed_windows(net, x, batch=1024).cpu().numpy()
    with torch.no_grad():
        er = port(torch.tensor(x).cuda()).cpu().numpy()
    np.testing.assert_allclose(e, er, atol=5e-5)


@pytest.mark.gpu
def test_embed_windows_bf16_against_bf16_oracle():
    """bf16 d-vectors (the c3 mixed-precision forward at T = 24, 512 windows) against the
    bf16-operand oracle (oracle/lstm_bf16.py) and the fp32 path.  Measured on MI355X with these
    (scale-2) weights: 4.9e-4 vs the oracle, 1.0e-3 vs fp32 (random-init net, 16384 windows:
    1.4e-4 vs fp32, min cosine 0.9999997); tolerance 5e-3, the c3/c4 embedding bound."""
    import recipe
    from conftest import model_dims
    from oracle import lstm_bf16
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(9, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.cuda()
    x = recipe.make_frames(11, 512, 24, 40)
    e16 = dvector.embed_windows(net, x, batch=512, precision="bf16").cpu().numpy()
    e32 = dvector.embed_windows(net, x, batch=512).cpu().numpy()
    eo, _ = lstm_bf16.embedder_forward(sd, x, 3, bf16=True)
    eo = eo.numpy()
    d_or = float(np.abs(e16 - eo).max())
    d_32 = float(np.abs(e16 - e32).max())
    print(f"\nMEASURED dvector_bf16 vs bf16 oracle max-abs {d_or:.2e}; vs fp32 {d_32:.2e}")
    assert d_or <= 5e-3 and d_32 <= 5e-3, (d_or, d_32)
    with pytest.raises(ValueError):
        dvector.embed_windows(net, x[:4], precision="fp16")


def test_embed_windows_rejects_unknown_precision():
    """The precision switch is validated before any device work (CPU-only check)."""
    with pytest.raises(ValueError):
        dvector.embed_windows(None, np.zeros((1, 24, 40), np.float32), precision="fp16")


@pytest.mark.gpu
@pytest.mark.parametrize("S", [512, 300])
def test_embed_windows_dvec_path_against_bf16_oracle(S):
    """The large-batch bf16 path (sv_dvector_embed_bf16: one 256 x 256 GEMM launch per timestep
    and layer over [x_t | h_{t-1}] with the LSTM cell in its epilogue; S = 300 pads the rows to
    512) against the bf16-operand oracle (oracle/lstm_bf16.py: the same bf16 rounding of the
    operands and of the input projection with its biases) and against the persistent bf16 path.
    The only difference from the oracle is the fp32 order of the h part's sum (MFMA k-steps added
    onto the rounded input projection), amplified through 24 steps x 3 layers."""
    import recipe
    from conftest import model_dims
    from oracle import lstm_bf16
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(9, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.cuda()
    x = recipe.make_frames(12, S, 24, 40)
    ed = dvector.embed_windows(net, x, precision="bf16", path="dvec").cpu().numpy()
    ep = dvector.embed_windows(net, x, precision="bf16", path="persist").cpu().numpy()
    eo, _ = lstm_bf16.embedder_forward(sd, x, 3, bf16=True)
    eo = eo.numpy()
    assert ed.shape == (S, 256) and np.isfinite(ed).all()
    d_or = float(np.abs(ed - eo).max())
    d_p = float(np.abs(ed - ep).max())
    print(f"\nMEASURED dvector_dvec_bf16[S={S}] vs bf16 oracle max-abs {d_or:.2e}; vs persistent bf16 {d_p:.2e}")
    assert d_or <= 5e-3 and d_p <= 5e-3, (d_or, d_p)
    np.testing.assert_allclose(np.linalg.norm(ed, axis=1), 1.0, atol=1e-5)


@pytest.mark.gpu
def test_embed_windows_dvec_auto_large_batch():
    """From DVEC_MIN windows on, embed_windows(precision='bf16') takes the per-step GEMM path;
    4096 windows of a random-init net against the fp32 path (bf16-level agreement)."""
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    torch.manual_seed(3)
    net = SpeechEmbedder().cuda()
    x = np.random.default_rng(4).standard_normal((4096, 24, 40)).astype(np.float32)
    assert x.shape[0] >= dvector.DVEC_MIN
    e16 = dvector.embed_windows(net, x, precision="bf16").cpu().numpy()
    e32 = dvector.embed_windows(net, x).cpu().numpy()
    d = float(np.abs(e16 - e32).max())
    cos = float((e16 * e32).sum(1).min())
    print(f"\nMEASURED dvector_dvec_bf16[4096] vs fp32 max-abs {d:.2e}, min cosine {cos:.7f}")
    assert d <= 5e-3 and cos > 0.9999, (d, cos)


def test_dvec_path_dimension_rule():
    """The large-batch bf16 path's dimension rule mirrors sv_dvector_embed_bf16's argument checks
    (include/sv_ge2e.h): model dims it cannot take fall back to the persistent batches."""
    assert dvector.dvec_ok(40, 768)
    assert not dvector.dvec_ok(80, 768)   # x part wider than one 64-column k-tile
    assert not dvector.dvec_ok(40, 96)    # 4H = 384: not whole 256-column tiles
    assert dvector.dvec_ok(40, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_graphed_per_file_calls_match_embed_windows(precision):
    """Per-file calls replayed from HIP graphs (dvector.GraphedEmbedder): the same kernels as
    embed_windows(..., batch=S), so a file whose window count is a whole bucket is bit-identical;
    one padded up to its bucket (zero rows, rows independent) agrees to fp32 rounding; repeated
    replays of one graph with new windows stay right; an in-place weight update is seen."""
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(19, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.cuda()
    ge = dvector.GraphedEmbedder(net, precision=precision)
    for seed, S in ((20, 128), (21, 128), (22, 100), (23, 37)):
        x = recipe.make_frames(seed, S, 24, 40)
        got = ge(x).cpu()
        ref = dvector.embed_windows(net, x, batch=S, precision=precision).cpu()
        assert got.shape == ref.shape
        dev = float((got - ref).abs().max())
        print(f"\nMEASURED graphed_{precision}_S{S} {dev:.3e}")
        if S % 32 == 0:
            assert dev == 0.0, (S, dev)
        else:
            assert dev <= (5e-3 if precision == "bf16" else 1e-5), (S, dev)
    with torch.no_grad():
        net.projection.bias.add_(0.5)
    x = recipe.make_frames(24, 128, 24, 40)
    assert float((ge(x).cpu() - dvector.embed_windows(net, x, batch=128, precision=precision).cpu()).abs().max()) == 0.0

@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_graphed_persistent_replays_interleaved_with_eager(precision):
    """Regression for r03's graph-replay mismatch: GraphedEmbedder with the persistent recurrences
    forced (schedule 'persist'), replays of three bucket graphs (128, 64, 640 windows) interleaved
    with eager persistent calls of the same shapes, twice over, each replay checked bit for bit
    against the eager persistent call, and both against the per-step schedule (bf16: bit-identical
    by construction; fp32: within 1e-5, its persistent layer 0 forms the input projection in the
    recurrence).  With the
    arrival counters reset by a hipMemsetAsync, 16-22 of 24 such replays came out wrong (one XCD's
    workgroups read a hand-off early; scripts/f32_replay_diag.py); the counters are now zeroed by a
    kernel (sv_zero_counters).  Padded buckets (100, 37 windows) agree to fp32 rounding."""
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(19, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.cuda()
    ge = dvector.GraphedEmbedder(net, precision=precision, schedule="persist")
    worst = 0.0
    for rep in range(2):
        for seed, S in ((20, 128), (21, 128), (22, 100), (23, 37), (25, 640), (26, 640)):
            x = recipe.make_frames(seed + 100 * rep, S, 24, 40)
            got = ge(x).cpu()
            eager = dvector.embed_windows(net, x, batch=S, precision=precision, schedule="persist").cpu()
            ref = dvector.embed_windows(net, x, batch=S, precision=precision, schedule="per_step").cpu()
            d_eager = float((eager - ref).abs().max())
            d_graph = float((got - ref).abs().max())
            worst = max(worst, d_graph)
            # bf16: persistent and per-step are bit-identical; fp32: they agree to rounding (the
            # persistent layer 0 forms its input projection in the recurrence), and the replay must
            # equal the eager persistent call bit for bit
            assert d_eager <= (0.0 if precision == "bf16" else 1e-5), (rep, S, d_eager)
            if S % 32 == 0:
                assert torch.equal(got, eager), (rep, S, float((got - eager).abs().max()))
            else:
                assert d_graph <= (5e-3 if precision == "bf16" else 1e-5), (rep, S, d_graph)
    print(f"\nMEASURED graphed_persist_{precision} worst vs per-step {worst:.3e}")
