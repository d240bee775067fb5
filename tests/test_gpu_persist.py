"""The persistent recurrence schedule (one launch per layer for all T, sv_persist.hip) must
reproduce the per-step-launch schedule bit for bit: same tiles, same MFMA order, same K1 GEMMs
(fp32 accumulation of identical products), only the launch structure and the h hand-off differ.
The schedules are selected per call (the C ABI's `schedule` flags, include/sv_ge2e.h)."""
import numpy as np
import pytest

import schedules

pytestmark = pytest.mark.gpu


def _run(tag, schedule, dims, N, M, T, precision="bf16"):
    return schedules.run(dims, N, M, T, precision, schedule)


@pytest.mark.parametrize("dims,N,M,T", [((40, 768, 3, 256), 64, 10, 12),   # c3 grid: 24 x 10 workgroups
                                        ((40, 768, 3, 256), 64, 10, 40),   # c3, hand-off slots past T = 33
                                        ((40, 768, 2, 256), 16, 10, 7),    # B = 160: 32-row tiles
                                        ((40, 96, 2, 32), 7, 5, 9)])       # ragged rows (B = 35)
def test_persistent_fwd_bf16_equals_per_step(dims, N, M, T):
    a = _run("step", "per_step", dims, N, M, T)
    b = _run("persist", "persist", dims, N, M, T)
    assert int(b["status"][0]) == 0
    # the forward's outputs; the step's gradients and update are the backward test's
    for k in a:
        if k in ("emb", "h_last", "loss") or k.startswith(("gates", "c")):
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)


@pytest.mark.parametrize("N,M,T", [(32, 10, 9),    # c5's per-rank 320 rows: 20 x 12 workgroups
                                   (32, 9, 7)])    # 288 rows: 18 row blocks
def test_persistent_fwd_bf16_16row_tile_against_per_step(N, M, T):
    """The 16-row wide forward (lstm_persist16_fwd_bf16_kernel, chosen for 257..320 rows, layer 0's
    x-projection fused) against the per-step schedule, bit for bit: its v_mfma_f32_16x16x32_bf16 sums
    each pre-activation over 32-wide k blocks where the per-step kernels' 32x32x16 sums 16-wide ones,
    in the same k order -- measured identical on gfx950 (r06), and asserted so."""
    dims = (40, 768, 3, 256)
    a = _run("step", "per_step", dims, N, M, T)
    b = _run("persist", "persist", dims, N, M, T)
    assert int(b["status"][0]) == 0
    for k in a:
        if k in ("emb", "h_last", "loss") or k.startswith(("gates", "c")):
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)


@pytest.mark.parametrize("dims,N,M,T", [((40, 768, 3, 256), 64, 10, 12),   # c3 grid: 24 x 10 workgroups
                                        ((40, 768, 3, 256), 64, 10, 40),   # c3, hand-off slots past T = 33
                                        ((40, 768, 3, 256), 56, 10, 9),    # B = 560: wide tiles, row-major dG
                                        ((40, 768, 2, 256), 16, 10, 7),    # B = 160: 32-row tiles
                                        ((40, 96, 2, 32), 7, 5, 9),        # ragged rows (B = 35)
                                        ((40, 64, 3, 32), 4, 5, 7)])       # H = 64: 2 unit blocks
def test_persistent_bwd_bf16_equals_per_step(dims, N, M, T):
    """W-stationary persistent backward recurrence (one launch per layer, dG handed off through
    HBM) vs per-step launches: the same per-gate MFMA order and the same gate-order sum, so dG,
    the weight gradients and dx are bit-identical (the weight gradients: where both schedules sum
    K = T Bp in one order, see below).  The bias gradients are summed inside the
    persistent kernel (over t per element, then rows, then row blocks) instead of by a row-sum
    kernel over dG^T: the same bf16 values in another fp32 order."""
    a = _run("step", "per_step", dims, N, M, T)
    b = _run("persist", "persist", dims, N, M, T)
    assert int(b["status"][0]) == 0
    np.testing.assert_array_equal(b["loss"], a["loss"])
    grads = [k for k in a if k.startswith("grad_")]
    assert len(grads) == 4 * dims[2] + 2
    # where the dx GEMM over all T (T * B / 256 * H / 256 tiles) exceeds one round of the 256 CUs,
    # the persistent schedule runs it as one whole-T GEMM while the per-step schedule runs it in
    # time chunks: the layers below the top then see dx summed in another fp32 order (measured
    # 2.3e-7 relative, r05_v10); the top layer, the projection and the loss stay bit-identical.  The
    # bound is ~40x that: a dropped or double-counted k-piece moves a gradient by O(1e-2)
    H = dims[1]
    sk = H == 768 and (T * N * M) % 256 == 0 and (T * N * M // 256) * (H // 256) > 256
    # r06: with 3 layers at H = 768 the persistent schedule forms every layer's weight gradients
    # after the last recurrence as ONE whole-K launch (one accumulator over K = T Bp, layer 0's
    # dW_ih as a partial tile of it); where the per-step schedule splits that K (split-K slabs:
    # dW_hh / dW_ih of the upper layers at K >= 8192, layer 0's narrow dW_ih always) they are the same
    # products summed in another fp32 order (bound 1e-5 relative, measured in the MEASURED line)
    Bp = (N * M + 7) // 8 * 8
    fk = dims[2] == 3 and H == 768 and (T * Bp) % 64 == 0
    top = f"_l{dims[2] - 1}"
    worst = worst_w = 0.0
    for k in grads:
        rel = float(np.abs(b[k] - a[k]).max()) / max(float(np.abs(a[k]).max()), 1e-30)
        if sk and top not in k and "projection" not in k:
            worst = max(worst, rel)
            assert rel <= 1e-5, (k, rel)
        elif ".bias_" in k:
            np.testing.assert_allclose(b[k], a[k], rtol=1e-5, atol=1e-6 * np.abs(a[k]).max(), err_msg=k)
        elif fk and ".weight_" in k and "projection" not in k:
            worst_w = max(worst_w, rel)
            assert rel <= 1e-5, (k, rel)
        else:
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)
    if sk:
        print(f"\nMEASURED persist_vs_per_step_bf16.T{T}.lower_layer_grad_rel {worst:.2e} (stream-K dx)")
    if fk:
        print(f"\nMEASURED persist_vs_per_step_bf16.T{T}.weight_grad_rel {worst_w:.2e} (whole-K dW)")
    np.testing.assert_allclose(b["flat_p"], a["flat_p"], rtol=0, atol=1e-6 if (sk or fk) else 1e-7)


@pytest.mark.parametrize("N,M,T", [(32, 10, 9),    # c5's per-rank 320 rows: 20 x 12 workgroups
                                   (33, 9, 7)])    # 297 rows: a partial last 16-row block
def test_persistent_bwd_bf16_16row_tile_against_per_step(N, M, T):
    """257..336 rows (c5's rank shape) through the persistent backward (the 32 x 32 tile) against
    the per-step schedule: the same products, the dx GEMM's K summed in another order (measured
    2.2e-7).  The oracle test of this shape is
    test_gpu_precision.py::test_c5_rank_shape_bf16_against_oracle; the loss is bit-identical."""
    dims = (40, 768, 3, 256)
    a = _run("step", "per_step", dims, N, M, T)
    b = _run("persist", "persist", dims, N, M, T)
    assert int(b["status"][0]) == 0
    np.testing.assert_array_equal(b["loss"], a["loss"])
    worst = 0.0
    for k in a:
        if not k.startswith("grad_"):
            continue
        dev = float(np.abs(b[k] - a[k]).max()) / max(float(np.abs(a[k]).max()), 1e-30)
        worst = max(worst, dev)
        assert dev <= 1e-5, (k, dev)   # measured 2.2e-7 (r05_v10)
    print(f"\nMEASURED persist_c5rows_vs_per_step_bf16.B{N * M}.grad_rel {worst:.2e}")
    np.testing.assert_allclose(b["flat_p"], a["flat_p"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("N,M,T", [(8, 10, 20),    # c4's per-rank shape: 3 x 3 x 24 = 216 workgroups
                                   (7, 5, 9)])     # ragged rows (B = 35, 2 row blocks)
def test_wavefront_fwd_bf16_against_per_layer(N, M, T):
    """Layer-wavefront forward (sv_wave.hip: all layers in one launch, input projection in the
    recurrence) vs the per-layer persistent schedule (K1 GEMM + one launch per layer): the same
    bf16 products, summed in another order (x and h parts in one accumulator), so agreement to
    bf16-operand level; then the training step through it."""
    dims = (40, 768, 3, 256)
    a = _run("layer", "per_layer", dims, N, M, T)
    b = _run("wave", "auto", dims, N, M, T)
    assert int(a["status"][0]) == 0 and int(b["status"][0]) == 0
    for k in ("gates0", "c0", "gates1", "c1", "gates2", "c2"):
        d = float(np.abs(b[k] - a[k]).max())
        print(f"\nMEASURED wave_fwd_vs_layer.{k} {d:.3e}")
        assert d < 2e-2, (k, d)
    d = float(np.abs(b["emb"] - a["emb"]).max())
    print(f"\nMEASURED wave_fwd_vs_layer.emb {d:.3e}")
    assert d < 5e-3, d
    np.testing.assert_allclose(b["loss"], a["loss"], rtol=1e-3)


@pytest.mark.parametrize("N,M,T", [(8, 10, 20),    # c4's per-rank shape: 3 x 24 x 3 = 216 workgroups
                                   (7, 5, 9)])     # ragged rows (B = 35: padded dG^T columns)
def test_wavefront_bwd_bf16_against_per_layer(N, M, T):
    """Layer-wavefront backward (lstm_wave_bwd_bf16_kernel: all layers' recurrences and dx in one
    launch) vs the per-layer schedule (one persistent launch + dx GEMM per layer).  The layers'
    dh_rec sums are ordered alike; dx is summed per gate then across gates (the GEMM: over K in
    k-tile order), so the lower layers see fp32-reordered upstream gradients that bf16 rounding of
    dG can amplify to a few bf16 ulps: agreement at bf16-operand level."""
    dims = (40, 768, 3, 256)
    a = _run("layer", "per_layer", dims, N, M, T)
    b = _run("wave", "auto", dims, N, M, T)
    assert int(a["status"][0]) == 0 and int(b["status"][0]) == 0
    d = abs(float(b["loss"][0]) - float(a["loss"][0])) / abs(float(a["loss"][0]))
    print(f"\nMEASURED wave_vs_layer.loss_rel {d:.3e}")
    assert d < 1e-3, d   # the forward wavefront differs from the per-layer forward at bf16 level
    grads = [k for k in a if k.startswith("grad_")]
    assert len(grads) == 4 * dims[2] + 2
    worst = 0.0
    for k in grads:
        d = float(np.abs(b[k] - a[k]).max() / max(np.abs(a[k]).max(), 1e-30))
        worst = max(worst, d)
        print(f"\nMEASURED wave_bwd_vs_layer.{k} {d:.3e}")
        assert d < 2e-2, (k, d)
    print(f"\nMEASURED wave_bwd_vs_layer.worst {worst:.3e}")


@pytest.mark.parametrize("precision", ["f32", "bf16"])
@pytest.mark.parametrize("B", [128, 640])
def test_graph_replayed_persistent_forward_state_bit_exact(precision, B):
    """The persistent forward captured in a HIP graph (save=True, so every layer's h_tm / gates /
    c_tm stays reachable), replayed with new frames, each replay followed by an eager persistent
    call of the same shape: every layer's h_tm (including slot 0, the zero initial state), gates
    and c_tm must equal, bit for bit, the per-step schedule's (bf16) or the eager persistent call's
    (fp32, whose layer 0 forms its input projection in the recurrence; per-step within 1e-5).  Before every zeroing in the library
    went through a kernel (sv_zero_bytes / sv_zero_counters), the replays left junk in the
    memset-zeroed arrival counters and h_tm slot 0, and one XCD's workgroups read a hand-off
    early (scripts/f32_replay_diag.py)."""
    import torch
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd._lib import PersistStatus
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dev = torch.device("cuda", 0)
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(19, *dims, scale=2.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    layers = net.LSTM_stack.layer_params()
    wp, bp = net.projection.weight, net.projection.bias
    fwd = ops.embedder_forward_bf16 if precision == "bf16" else ops.embedder_forward
    st_ = PersistStatus(dev)
    xs = torch.zeros((B, 24, 40), device=dev)

    def f():
        return fwd(xs, layers, wp, bp, save=True, schedule="persist", status=st_)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        f()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        emb, st = f()
    for rep in range(4):
        x = torch.as_tensor(recipe.make_frames(300 + rep, B, 24, 40)).to(dev)
        xs.copy_(x)
        g.replay()
        eag, est = fwd(x, layers, wp, bp, save=True, schedule="persist")
        if precision == "f32":
            # fp32: the persistent forward forms layer 0's input projection inside the recurrence
            # (a different summation order from the per-step schedule's K1 GEMM + K2), so the bit-exact
            # reference is the eager persistent call, and the per-step schedule agrees to rounding
            per, _ = fwd(x, layers, wp, bp, save=False, schedule="per_step")
            torch.cuda.synchronize()
            assert float((eag - per).abs().max()) < 1e-5, (rep, float((eag - per).abs().max()))
            ref, rst = eag, est
        else:
            ref, rst = fwd(x, layers, wp, bp, save=True, schedule="per_step")
        torch.cuda.synchronize()
        assert int(st_.block[0]) == 0
        assert torch.equal(emb, ref), (rep, float((emb - ref).abs().max()))
        for l in range(3):
            # (bf16: the persistent kernels keep fp32 h only for the last step; the bf16 copies of
            # h, the next layer's input, are x_tm[l + 1])
            if precision == "f32":
                assert torch.equal(st.h_tm[l], rst.h_tm[l]), (rep, l, "h_tm")
                assert float(st.h_tm[l][0].abs().max()) == 0.0
            elif l + 1 < 3:
                assert torch.equal(st.x_tm[l + 1], rst.x_tm[l + 1]), (rep, l, "h_bf")
            assert torch.equal(st.gates[l], rst.gates[l]), (rep, l, "gates")
            assert torch.equal(st.c_tm[l], rst.c_tm[l]), (rep, l, "c_tm")
        assert torch.equal(st.h_last, rst.h_last), (rep, "h_last")


@pytest.mark.parametrize("N,M,T", [(8, 10, 160),   # c4's per-rank shape: whole-K tiles + first pieces (split form)
                                   (8, 10, 40)])
def test_wavefront_weight_gradients_against_fp64_of_same_operands(N, M, T):
    """The layer wavefront's weight gradients (gemm_bf16_8qf_kernel: every layer's 256 x 256 tiles
    in one launch; at the c4 rank shape the free CUs compute each tile's first k-tiles and hand the
    fp32 partial over through a flag) against an fp64 product of the SAME bf16 operands the launch
    reads -- dG^T (st.dgT) times the time-shifted h^T / x^T -- bounded at fp32 level per element
    (1e-5 of the sum of |products|): a stale partial from the previous step, a lost flag, or a wrong
    first-piece / whole-K k split moves an element by O(1) of that bound.  Two consecutive backward
    calls on different inputs, so a partial left over from the first would show in the second."""
    import torch
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd._lib import lib
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dev = torch.device("cuda", 0)
    dims = (40, 768, 3, 256)
    B, H, F = N * M, dims[1], dims[0]
    assert lib().sv_wave_ok(3, T, B, F, H)
    sd = recipe.make_weights(77, *dims, scale=3.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    layers = net.LSTM_stack.layer_params()
    wp, bp = net.projection.weight, net.projection.bias
    Bp = (B + 7) // 8 * 8
    worst = 0.0
    for rep in range(2):
        x = torch.as_tensor(recipe.make_frames(500 + rep, B, T, F)).to(dev)
        demb = torch.as_tensor(np.random.default_rng(600 + rep).standard_normal((B, dims[3])).astype(np.float32)).to(dev)
        emb, st = ops.embedder_forward_bf16(x, layers, wp, bp, save=True)
        grads = ops.embedder_backward_bf16(st, demb, layers, wp)
        torch.cuda.synchronize()
        for l in range(3):
            A = st.dgT[l].double()                                   # [4H, T Bp]
            hprev = st.hT[l][:, :T * Bp].double()                    # column block t = h_{t-1}
            xin = (st.xT0 if l == 0 else st.hT[l - 1][:, Bp:(T + 1) * Bp]).double()
            for name, Bop, got in (("w_hh", hprev, grads[4 * l + 1]), ("w_ih", xin, grads[4 * l])):
                ref = A @ Bop.T
                bound = A.abs() @ Bop.abs().T
                err = ((got.double() - ref).abs() / (bound + 1e-30)).max().item()
                worst = max(worst, err)
                assert err <= 1e-5, (rep, l, name, err)
    print(f"\nMEASURED wave_dw_vs_fp64_same_operands.T{T} {worst:.2e} (of sum |products|)")


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,schedule", [(80, 24, "auto"), (320, 12, "auto"), (64, 8, "per_step")])
def test_weights_bf16_transposes_handed_to_the_backward(B, T, schedule):
    """sv_lstm_weights_bf16 (ABI v10): the forward's one launch writes every layer's bf16 weights
    and, into the stack backward's workspace, the transposes that backward would otherwise form;
    SV_SCHED_WT_READY makes the backward use them.  The gradients must be bit-identical to a
    backward that transposes on its own (st.bws dropped), under the wavefront (B = 80), persistent
    (B = 320) and per-step schedules; the row-major copies must equal torch's bf16 rounding."""
    import recipe
    import torch
    from conftest import model_dims
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd._lib import call, stream_of
    from pytorch_speaker_verification_amd.ops import _parr
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dev = torch.device("cuda", 0)
    dims = (40, 768, 3, 256)
    F, H = dims[0], dims[1]
    sd = recipe.make_weights(91, *dims, scale=3.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    layers = net.LSTM_stack.layer_params()
    wp, bp = net.projection.weight, net.projection.bias
    x = torch.as_tensor(recipe.make_frames(700, B, T, F)).to(dev)
    demb = torch.as_tensor(np.random.default_rng(701).standard_normal((B, dims[3])).astype(np.float32)).to(dev)
    out = []
    for handed in (True, False):
        emb, st = ops.embedder_forward_bf16(x, layers, wp, bp, save=True, schedule=schedule)
        assert st.bws is not None
        if not handed:
            st.bws = None
        out.append([g.clone() for g in ops.embedder_backward_bf16(st, demb, layers, wp, schedule=schedule)])
    torch.cuda.synchronize()
    for a, b in zip(*out):
        assert torch.equal(a, b)
    # the row-major copies alone (no workspace) against torch's RNE rounding
    wih = [torch.empty_like(l[0], dtype=torch.bfloat16) for l in layers]
    whh = [torch.empty_like(l[1], dtype=torch.bfloat16) for l in layers]
    call("sv_lstm_weights_bf16", 3, T, B, F, H, _parr([l[0] for l in layers]), _parr([l[1] for l in layers]),
         _parr(wih), _parr(whh), None, stream_of(x))
    torch.cuda.synchronize()
    for l in range(3):
        assert torch.equal(wih[l], layers[l][0].to(torch.bfloat16))
        assert torch.equal(whh[l], layers[l][1].to(torch.bfloat16))
    # sv_lstm_prep_bf16 (ABI v11): the frames' launch folded into the weights' one -- the same bytes
    # as sv_frames_to_bf16 + sv_lstm_weights_bf16 (padding columns of x^T included)
    Bp = (B + 7) // 8 * 8
    outs = []
    for fused in (True, False):
        xb = torch.full((T, B, F), float("nan"), device=dev).bfloat16()
        xT = torch.full((F, T * Bp), float("nan"), device=dev).bfloat16()
        wi = [torch.zeros_like(l[0], dtype=torch.bfloat16) for l in layers]
        wh = [torch.zeros_like(l[1], dtype=torch.bfloat16) for l in layers]
        wargs = (_parr([l[0] for l in layers]), _parr([l[1] for l in layers]), _parr(wi), _parr(wh), None,
                 stream_of(x))
        if fused:
            call("sv_lstm_prep_bf16", 3, T, B, F, H, x.data_ptr(), xb.data_ptr(), xT.data_ptr(), Bp, *wargs)
        else:
            call("sv_frames_to_bf16", x.data_ptr(), B, T, F, xb.data_ptr(), xT.data_ptr(), Bp, stream_of(x))
            call("sv_lstm_weights_bf16", 3, T, B, F, H, *wargs)
        torch.cuda.synchronize()
        outs.append([xb, xT] + wi + wh)
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert torch.equal(outs[0][0].float(), x.transpose(0, 1).bfloat16().float())


@pytest.mark.gpu
@pytest.mark.parametrize("B,schedule", [(80, "auto"), (320, "per_layer")])
def test_second_backward_zeroes_its_own_counters(B, schedule):
    """SV_SCHED_CNT_READY (ABI v11): the stack forward zeroes the backward's counter channels, so the
    first backward on its sync block launches no zeroing; a second backward of the same forward on
    the same block (as retain_graph would run it) must zero them itself -- with stale counters its
    hand-off waits would pass at once.  Both backwards must give the same gradients bit for bit."""
    import recipe
    import torch
    from conftest import model_dims
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dev = torch.device("cuda", 0)
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(23, *dims, scale=3.0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd._lib import PersistStatus
    layers = net.LSTM_stack.layer_params()
    wp, bp = net.projection.weight, net.projection.bias
    x = torch.as_tensor(recipe.make_frames(24, B, 12, 40)).to(dev)
    demb = torch.as_tensor(np.random.default_rng(25).standard_normal((B, 256)).astype(np.float32)).to(dev)
    status = PersistStatus(dev)  # one caller-owned sync block for the forward and both backwards
    _, st = ops.embedder_forward_bf16(x, layers, wp, bp, save=True, status=status, schedule=schedule)
    assert status.bwd_counters_clean
    g = []
    for _ in range(2):
        g.append([t.clone() for t in ops.embedder_backward_bf16(st, demb, layers, wp, status=status,
                                                                 schedule=schedule)])
        assert not status.bwd_counters_clean
    torch.cuda.synchronize()
    status.poll(wait=True)
    assert int(status.block[0]) == 0
    for a, b in zip(*g):
        assert torch.equal(a, b)
