"""The persistent recurrence schedule (one launch per layer for all T, sv_persist.hip) must
reproduce the per-step-launch schedule bit for bit: same tiles, same MFMA order, same K1 GEMMs
(fp32 accumulation of identical products), only the launch structure and the h hand-off differ.
Each schedule runs in its own process (the library reads SV_PERSIST once)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(tmp_path, tag, env_extra, dims, N, M, T, precision):
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "_schedule_worker.py"), out, ",".join(map(str, dims)),
                        str(N), str(M), str(T), precision], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return dict(np.load(out))


@pytest.mark.parametrize("dims,N,M,T", [((40, 768, 3, 256), 64, 10, 12),   # c3 grid: 24 x 10 workgroups
                                        ((40, 768, 2, 256), 16, 10, 7),    # B = 160: 32-row tiles
                                        ((40, 96, 2, 32), 7, 5, 9)])       # ragged rows (B = 35)
def test_persistent_fwd_bf16_equals_per_step(tmp_path, dims, N, M, T):
    a = _run(tmp_path, "step", {"SV_PERSIST": "0", "SV_WAVEFRONT": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "persist", {"SV_PERSIST": "1"}, dims, N, M, T, "bf16")
    assert int(b["status"][0]) == 0
    for k in a:
        if k == "status":
            continue
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)


def test_wavefront_fwd_bf16_equals_per_step(tmp_path):
    """The wavefront schedule (all layers per launch, two K segments per tile) changes only the
    accumulation split of the upper layers' pre-activations: fp32-rounding-level agreement."""
    dims, N, M, T = (40, 96, 3, 32), 6, 4, 10
    a = _run(tmp_path, "step", {"SV_PERSIST": "0", "SV_WAVEFRONT": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "wave", {"SV_PERSIST": "0", "SV_WAVEFRONT": "1"}, dims, N, M, T, "bf16")
    for k in ("gates0", "c0"):
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)   # layer 0 is computed identically
    for k in ("gates1", "gates2", "c2", "emb", "loss"):
        np.testing.assert_allclose(b[k], a[k], rtol=2e-2, atol=2e-2, err_msg=k)


@pytest.mark.parametrize("dims,N,M,T", [((40, 768, 3, 256), 64, 10, 12),   # c3 grid: 24 x 10 workgroups
                                        ((40, 768, 2, 256), 16, 10, 7),    # B = 160: 32-row tiles
                                        ((40, 96, 2, 32), 7, 5, 9),        # ragged rows (B = 35)
                                        ((40, 64, 3, 32), 4, 5, 7)])       # H = 64: 2 unit blocks
def test_persistent_bwd_bf16_equals_per_step(tmp_path, dims, N, M, T):
    """W-stationary persistent backward recurrence (one launch per layer, dG handed off through
    HBM) vs per-step launches: the same per-gate MFMA order and the same gate-order sum, so dG,
    the weight gradients and dx are bit-identical.  The bias gradients are summed inside the
    persistent kernel (over t per element, then rows, then row blocks) instead of by a row-sum
    kernel over dG^T: the same bf16 values in another fp32 order."""
    a = _run(tmp_path, "step", {"SV_PERSIST_BWD": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "persist", {"SV_PERSIST_BWD": "1"}, dims, N, M, T, "bf16")
    c = _run(tmp_path, "persist_side", {"SV_PERSIST_BWD": "1", "SV_PBWD_DW_SIDE": "1"}, dims, N, M, T, "bf16")
    assert int(b["status"][0]) == 0 and int(c["status"][0]) == 0
    np.testing.assert_array_equal(b["loss"], a["loss"])
    np.testing.assert_array_equal(c["loss"], a["loss"])
    grads = [k for k in a if k.startswith("grad_")]
    assert len(grads) == 4 * dims[2] + 2
    for k in grads:
        for other in (b, c):
            if ".bias_" in k:
                np.testing.assert_allclose(other[k], a[k], rtol=1e-5, atol=1e-6 * np.abs(a[k]).max(), err_msg=k)
            else:
                np.testing.assert_array_equal(other[k], a[k], err_msg=k)
    for other in (b, c):
        np.testing.assert_allclose(other["flat_p"], a["flat_p"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("N,M,T", [(8, 10, 20),    # c4's per-rank shape: 3 x 3 x 24 = 216 workgroups
                                   (7, 5, 9)])     # ragged rows (B = 35, 2 row blocks)
def test_wavefront_fwd_bf16_against_per_layer(tmp_path, N, M, T):
    """Layer-wavefront forward (sv_wave.hip: all layers in one launch, input projection in the
    recurrence) vs the per-layer persistent schedule (K1 GEMM + one launch per layer): the same
    bf16 products, summed in another order (x and h parts in one accumulator), so agreement to
    bf16-operand level; then the training step through it."""
    dims = (40, 768, 3, 256)
    a = _run(tmp_path, "layer", {"SV_WAVE2": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "wave", {"SV_WAVE2": "1"}, dims, N, M, T, "bf16")
    assert int(a["status"][0]) == 0 and int(b["status"][0]) == 0
    for k in ("gates0", "c0", "gates1", "c1", "gates2", "c2"):
        d = float(np.abs(b[k] - a[k]).max())
        print(f"\nMEASURED wave2_vs_layer.{k} {d:.3e}")
        assert d < 2e-2, (k, d)
    d = float(np.abs(b["emb"] - a["emb"]).max())
    print(f"\nMEASURED wave2_vs_layer.emb {d:.3e}")
    assert d < 5e-3, d
    np.testing.assert_allclose(b["loss"], a["loss"], rtol=1e-3)


@pytest.mark.parametrize("N,M,T", [(8, 10, 20),    # c4's per-rank shape: 3 x 24 x 3 = 216 workgroups
                                   (7, 5, 9)])     # ragged rows (B = 35: padded dG^T columns)
def test_wavefront_bwd_bf16_against_per_layer(tmp_path, N, M, T):
    """Layer-wavefront backward (lstm_wave_bwd_bf16_kernel: all layers' recurrences and dx in one
    launch) vs the per-layer schedule (one persistent launch + dx GEMM per layer).  The layers'
    dh_rec sums are ordered alike; dx is summed per gate then across gates (the GEMM: over K in
    k-tile order), so the lower layers see fp32-reordered upstream gradients that bf16 rounding of
    dG can amplify to a few bf16 ulps: agreement at bf16-operand level."""
    dims = (40, 768, 3, 256)
    a = _run(tmp_path, "layer", {"SV_WAVE_BWD": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "wave", {"SV_WAVE_BWD": "1"}, dims, N, M, T, "bf16")
    assert int(a["status"][0]) == 0 and int(b["status"][0]) == 0
    np.testing.assert_array_equal(b["loss"], a["loss"])   # the forward is unchanged
    grads = [k for k in a if k.startswith("grad_")]
    assert len(grads) == 4 * dims[2] + 2
    worst = 0.0
    for k in grads:
        d = float(np.abs(b[k] - a[k]).max() / max(np.abs(a[k]).max(), 1e-30))
        worst = max(worst, d)
        print(f"\nMEASURED wave_bwd_vs_layer.{k} {d:.3e}")
        assert d < 2e-2, (k, d)
    print(f"\nMEASURED wave_bwd_vs_layer.worst {worst:.3e}")


@pytest.mark.parametrize("N,M,T", [(8, 10, 20), (7, 5, 9)])
def test_wave3_fwd_equals_wave2(tmp_path, N, M, T):
    """The LDS-DMA-staged wavefront forward (wave3) forms the same products in the same order as
    the register-staged one (wave2; its step-0 h-part adds exact zeros): bit-identical outputs."""
    dims = (40, 768, 3, 256)
    a = _run(tmp_path, "w2", {"SV_WAVE3": "0"}, dims, N, M, T, "bf16")
    b = _run(tmp_path, "w3", {"SV_WAVE3": "1"}, dims, N, M, T, "bf16")
    assert int(a["status"][0]) == 0 and int(b["status"][0]) == 0
    for k in a:
        if k != "status":
            np.testing.assert_array_equal(b[k], a[k], err_msg=k)
