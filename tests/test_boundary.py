"""Host-side boundary checks (no GPU): config surface, C-ABI exports, module surface."""
import json
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, golden, model_dims


def test_hparam_matches_reference_config():
    from pytorch_speaker_verification_amd.hparam import Hparam
    ref = json.load(open(os.path.join(GOLDEN, "hparam.json")))
    hp = Hparam(os.path.join(ROOT, "pytorch_speaker_verification_amd", "config", "config.yaml"))
    assert json.loads(json.dumps(hp)) == ref
    assert hp.train.N == 4 and hp.model.hidden == 768 and hp.data.nmels == 40


def test_hparam_cwd_config(tmp_path, monkeypatch):
    (tmp_path / "config").mkdir()
    (tmp_path / "config" / "config.yaml").write_text("training: false\n---\nmodel:\n  hidden: 12\n")
    monkeypatch.chdir(tmp_path)
    from pytorch_speaker_verification_amd.hparam import Hparam
    hp = Hparam()
    assert hp.training is False and hp.model.hidden == 12


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "sv_ge2e.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sv_\w+)\s*\(", src)))


def test_c_abi_library_exports_every_header_symbol():
    from pytorch_speaker_verification_amd import _lib
    h = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(h, s), s
        assert s in _lib.SIGNATURES, f"{s} missing from the ctypes signature table"
    assert h.sv_abi_version() == _lib.ABI_VERSION == 11
    assert not hasattr(h, "sv_test_set_fault")  # the fault injector exists only in the test build
    # workspace queries are host-only and callable without a GPU
    assert h.sv_ge2e_workspace_size(64, 10, 256, 64) > 0
    assert h.sv_lstm_layer_bwd_workspace(160, 640, 768, 768) > 0
    ws = h.sv_gemm_f32_workspace(3072, 768, 102400)  # split-K slabs
    assert ws > 0 and ws % (3072 * 768 * 4) == 0


def test_dtype_enum_entry_points_dispatch():
    """SURVEY §8 b's dtype argument: sv_lstm_fwd / sv_lstm_bwd forward to the fp32 or bf16 stack
    functions (ops.py calls only these); host-side checks, no launch: the workspace query of each
    dtype is the dtype-specific one, and an unknown dtype is an argument error before any work."""
    from pytorch_speaker_verification_amd import _lib
    h = _lib.lib()
    for dims in ((3, 160, 640, 40, 768), (3, 24, 32, 40, 64)):
        assert h.sv_lstm_bwd_workspace(_lib.SV_DTYPE_F32, *dims) == h.sv_lstm_stack_bwd_workspace(*dims)
        assert h.sv_lstm_bwd_workspace(_lib.SV_DTYPE_BF16, *dims) == h.sv_lstm_stack_bwd_bf16_workspace(*dims)
        assert h.sv_lstm_bwd_workspace(2, *dims) == 0
    nul = [None] * 10
    assert h.sv_lstm_fwd(2, 3, 4, 8, 40, 64, *nul, 0, None, None, None, 0, 0, None, None) == -1  # SV_EARG
    assert h.sv_lstm_bwd(-1, 3, 4, 8, 40, 64, *([None] * 16), 0, None, None, None, 0, None, None, 0, None) == -1


def test_library_binds_torch_hip_runtime():
    from pytorch_speaker_verification_amd import _lib
    _lib.lib()
    maps = open("/proc/self/maps").read()
    hips = sorted(set(re.findall(r"\S*libamdhip64\S*", maps)))
    assert len(hips) == 1, hips


def test_state_dict_keys_and_init_rng_parity():
    """Same names/shapes/order as the reference; same init under the same torch seed
    (nn.LSTM uniform init, then xavier_normal_/0, then Linear -- speech_embedder_net.py:17-25)."""
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    ref = golden("init_seed1234.npz")
    with model_dims(40, 64, 3, 32):
        torch.manual_seed(1234)
        net = SpeechEmbedder()
    sd = net.state_dict()
    assert list(sd.keys()) == list(ref.files)
    for k in ref.files:
        np.testing.assert_array_equal(sd[k].numpy(), ref[k])


def test_full_size_parameter_count():
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    net = SpeechEmbedder()
    assert sum(p.numel() for p in net.parameters()) == 12134656


def test_ge2e_loss_module_surface():
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss
    m = GE2ELoss("cpu")
    ps = list(m.parameters())
    assert len(ps) == 2 and ps[0].dim() == 0 and float(ps[0]) == 10.0 and float(ps[1]) == -5.0


def test_ops_refuse_cpu_tensors():
    """No CPU fallback: the product path raises on host tensors."""
    import pytest
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    with model_dims(40, 16, 1, 8):
        net = SpeechEmbedder()
    with pytest.raises(RuntimeError, match="GPU only"):
        net(torch.zeros(4, 3, 40))
    with pytest.raises(RuntimeError, match="GPU only"):
        GE2ELoss("cpu")(torch.randn(2, 2, 8))


def test_shipped_library_reads_no_environment():
    """Modes are explicit arguments (include/sv_ge2e.h): no getenv in the product sources, so
    nothing outside a call's arguments changes what it computes."""
    import glob
    for f in glob.glob(os.path.join(ROOT, "pytorch_speaker_verification_amd", "csrc", "*")):
        assert "getenv" not in open(f).read(), f


def test_fault_injection_build_exports_the_test_hook():
    import ctypes
    from pytorch_speaker_verification_amd import _lib
    h = ctypes.CDLL(_lib.FAULT_LIB_PATH)
    assert hasattr(h, "sv_test_set_fault") and h.sv_abi_version() == _lib.ABI_VERSION


def test_graft_build_entry_point():
    """__graft_entry__.build(): the driver's build check (make + import + the library's ABI equal to
    the binding's; a stale ABI assertion there once failed every build)."""
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    importlib.import_module("__graft_entry__").build()


@pytest.mark.gpu
def test_graft_smoke_entry_point():
    """__graft_entry__.smoke(): one small training step on cuda:0 against the numpy oracle."""
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    importlib.import_module("__graft_entry__").smoke()
