"""Host logic of the bf16 row chunks (trainer.bf16_row_chunks) against the residency rules of the
library, without a GPU: the C-ABI residency checks (sv_persist_fwd_ok / sv_persist_bwd_ok /
sv_wave_ok) are replaced by their MI355X answers at H = 768 on 256 CUs (include/sv_ge2e.h):
the persistent grid takes up to 672 rows (21 row blocks of 32 x 12 unit blocks), the one-launch
layer wavefront up to 96 rows (3 layers x 24 unit blocks x 3 row blocks of 32)."""
import pytest

from pytorch_speaker_verification_amd import _lib
from pytorch_speaker_verification_amd.trainer import bf16_row_chunks


class _FakeLib:
    def sv_persist_fwd_ok(self, B, H):
        return int(H == 768 and 0 < B and (B + 31) // 32 * 12 <= 256)

    def sv_persist_bwd_ok(self, B, H):
        return self.sv_persist_fwd_ok(B, H)

    def sv_wave_ok(self, L, T, B, F, H):
        return int(L == 3 and F == 40 and H == 768 and 0 < B and 3 * 24 * ((B + 31) // 32) <= 256)


@pytest.fixture
def fake_lib(monkeypatch):
    fake = _FakeLib()
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    return fake


def _covers(chunks, B):
    assert chunks[0][0] == 0 and chunks[-1][1] == B
    assert all(a < b for a, b in chunks)
    assert all(chunks[i][1] == chunks[i + 1][0] for i in range(len(chunks) - 1))


@pytest.mark.parametrize("B, expect", [
    (80, [(0, 80)]),                          # c4 at 8 GPUs: one wavefront launch
    (96, [(0, 96)]),
    (160, [(0, 80), (80, 160)]),              # c4 at 4 GPUs: two wavefront halves
    (192, [(0, 96), (96, 192)]),
    (320, [(0, 320)]),                        # c4 at 2 GPUs / c5 at 8: the persistent grid whole
    (640, [(0, 640)]),                        # c3
    (672, [(0, 672)]),
    (1280, [(0, 640), (640, 1280)]),          # c5 at 2 GPUs: two persistent chunks
    (2560, [(0, 640), (640, 1280), (1280, 1920), (1920, 2560)]),  # c5 on one GPU
    (700, [(0, 350), (350, 700)]),            # ragged
])
def test_bf16_row_chunks_rules(fake_lib, B, expect):
    got = bf16_row_chunks(B, 768)
    assert got == expect
    _covers(got, B)
    for a, b in got:  # every chunk fits one of the two co-resident schedules
        assert fake_lib.sv_wave_ok(3, 160, b - a, 40, 768) or fake_lib.sv_persist_fwd_ok(b - a, 768)


def test_bf16_row_chunks_only_under_auto(fake_lib):
    for sched in ("per_step", "per_layer", "persist"):
        assert bf16_row_chunks(1280, 768, sched) == [(0, 1280)]
    assert bf16_row_chunks(0, 768) == [(0, 0)]


def test_bf16_row_chunks_other_dims_take_no_wavefront(fake_lib):
    # F != 40 (or L != 3): no wavefront; 160 rows fit the persistent grid whole
    assert bf16_row_chunks(160, 768, F=64) == [(0, 160)]
    assert bf16_row_chunks(160, 768, L=2) == [(0, 160)]
