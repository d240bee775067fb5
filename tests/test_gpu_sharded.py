"""Speaker-sharded GE2E on the GPU without torch.distributed (SURVEY §8e, config c5's path).

ShardedGE2E (sharded_ge2e.py) runs the GE2E kernels per rank around two exchanges: an
all-gather of the per-speaker sums and a SUM all-reduce of the [dC^ | beta] buffer.  Here the
ranks are virtual: one process runs every shard's kernels on its own slice of the speakers with
the shard's speaker offset s0 > 0, and the exchanges are done by hand (concatenation of the
sums, a plain sum of the reduce buffers).  So the per-shard arithmetic that c4 and c5 run on 8
GPUs (global N = 64 and 256: the fused sv_ge2e_shard_prep / _rows / _finalize) and the split
kernels (sv_ge2e_fwd_rows / bwd_rows / bwd_finalize, any N) are checked against
the reference's golden vectors (tests/golden/ge2e_n256m10.npz, ge2e_n64m10.npz; reference math
utils.py:72-132) and the numpy oracle.  Tolerances: loss 1e-4 relative (north_star), dE 1e-4 of
its largest entry, dw 1e-4, db 1e-5 per row."""
import numpy as np
import pytest
import torch

import recipe
from conftest import golden
from oracle import ge2e_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(tag):
    g = golden(f"ge2e_{tag}.npz")
    E = recipe.make_embeddings(int(g["seed"]), int(g["n"]), int(g["m"]), int(g["d"]), bool(g["clustered"]))
    return g, E, float(g["w"]), float(g["b"])


def _check(tag, g, E, w, b, loss, per, dE, dw, db, label):
    ref_loss = float(g["loss"])
    o_dE, o_dw, o_db = ge2e_np.ge2e_backward(E, w, b)
    scale = float(np.abs(o_dE).max())
    d_loss = abs(loss - ref_loss) / abs(ref_loss)
    d_dE = float(np.abs(dE - o_dE).max()) / scale
    print(f"\nMEASURED {label}.{tag} loss_rel {d_loss:.2e} dE_rel {d_dE:.2e} dw {abs(dw - o_dw):.2e} "
          f"db {abs(db - o_db):.2e}")
    assert d_loss <= 1e-4, (loss, ref_loss)
    np.testing.assert_allclose(per, g["per"], atol=1e-4)
    assert d_dE <= 1e-4
    if "dE" in g.files:  # the reference's own dE
        np.testing.assert_allclose(dE, g["dE"], atol=1e-4 * scale)
    else:               # the reference's first speakers and the norm of the whole dE
        np.testing.assert_allclose(dE[:g["dE_head"].shape[0]], g["dE_head"], atol=1e-4 * scale)
        assert abs(float(np.linalg.norm(dE)) - float(g["dE_norm"])) <= 1e-4 * float(g["dE_norm"])
    assert abs(dw - float(g["dw"])) <= 1e-4 * max(1.0, abs(float(g["dw"])))
    assert abs(db - float(g["db"])) <= 1e-5 * E.shape[0] * E.shape[1]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_split_shard_kernels_n256(world):
    """c5's GE2E at N = 256 x M = 10 split over `world` virtual ranks on the split kernels
    (HipShardKernels, every shard but the first with s0 > 0), as ShardedGE2E.forward/backward run
    them: sums -> (all-gather) -> rows -> bwd rows -> (SUM all-reduce of [dC^|beta]) -> finalize."""
    from pytorch_speaker_verification_amd.sharded_ge2e import HipShardKernels
    g, E, w, b = _inputs("n256m10")
    N, M, D = E.shape
    Nl = N // world
    k = HipShardKernels()
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    shards = [Et[r * Nl:(r + 1) * Nl].contiguous() for r in range(world)]
    ssum_all = torch.cat([k.speaker_sums(s) for s in shards])
    fwd = [k.fwd_rows(shards[r], r * Nl, N, ssum_all, wt, bt) for r in range(world)]
    loss = sum(float(f[0]) for f in fwd)
    per = np.concatenate([f[1].cpu().numpy() for f in fwd])
    bwd = [k.bwd_rows(f[2], wt, bt, None) for f in fwd]
    red = torch.stack([r_[0] for r_ in bwd]).sum(0)
    dE = torch.cat([k.finalize(f[2], red.clone()) for f in fwd]).cpu().numpy()
    dw = sum(float(r_[1][0]) for r_ in bwd)
    db = sum(float(r_[1][1]) for r_ in bwd)
    _check("n256m10", g, E, w, b, loss, per, dE, dw, db, f"ge2e_split_shards{world}")


@pytest.mark.parametrize("tag,world", [("n64m10", 2), ("n64m10", 4), ("n64m10", 8),
                                       ("n256m10", 2), ("n256m10", 4), ("n256m10", 8)])
def test_fused_shard_kernels(tag, world):
    """The fused sharded form (HipFusedShard: sv_ge2e_shard_prep / _rows / _finalize) that
    ShardedGE2E.train takes for global N <= 256: c4 (N = 64 over 8 GPUs, 8 speakers per rank) and
    c5 (N = 256: 32 speakers per rank at 8 GPUs, s0 up to 224; the centroids in two LDS tiles)."""
    from pytorch_speaker_verification_amd.sharded_ge2e import HipFusedShard
    g, E, w, b = _inputs(tag)
    N, M, D = E.shape
    Nl = N // world
    assert HipFusedShard.ok(N, M, D)
    f = HipFusedShard()
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    shards = [Et[r * Nl:(r + 1) * Nl].contiguous() for r in range(world)]
    prep = [f.prep(s, N) for s in shards]
    ssum_all = torch.cat([p[0] for p in prep])
    rows = [f.rows(shards[r], r * Nl, N, ssum_all, wt, bt, prep[r][1]) for r in range(world)]
    loss = sum(float(r_[0]) for r_ in rows)
    per = np.concatenate([r_[1].cpu().numpy() for r_ in rows])
    red = torch.stack([r_[2] for r_ in rows]).sum(0)
    dE = torch.cat([f.finalize(shards[r], r * Nl, N, red.clone(), prep[r][1]) for r in range(world)]).cpu().numpy()
    dw = sum(float(r_[3][0]) for r_ in rows)
    db = sum(float(r_[3][1]) for r_ in rows)
    _check(tag, g, E, w, b, loss, per, dE, dw, db, f"ge2e_fused_shards{world}")


@pytest.mark.parametrize("N,M,D,world", [(160, 4, 64, 2), (160, 4, 64, 5), (200, 3, 100, 4)])
def test_fused_shard_kernels_wide_n_other_d(N, M, D, world):
    """The fused sharded form at 128 < N <= 256 with D != 256 (the two-tile rows kernel, every
    shard after the first with s0 > 0) against the fp64 numpy oracle."""
    from pytorch_speaker_verification_amd.sharded_ge2e import HipFusedShard
    E = recipe.make_embeddings(N * 17 + D, N, M, D, True)
    w, b = 7.0, -3.0
    Nl = N // world
    assert HipFusedShard.ok(N, M, D)
    f = HipFusedShard()
    Et = torch.tensor(E, device=DEV)
    wt = torch.tensor(w, dtype=torch.float32, device=DEV)
    bt = torch.tensor(b, dtype=torch.float32, device=DEV)
    shards = [Et[r * Nl:(r + 1) * Nl].contiguous() for r in range(world)]
    prep = [f.prep(s, N) for s in shards]
    ssum_all = torch.cat([p[0] for p in prep])
    rows = [f.rows(shards[r], r * Nl, N, ssum_all, wt, bt, prep[r][1]) for r in range(world)]
    loss = sum(float(r_[0]) for r_ in rows)
    per = np.concatenate([r_[1].cpu().numpy() for r_ in rows])
    red = torch.stack([r_[2] for r_ in rows]).sum(0)
    dE = torch.cat([f.finalize(shards[r], r * Nl, N, red.clone(), prep[r][1]) for r in range(world)]).cpu().numpy()
    dw = sum(float(r_[3][0]) for r_ in rows)
    db = sum(float(r_[3][1]) for r_ in rows)
    o_loss, o_per = ge2e_np.ge2e_forward(E, w, b)[:2]
    o_dE, o_dw, o_db = ge2e_np.ge2e_backward(E, w, b)
    scale = float(np.abs(o_dE).max())
    d_loss = abs(loss - float(o_loss)) / abs(float(o_loss))
    d_dE = float(np.abs(dE - o_dE).max()) / scale
    print(f"\nMEASURED ge2e_fused_shards{world}_wide.N{N}M{M}D{D} loss_rel {d_loss:.2e} dE_rel {d_dE:.2e}")
    assert d_loss <= 1e-4
    np.testing.assert_allclose(per, o_per, atol=1e-4)
    assert d_dE <= 1e-4
    assert abs(dw - o_dw) <= 1e-4 * max(1.0, abs(o_dw))
    assert abs(db - o_db) <= 1e-5 * N * M
