"""The RCCL code paths on hardware.  The GPU box has one GPU and RCCL needs one GPU per rank, so
the data-parallel tests (test_gpu_dp.py) run gloo; here a WORLD-1 `nccl` process group drives the
same code through RCCL itself:

* the fused sharded GE2E exchange -- `all_gather_rows` (all_gather_into_tensor under nccl) of the
  speaker sums, then the SUM all-reduce of (dC^, beta) -- against the single-GPU fused kernels;
* the trainer's data-parallel machinery switched on at world 1 (`GE2ETrainer.dp`): the comm
  stream, the per-layer buckets all-reduced from the backward's completion events, the status
  flags and the loss word riding the head bucket.  A SUM over one rank is the identity, so the
  step must equal the plain trainer's bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import recipe
from conftest import model_dims

pytestmark = pytest.mark.gpu
DIMS = (40, 64, 2, 32)


def _model(dev):
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    with model_dims(*DIMS):
        net = SpeechEmbedder()
    sd = recipe.make_weights(7, *DIMS, scale=3.0)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    return net.to(dev), GE2ELoss(dev)


def _steps(precision, dp, x, N, M, steps=2):
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    net, ge2e = _model(x.device)
    net.precision = precision
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    if dp:
        tr.dp = True
    losses = [float(tr.step(x, N, M)) for _ in range(steps)]
    tr.check()
    return losses, {k: v.cpu().numpy() for k, v in net.state_dict().items()}, [ge2e.w.item(), ge2e.b.item()]


def _worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {"backend": dist.get_backend()}
    try:
        from pytorch_speaker_verification_amd.ops import ge2e_train
        from pytorch_speaker_verification_amd.sharded_ge2e import HipFusedShard, all_gather_rows
        g = torch.Generator().manual_seed(3)
        for N, M in ((64, 10), (256, 10)):
            E = torch.randn(N, M, 256, generator=g).to(dev)
            w = torch.tensor(10.0, device=dev)
            b = torch.tensor(-5.0, device=dev)
            f = HipFusedShard()
            ssum, ws = f.prep(E, N)
            ssum_all = all_gather_rows(ssum, 0, 1)
            loss, _, red, dwdb = f.rows(E, 0, N, ssum_all, w, b, ws)
            dist.all_reduce(red)
            dE = f.finalize(E, 0, N, red, ws)
            loss_r, _, dE_r, dwdb_r = ge2e_train(E, w, b)
            torch.cuda.synchronize()
            out[f"ge2e_N{N}"] = (float(loss), float(loss_r), float((dE - dE_r).abs().max()),
                                 float(dE_r.abs().max()), dwdb.cpu().numpy(), dwdb_r.cpu().numpy(),
                                 bool(torch.equal(ssum_all, ssum)))
        NL, M, T = 6, 4, 12
        x = torch.tensor(recipe.make_frames(5, NL * M, T, DIMS[0]), device=dev)
        for precision in ("f32", "bf16"):
            out[f"trainer_{precision}"] = (_steps(precision, False, x, NL, M), _steps(precision, True, x, NL, M))
        q.put(out)
    except Exception as e:  # noqa: BLE001 -- reported by the parent
        q.put({"error": repr(e)})
    finally:
        dist.destroy_process_group()


def test_rccl_world1_exchanges_and_dp_trainer():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(port, q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert "error" not in out, out.get("error")
    assert out["backend"] == "nccl"
    for N in (64, 256):
        loss, loss_r, dmax, dref, dwdb, dwdb_r, gathered = out[f"ge2e_N{N}"]
        print(f"\nMEASURED rccl_world1.fused_shard_vs_fused.N{N} loss rel {abs(loss / loss_r - 1):.2e} "
              f"dE rel {dmax / dref:.2e}")
        assert gathered  # all_gather_into_tensor over one rank copies the sums exactly
        assert abs(loss / loss_r - 1) < 1e-5
        assert dmax <= 1e-5 * dref
        np.testing.assert_allclose(dwdb, dwdb_r, rtol=1e-5, atol=1e-6)
    for precision in ("f32", "bf16"):
        (l0, sd0, wb0), (l1, sd1, wb1) = out[f"trainer_{precision}"]
        print(f"MEASURED rccl_world1.dp_trainer.{precision} losses {l1} (plain {l0})")
        assert l1 == l0, (l1, l0)
        for k in sd0:
            assert np.array_equal(sd0[k], sd1[k]), k
        assert wb0 == wb1
