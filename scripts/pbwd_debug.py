"""Debug aid: run the bf16 stack backward under the schedule in the environment and save
dG (row-major + transposed), dx and the weight gradients per layer.  Usage:
  python scripts/pbwd_debug.py out.npz   (then compare two runs with --cmp a.npz b.npz)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(out):
    import torch
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd._lib import PersistStatus
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims, N, M, T = (40, 768, 3, 256), 64, 10, 12
    dev = torch.device("cuda", 0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    sd = recipe.make_weights(7, *dims, scale=3.0)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    x = torch.tensor(recipe.make_frames(11, N * M, T, dims[0]), device=dev)
    layers = net.LSTM_stack.layer_params()
    ps = PersistStatus(dev)
    emb, st = ops.embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, status=ps)
    torch.manual_seed(3)
    demb = torch.randn_like(emb)
    cap = []
    orig = ops._bf

    def spy(shape, d):
        t = orig(shape, d)
        cap.append(t)
        return t
    ops._bf = spy
    grads = ops.embedder_backward_bf16(st, demb, layers, net.projection.weight, status=ps)
    torch.cuda.synchronize()
    res = {f"buf{i}": c.float().cpu().numpy() for i, c in enumerate(cap)}
    for i, g in enumerate(grads):
        res[f"g{i}"] = g.float().cpu().numpy()
    res["status"] = np.array([int(ps.block[0])])
    np.savez(out, **res)


def cmp(a, b):
    a, b = np.load(a), np.load(b)
    for k in a.files:
        x, y = a[k], b[k]
        if x.shape != y.shape:
            print(k, "shape", x.shape, y.shape)
            continue
        d = np.abs(x - y)
        if d.max() == 0:
            print(k, x.shape, "equal")
            continue
        idx = np.unravel_index(np.argmax(d), d.shape)
        first = np.argwhere(d > 0)[0]
        if x.ndim == 3:
            print("  per-t ndiff", [int((d[t] > 0).sum()) for t in range(x.shape[0])])
        print(k, x.shape, "maxdiff", d.max(), "at", idx, "ndiff", int((d > 0).sum()), "first", first,
              "vals", x[tuple(first)], y[tuple(first)])


if __name__ == "__main__":
    if sys.argv[1] == "--cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
