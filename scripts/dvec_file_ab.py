"""Per-file d-vector call (dvector_create.py:96-101: one file's windows per call), bf16, T = 24:
the persistent per-layer forward on all S windows vs the one-launch layer wavefront on row chunks
that fit it (trainer.bf16_row_chunks).  Prints ms per call for S in a few file sizes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorch_speaker_verification_amd.dvector import embed_windows  # noqa: E402
from pytorch_speaker_verification_amd.ops import embedder_forward_bf16, check_persistent_status  # noqa: E402
from pytorch_speaker_verification_amd.trainer import bf16_row_chunks  # noqa: E402

dev = torch.device("cuda", 0)
net, _ = bench.build_model(bench.DIMS, dev)
layers = net.LSTM_stack.layer_params()


@torch.no_grad()
def chunked(xw):
    x = torch.as_tensor(xw, dtype=torch.float32).to(dev)
    ch = bf16_row_chunks(x.shape[0], 768, "auto", 3, x.shape[1], x.shape[2])
    out = [embedder_forward_bf16(x[a:b].contiguous(), layers, net.projection.weight, net.projection.bias,
                                 save=False)[0] for a, b in ch]
    check_persistent_status(wait=True)
    return torch.cat(out), ch


for S in (64, 96, 128, 160, 192, 256):
    xw = torch.randn(S, 24, 40).numpy()
    ref = embed_windows(net, xw, precision="bf16")
    got, ch = chunked(xw)
    ms_p = bench._timed(lambda: embed_windows(net, xw, precision="bf16"), dev, 20)
    ms_c = bench._timed(lambda: chunked(xw), dev, 20)
    print(json.dumps({"S": S, "chunks": ch, "persist_ms": round(ms_p, 3), "chunked_ms": round(ms_c, 3),
                      "max_abs_diff": float((ref - got).abs().max())}), flush=True)
