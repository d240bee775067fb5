"""Runs the bf16 stack forward + one training step under a given bf16 schedule (the `schedule`
argument of the C ABI, include/sv_ge2e.h SV_SCHED_*) in this process and returns every output
as numpy arrays (tests/test_gpu_persist.py compares schedules with it)."""
import numpy as np
import torch

import recipe
from conftest import model_dims


def run(dims, N, M, T, precision="bf16", schedule="auto", seed_w=7, seed_x=11):
    from pytorch_speaker_verification_amd._lib import PersistStatus
    from pytorch_speaker_verification_amd.ops import embedder_forward, embedder_forward_bf16
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    dev = torch.device("cuda", 0)
    with model_dims(*dims):
        net = SpeechEmbedder()
    sd = recipe.make_weights(seed_w, *dims, scale=3.0)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to(dev)
    net.precision = precision
    net.schedule = schedule
    x = torch.tensor(recipe.make_frames(seed_x, N * M, T, dims[0]), device=dev)
    layers = net.LSTM_stack.layer_params()
    status = PersistStatus(dev)
    if precision == "bf16":
        emb, st = embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, status=status,
                                        schedule=schedule)
    else:
        emb, st = embedder_forward(x, layers, net.projection.weight, net.projection.bias)
    res = {"emb": emb, "h_last": st.h_last}
    for l in range(len(layers)):
        res[f"gates{l}"] = st.gates[l]
        res[f"c{l}"] = st.c_tm[l]
    tr = GE2ETrainer(net, GE2ELoss(dev), lr=0.01)
    res["loss"] = tr.step(x, N, M).reshape(1)
    res["flat_p"] = tr.flat_p
    res["flat_g"] = tr.flat_g
    for name, prm in net.named_parameters():
        res["grad_" + name] = prm.grad
    torch.cuda.synchronize()
    out = {k: v.detach().float().cpu().numpy() for k, v in res.items()}
    out["status"] = np.array([int(status.block[0]) | int(tr.status.block[0])])
    del res, st, emb, tr, net
    torch.cuda.empty_cache()
    return out
