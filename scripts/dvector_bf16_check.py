import sys, os, json, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
from pytorch_speaker_verification_amd.dvector import embed_windows
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
g = torch.Generator().manual_seed(24)
for S in (3000, 16384):
    xw = torch.randn(S, 24, 40, generator=g).to(dev)
    e32 = embed_windows(net, xw, batch=S)
    e16 = embed_windows(net, xw, batch=S, precision="bf16")
    torch.cuda.synchronize()
    dev_max = float((e16 - e32).abs().max())
    cos = float((e16 * e32).sum(1).min())
    out = {"S": S, "bf16_vs_f32_maxabs": dev_max, "min_cos": cos}
    for prec in ("f32", "bf16"):
        ms = bench._timed(lambda: embed_windows(net, xw, batch=S, precision=prec), dev, 3)
        out[prec + "_ms"] = round(ms, 3)
        out[prec + "_wps"] = round(S / ms * 1e3, 1)
    print(json.dumps(out), flush=True)
