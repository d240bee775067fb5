"""Per-parameter gradient deviation of the bf16 schedules (per_step / persist) from the bf16
oracle on the GPU at c3 dims and a few T (debug aid for tests/test_gpu_persist.py)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import recipe  # noqa: E402
import schedules  # noqa: E402
from oracle import lstm_bf16  # noqa: E402

dims, N, M = (40, 768, 3, 256), 64, 10
for T in [int(v) for v in (sys.argv[1:] or ["32", "33", "40"])]:
    a = schedules.run(dims, N, M, T, "bf16", "per_step")
    b = schedules.run(dims, N, M, T, "bf16", "persist")
    sd = recipe.make_weights(7, *dims, scale=3.0)
    x = recipe.make_frames(11, N * M, T, dims[0])
    r = lstm_bf16.train_step(sd, 10.0, -5.0, x, N, M, dims[2], bf16=True, device="cuda")
    rg = {k: v.detach().cpu().numpy() for k, v in r[5].items()}
    tot = float(np.sqrt(sum(float((v.astype(np.float64) ** 2).sum()) for v in rg.values())))
    coef = min(1.0, 3.0 / (tot + 1e-6))
    print(f"T={T} loss step {a['loss'][0]:.6f} persist {b['loss'][0]:.6f} oracle {r[0]:.6f}")
    for k in rg:
        ref = coef * rg[k]
        s = max(np.abs(ref).max(), 1e-30)
        da = np.abs(a["grad_" + k] - ref).max() / s
        db = np.abs(b["grad_" + k] - ref).max() / s
        dd = np.abs(a["grad_" + k] - b["grad_" + k]).max() / s
        print(f"  {k:30s} step-oracle {da:.2e} persist-oracle {db:.2e} step-persist {dd:.2e}")
