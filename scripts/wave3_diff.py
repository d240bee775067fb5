"""Diagnostics: run tests/_schedule_worker.py under two env settings and print per-key max
differences (and the differing rows of 2-D/3-D outputs).  Usage: python scripts/wave3_diff.py
'A=1,B=2' 'A=0'"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
W = os.path.join(HERE, "..", "tests", "_schedule_worker.py")


def run(envs, out):
    env = dict(os.environ)
    for kv in envs.split(","):
        if kv:
            k, v = kv.split("=")
            env[k] = v
    r = subprocess.run([sys.executable, W, out, "40,768,3,256", "8", "10", "20", "bf16"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(np.load(out))


d = tempfile.mkdtemp()
a = run(sys.argv[1], os.path.join(d, "a.npz"))
b = run(sys.argv[2], os.path.join(d, "b.npz"))
for k in a:
    x, y = a[k].astype(np.float64), b[k].astype(np.float64)
    diff = np.abs(x - y)
    msg = f"{k} shape {a[k].shape} maxdiff {diff.max():.3e}"
    if diff.max() > 0 and x.ndim >= 2:
        red = diff.reshape(-1, x.shape[-1]).max(1) if x.ndim == 2 else diff.max(-1)
        idx = np.argwhere(red > 0)
        msg += f" n_bad {len(idx)} first {idx[:8].tolist()}"
    print(msg, flush=True)
