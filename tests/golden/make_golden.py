#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the build container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box).  The reference is imported
in-process, read-only, with the two shims SURVEY.md §8c lists:

  1. ``yaml.load_all`` gets an explicit SafeLoader (``hparam.py:9`` omits it and
     PyYAML >= 6 raises);
  2. ``librosa`` is stubbed (only used by preprocessing, ``utils.py:8,138-164``).

What is recorded (inputs + expected outputs; no reference source is copied):
  kat0.npz            -- the reference's own ``utils.py:166-173`` example (KAT-0).
  ge2e_*.npz          -- GE2E loss / per-embedding loss / dE / dw / db for seeded E.
  cossim_ext.npz      -- get_cossim with external (enrollment) centroids, the
                         ``train_speech_embedder.py:127-129`` call shape.
  net_small.npz       -- full training step (fwd, GE2E, bwd, clip 3.0/1.0, SGD) of the
                         reference SpeechEmbedder at small dims, 3 steps.
  net_full_c1.npz     -- one step at the full dims (40->768x3->256), N=4 x M=5, T=160.
  net_full_c2.npz     -- one step at the headline config c2 (N=64 x M=10, T=160, full dims).
  net_fwd_c5.npz      -- forward + loss at c5's global batch (N=256 x M=10, T=180, full dims).
  net_full_c5.npz     -- one training step at c5's global batch (forward, GE2E, backward, clip,
                         SGD): gradient norms and 8x8 heads, update norms (≈5 min of CPU).
  hparam.json         -- the parsed config/config.yaml as the reference sees it.

Weights/inputs come from tests/golden/recipe.py (numpy PCG64), so fixtures hold the
recipe parameters, not the weights.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import recipe  # noqa: E402


def import_reference():
    import yaml
    orig = yaml.load_all
    yaml.load_all = lambda s, Loader=yaml.SafeLoader: orig(s, Loader=Loader)
    sys.modules.setdefault("librosa", types.ModuleType("librosa"))
    sys.dont_write_bytecode = True
    cwd = os.getcwd()
    os.chdir(REF)
    sys.path.insert(0, REF)
    try:
        import hparam as ref_hparam  # noqa: F401
        import utils as ref_utils
        import speech_embedder_net as ref_net
    finally:
        os.chdir(cwd)
    return ref_hparam, ref_utils, ref_net


def ge2e_case(ref_utils, ref_net, E_np, w, b):
    import torch
    E = torch.tensor(E_np, requires_grad=True)
    loss_mod = ref_net.GE2ELoss("cpu")
    with torch.no_grad():
        loss_mod.w.fill_(w)
        loss_mod.b.fill_(b)
    loss = loss_mod(E)
    loss.backward()
    with torch.no_grad():
        C = ref_utils.get_centroids(E)
        cos = ref_utils.get_cossim(E, C)
        _, per = ref_utils.calc_loss(loss_mod.w * cos + loss_mod.b)
    return dict(loss=np.float64(loss.item()), per=per.numpy(), cossim=cos.numpy(),
                centroids=C.numpy(), dE=E.grad.numpy(),
                dw=np.float64(loss_mod.w.grad.item()), db=np.float64(loss_mod.b.grad.item()))


def train_steps(ref_net, ref_hparam, dims, wseed, wscale, xseed, N, M, T, steps, lr=0.01):
    """Run the reference train() step body (train_speech_embedder.py:44-65) `steps` times
    on fixed recipe input (the random perm/unperm is a no-op on values: rows are
    independent, SURVEY §8 a-J)."""
    import torch
    hp = ref_hparam.hparam
    old = (hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj)
    hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = dims
    try:
        net = ref_net.SpeechEmbedder()
    finally:
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = old
    sd = recipe.make_weights(wseed, *dims, scale=wscale)
    net.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    ge2e = ref_net.GE2ELoss("cpu")
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": ge2e.parameters()}], lr=lr)
    x = torch.tensor(recipe.make_frames(xseed, N * M, T, dims[0]))
    rec = {"losses": [], "per": [], "emb": []}
    for s in range(steps):
        opt.zero_grad()
        emb = net(x)
        emb = emb.reshape(N, M, emb.size(1))
        loss = ge2e(emb)
        loss.backward()
        if s == 0:
            rec["grads"] = {k: p.grad.detach().numpy().copy() for k, p in net.named_parameters()}
            rec["dw0"] = ge2e.w.grad.item()
            rec["db0"] = ge2e.b.grad.item()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 3.0)
        torch.nn.utils.clip_grad_norm_(ge2e.parameters(), 1.0)
        opt.step()
        rec["losses"].append(loss.item())
        rec["emb"].append(emb.detach().numpy().copy())
        if s == 0:
            rec["params1"] = {k: p.detach().numpy().copy() for k, p in net.named_parameters()}
            rec["wb1"] = (ge2e.w.item(), ge2e.b.item())
    rec["params_final"] = {k: p.detach().numpy().copy() for k, p in net.named_parameters()}
    rec["wb_final"] = (ge2e.w.item(), ge2e.b.item())
    return rec


def eer_and_loader_fixtures(ref_hparam, ref_net):
    import contextlib
    import io
    import random
    import tempfile
    import torch
    hp = ref_hparam.hparam
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        import data_load as ref_data
        import train_speech_embedder as ref_train
    finally:
        os.chdir(cwd)
    tmp = tempfile.mkdtemp(prefix="sv_golden_")
    recipe.make_speaker_dir(os.path.join(tmp, "test"), 12, 77)
    saved = {k: dict(v) for k, v in hp.items() if isinstance(v, dict)}
    saved_top = {k: v for k, v in hp.items() if not isinstance(v, dict)}
    try:
        hp.training = False
        hp.data.test_path = os.path.join(tmp, "test")
        hp.data.train_path = os.path.join(tmp, "test")
        hp.test.N, hp.test.M, hp.test.epochs, hp.test.num_workers = 4, 6, 2, 0
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = 40, 64, 3, 32
        # (1) the preprocessed dataset under fixed seeds: shuffle=True and shuffle=False items
        random.seed(123)
        np.random.seed(123)
        ds = ref_data.SpeakerDatasetTIMITPreprocessed()
        files = sorted(os.listdir(hp.data.test_path))
        items = [ds[i].numpy() for i in range(3)]
        ds2 = ref_data.SpeakerDatasetTIMITPreprocessed(shuffle=False, utter_start=1)
        items_ns = [ds2[i].numpy() for i in range(2)]
        np.savez_compressed(os.path.join(HERE, "loader.npz"), seed=123, M=6, n_spk=12, data_seed=77,
                            listdir=np.array(os.listdir(hp.data.test_path)), sorted_files=np.array(files),
                            items=np.stack(items), items_noshuffle=np.stack(items_ns))
        # (2) test(): EER on the synthetic test set with a recipe-weight checkpoint
        net = ref_net.SpeechEmbedder()
        sd = recipe.make_weights(41, 40, 64, 3, 32, scale=3.0)
        net.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
        ckpt = os.path.join(tmp, "model.model")
        torch.save(net.state_dict(), ckpt)
        sims = []
        orig = ref_train.get_cossim

        def rec(a, b):
            out = orig(a, b)
            sims.append(out.detach().numpy().copy())
            return out
        ref_train.get_cossim = rec
        random.seed(5)
        np.random.seed(5)
        torch.manual_seed(5)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            ref_train.test(ckpt)
        ref_train.get_cossim = orig
        lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("EER")]
        vals = np.array([[float(x) for x in
                          ln.replace("EER :", "").replace("(thres:", " ").replace("FAR:", " ").replace("FRR:", " ")
                          .replace(")", " ").replace(",", " ").split()] for ln in lines])
        avg = float(buf.getvalue().strip().splitlines()[-1].split(":")[-1])
        np.savez_compressed(os.path.join(HERE, "eer.npz"), sims=np.stack(sims), printed=vals, avg_eer=avg,
                            wseed=41, dims=np.array([40, 64, 3, 32]), data_seed=77, n_spk=12, N=4, M=6, epochs=2,
                            seed=5)
        torch.save(net.state_dict(), os.path.join(HERE, "ref_small_checkpoint.pth"))
        print("eer fixture: batches", len(sims), "avg", avg)
    finally:
        for k, v in saved.items():
            hp[k].update(v)
        for k, v in saved_top.items():
            hp[k] = v
        os.chdir(cwd)


def net_full_c2(ref_net, ref_hparam):
    """One training step at c2 (N=64 x M=10, T=160, full dims, fp32): the headline config pinned
    to the reference itself (≈13 s of CPU).  Whole-tensor gradient and update norms plus 8x8 heads;
    the embeddings in full (640 x 256)."""
    dims = (40, 768, 3, 256)
    rec = train_steps(ref_net, ref_hparam, dims, wseed=61, wscale=2.0, xseed=62, N=64, M=10, T=160, steps=1)
    sd0 = recipe.make_weights(61, *dims, scale=2.0)
    out = dict(dims=np.array(dims), wseed=61, wscale=2.0, xseed=62, N=64, M=10, T=160,
               loss=rec["losses"][0], emb=rec["emb"][0], dw0=rec["dw0"], db0=rec["db0"], wb1=np.array(rec["wb1"]))
    for k, g in rec["grads"].items():
        out["gnorm." + k] = np.linalg.norm(g.astype(np.float64))
        out["ghead." + k] = g.reshape(g.shape[0], -1)[:8, :8] if g.ndim == 2 else g[:64]
    for k, p in rec["params1"].items():
        out["p1head." + k] = p.reshape(p.shape[0], -1)[:8, :8] if p.ndim == 2 else p[:64]
        out["dpnorm." + k] = np.linalg.norm(p.astype(np.float64) - sd0[k].astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "net_full_c2.npz"), **out)
    print("net_full_c2 loss", rec["losses"][0])


def net_full_c5(ref_net, ref_hparam):
    """One training step at c5's global batch (N=256 x M=10, T=180, full dims, fp32): the backward
    at the largest config pinned to the reference itself.  Every 8th embedding row, all rows on 4
    fixed directions, gradient / update norms and 8x8 heads (as net_full_c2)."""
    dims = (40, 768, 3, 256)
    N, M, T = 256, 10, 180
    rec = train_steps(ref_net, ref_hparam, dims, wseed=81, wscale=2.0, xseed=82, N=N, M=M, T=T, steps=1)
    sd0 = recipe.make_weights(81, *dims, scale=2.0)
    e = rec["emb"][0].reshape(N * M, -1)
    dirs = np.random.default_rng(83).standard_normal((4, dims[3]))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    out = dict(dims=np.array(dims), wseed=81, wscale=2.0, xseed=82, N=N, M=M, T=T,
               loss=rec["losses"][0], emb_rows=e[::8], dirs=dirs, emb_proj=e.astype(np.float64) @ dirs.T,
               dw0=rec["dw0"], db0=rec["db0"], wb1=np.array(rec["wb1"]))
    for k, g in rec["grads"].items():
        out["gnorm." + k] = np.linalg.norm(g.astype(np.float64))
        out["ghead." + k] = g.reshape(g.shape[0], -1)[:8, :8] if g.ndim == 2 else g[:64]
    for k, p in rec["params1"].items():
        out["p1head." + k] = p.reshape(p.shape[0], -1)[:8, :8] if p.ndim == 2 else p[:64]
        out["dpnorm." + k] = np.linalg.norm(p.astype(np.float64) - sd0[k].astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "net_full_c5.npz"), **out)
    print("net_full_c5 loss", rec["losses"][0])


def net_fwd_c5(ref_net, ref_hparam):
    """Forward + GE2E loss at c5's global batch (N=256 x M=10, T=180, full dims, fp32; ≈20 s of
    CPU).  Every 8th embedding row in full, all 2560 rows projected on 4 fixed unit directions
    (a checksum of every row), the per-embedding loss and the loss."""
    import torch
    dims = (40, 768, 3, 256)
    N, M, T = 256, 10, 180
    hp = ref_hparam.hparam
    old = (hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj)
    hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = dims
    try:
        net = ref_net.SpeechEmbedder()
    finally:
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = old
    sd = recipe.make_weights(71, *dims, scale=2.0)
    net.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    x = torch.tensor(recipe.make_frames(72, N * M, T, dims[0]))
    ge2e = ref_net.GE2ELoss("cpu")
    with torch.no_grad():
        emb = net(x)
        loss = ge2e(emb.reshape(N, M, -1))
        import utils as ref_utils
        cos = ref_utils.get_cossim(emb.reshape(N, M, -1), ref_utils.get_centroids(emb.reshape(N, M, -1)))
        _, per = ref_utils.calc_loss(ge2e.w * cos + ge2e.b)
    dirs = np.random.default_rng(73).standard_normal((4, dims[3]))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    e = emb.numpy()
    np.savez_compressed(os.path.join(HERE, "net_fwd_c5.npz"), dims=np.array(dims), wseed=71, wscale=2.0, xseed=72,
                        N=N, M=M, T=T, loss=loss.item(), per=per.numpy(), emb_rows=e[::8], dirs=dirs,
                        emb_proj=e.astype(np.float64) @ dirs.T)
    print("net_fwd_c5 loss", loss.item())


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return
    import torch
    torch.set_num_threads(os.cpu_count())
    ref_hparam, ref_utils, ref_net = import_reference()
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    if only:  # e.g. `make_golden.py net_full_c2,net_fwd_c5`: just those fixtures
        for name in only:
            {"net_full_c2": net_full_c2, "net_fwd_c5": net_fwd_c5, "net_full_c5": net_full_c5}[name](ref_net, ref_hparam)
        return

    # ---- KAT-0: utils.py:166-173 -------------------------------------------------
    E0 = np.array([[0, 1, 0], [0, 0, 1], [0, 1, 0], [0, 1, 0], [1, 0, 0], [1, 0, 0]],
                  dtype=np.float32).reshape(3, 2, 3)
    r = ge2e_case(ref_utils, ref_net, E0, 1.0, 0.0)
    np.savez(os.path.join(HERE, "kat0.npz"), E=E0, w=1.0, b=0.0, **r)
    print("kat0 loss", r["loss"])

    # ---- GE2E vectors -----------------------------------------------------------
    cases = [("n4m5", 5, 4, 5, 10.0, -5.0, True),
             ("n4m5_flat", 6, 4, 5, 10.0, -5.0, False),
             ("n8m10_wb", 7, 8, 10, 3.7, -1.2, True),
             ("n64m10", 8, 64, 10, 10.0, -5.0, True),
             ("n256m10", 9, 256, 10, 10.0, -5.0, True),
             ("n3m2", 10, 3, 2, 10.0, -5.0, True)]
    for tag, seed, n, m, w, b, clustered in cases:
        E = recipe.make_embeddings(seed, n, m, 256, clustered)
        r = ge2e_case(ref_utils, ref_net, E, w, b)
        keep = dict(seed=seed, n=n, m=m, d=256, w=w, b=b, clustered=clustered,
                    loss=r["loss"], per=r["per"], dw=r["dw"], db=r["db"])
        if n * m <= 640:
            keep.update(dE=r["dE"], cossim=r["cossim"], centroids=r["centroids"])
        else:
            keep.update(dE_norm=np.linalg.norm(r["dE"].astype(np.float64)),
                        dE_head=r["dE"][:4], cossim_head=r["cossim"][:4],
                        cossim_diag=np.stack([r["cossim"][j, :, j] for j in range(n)]))
        if tag == "n4m5":  # the naive *_prior loop twins (utils.py:16-25,60-70,117-124)
            import torch
            Et = torch.tensor(E)
            Cp = ref_utils.get_centroids_prior(Et)
            cp = ref_utils.get_cossim_prior(Et, Cp)
            lp, pp = ref_utils.calc_loss_prior(w * cp + b)
            keep.update(prior_cossim=cp.numpy(), prior_loss=lp.item(), prior_per=pp.numpy())
        np.savez_compressed(os.path.join(HERE, f"ge2e_{tag}.npz"), **keep)
        print(tag, "loss", r["loss"], "dw", r["dw"], "db", r["db"])

    # ---- get_cossim with external centroids (test() call shape) ----------------
    import torch
    Ev = recipe.make_embeddings(31, 4, 3, 256, True)
    Ee = recipe.make_embeddings(32, 4, 3, 256, True)
    Cen = ref_utils.get_centroids(torch.tensor(Ee))
    cs = ref_utils.get_cossim(torch.tensor(Ev), Cen)
    np.savez_compressed(os.path.join(HERE, "cossim_ext.npz"), verif=Ev, enroll=Ee,
                        enroll_centroids=Cen.numpy(), cossim=cs.numpy())

    # ---- full training step, small dims ----------------------------------------
    dims = (40, 64, 3, 32)
    rec = train_steps(ref_net, ref_hparam, dims, wseed=11, wscale=3.0, xseed=12,
                      N=4, M=5, T=24, steps=3)
    out = dict(dims=np.array(dims), wseed=11, wscale=3.0, xseed=12, N=4, M=5, T=24, steps=3,
               losses=np.array(rec["losses"]), emb0=rec["emb"][0], emb_last=rec["emb"][-1],
               dw0=rec["dw0"], db0=rec["db0"], wb1=np.array(rec["wb1"]),
               wb_final=np.array(rec["wb_final"]))
    for k, v in rec["grads"].items():
        out["grad." + k] = v
    for k, v in rec["params1"].items():
        out["p1." + k] = v
    for k, v in rec["params_final"].items():
        out["pf." + k] = v
    np.savez_compressed(os.path.join(HERE, "net_small.npz"), **out)
    print("net_small losses", rec["losses"])

    # ---- one step at the full dims (c1: N=4 x M=5, T=160) ----------------------
    dims = (40, 768, 3, 256)
    rec = train_steps(ref_net, ref_hparam, dims, wseed=21, wscale=2.0, xseed=22,
                      N=4, M=5, T=160, steps=1)
    out = dict(dims=np.array(dims), wseed=21, wscale=2.0, xseed=22, N=4, M=5, T=160,
               loss=rec["losses"][0], emb=rec["emb"][0], dw0=rec["dw0"], db0=rec["db0"],
               wb1=np.array(rec["wb1"]))
    for k, g in rec["grads"].items():
        out["gnorm." + k] = np.linalg.norm(g.astype(np.float64))
        out["ghead." + k] = g.reshape(g.shape[0], -1)[:8, :8] if g.ndim == 2 else g[:64]
    for k, p in rec["params1"].items():
        out["p1head." + k] = p.reshape(p.shape[0], -1)[:8, :8] if p.ndim == 2 else p[:64]
    np.savez_compressed(os.path.join(HERE, "net_full_c1.npz"), **out)
    print("net_full_c1 loss", rec["losses"][0])

    # ---- the headline config (c2) and c5's global forward, pinned to the reference -------
    net_full_c2(ref_net, ref_hparam)
    net_fwd_c5(ref_net, ref_hparam)
    net_full_c5(ref_net, ref_hparam)

    # ---- init RNG parity: reference SpeechEmbedder() under torch.manual_seed ------
    hp = ref_hparam.hparam
    old = (hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj)
    hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = (40, 64, 3, 32)
    try:
        torch.manual_seed(1234)
        net = ref_net.SpeechEmbedder()
    finally:
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = old
    np.savez_compressed(os.path.join(HERE, "init_seed1234.npz"),
                        **{k: v.detach().numpy() for k, v in net.state_dict().items()})

    # ---- data loader + EER evaluation (train_speech_embedder.py:92-154) ---------
    eer_and_loader_fixtures(ref_hparam, ref_net)

    # ---- the parsed config -----------------------------------------------------
    hp = ref_hparam.hparam
    with open(os.path.join(HERE, "hparam.json"), "w") as f:
        json.dump(json.loads(json.dumps(hp)), f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
