"""CPU: ``dropin/run.py`` binds a reference-layout script to this package.

A script started as ``python script.py`` gets its own directory at ``sys.path[0]``, ahead of
``PYTHONPATH``, so sibling modules named ``hparam`` / ``data_load`` / ``speech_embedder_net`` /
``utils`` would win over any shim directory.  These tests build such a directory with decoy
siblings (the builder's own stubs that refuse to import) and a script that imports them the way the
reference's scripts do (train_speech_embedder.py:15-17, data_load.py:16-17), run it through the
launcher in a fresh interpreter, and check where every name resolved.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "dropin")
PKG = os.path.join(ROOT, "pytorch_speaker_verification_amd")
REFERENCE = "/root/reference"

DECOY = 'raise ImportError("decoy sibling {name}.py was imported: the launcher let the script directory win")\n'

SCRIPT = textwrap.dedent('''
    import json, sys
    from hparam import hparam as hp
    from data_load import SpeakerDatasetTIMIT, SpeakerDatasetTIMITPreprocessed
    from speech_embedder_net import SpeechEmbedder, GE2ELoss, get_centroids, get_cossim
    from utils import mfccs_and_spec
    import sibling_only
    out = {m: sys.modules[m].__file__ for m in ("hparam", "data_load", "speech_embedder_net", "utils", "sibling_only")}
    out["classes"] = [c.__module__ for c in (SpeechEmbedder, GE2ELoss, SpeakerDatasetTIMITPreprocessed)]
    out["funcs"] = [f.__module__ for f in (get_centroids, get_cossim)]
    out["argv"] = sys.argv
    out["name"] = __name__
    out["train_N"] = hp.train.N
    try:
        mfccs_and_spec("x.wav")
        out["mfcc"] = "returned"
    except NotImplementedError as e:
        out["mfcc"] = "NotImplementedError"
    json.dump(out, open(sys.argv[1], "w"))
''')


def _layout(tmp_path):
    ref = tmp_path / "refckout"
    (ref / "config").mkdir(parents=True)
    for name in ("hparam", "data_load", "speech_embedder_net", "utils"):
        (ref / f"{name}.py").write_text(DECOY.format(name=name))
    (ref / "sibling_only.py").write_text("VALUE = 1\n")
    (ref / "train_like.py").write_text(SCRIPT)
    # a CWD-relative config as the reference reads it (hparam.py:49), with one distinctive value
    cfg = open(os.path.join(PKG, "config", "config.yaml")).read()
    assert "N : 4" in cfg or "N: 4" in cfg
    (ref / "config" / "config.yaml").write_text(cfg.replace("N : 4", "N : 7", 1).replace("N: 4", "N: 7", 1))
    return ref


def _run(args, cwd, env_extra=None):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    env.pop("PYTHONPATH", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True, timeout=300)


def test_launcher_resolves_every_shimmed_module_to_dropin(tmp_path):
    ref = _layout(tmp_path)
    out = tmp_path / "out.json"
    # even with the reference checkout on PYTHONPATH ahead of everything, dropin/ must win
    r = _run([os.path.join(DROPIN, "run.py"), "train_like.py", str(out), "extra"], cwd=str(ref),
             env_extra={"PYTHONPATH": str(ref)})
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(out.read_text())
    for m in ("hparam", "data_load", "speech_embedder_net", "utils"):
        assert os.path.dirname(os.path.realpath(got[m])) == os.path.realpath(DROPIN), (m, got[m])
    # modules without a shim still come from the script's own directory
    assert os.path.realpath(got["sibling_only"]) == os.path.realpath(ref / "sibling_only.py")
    assert all(c.startswith("pytorch_speaker_verification_amd.") for c in got["classes"] + got["funcs"]), got
    assert got["argv"] == [str(ref / "train_like.py"), str(out), "extra"]
    assert got["name"] == "__main__"
    assert got["train_N"] == 7  # the CWD's config/config.yaml, as the reference reads it
    assert got["mfcc"] == "NotImplementedError"


def test_plain_pythonpath_recipe_does_not_bind(tmp_path):
    """The old documented recipe (PYTHONPATH=dropin python script.py) imports the script's siblings:
    kept as a regression check on why the launcher exists."""
    ref = _layout(tmp_path)
    r = _run(["train_like.py", str(tmp_path / "o.json")], cwd=str(ref),
             env_extra={"PYTHONPATH": os.pathsep.join([DROPIN, ROOT])})
    assert r.returncode != 0 and "decoy sibling" in r.stderr


def test_launcher_refuses_missing_script_and_preimported_modules(tmp_path):
    r = _run([os.path.join(DROPIN, "run.py"), str(tmp_path / "nope.py")], cwd=str(tmp_path))
    assert r.returncode == 2 and "no such script" in r.stderr
    r = _run([os.path.join(DROPIN, "run.py")], cwd=str(tmp_path))
    assert r.returncode == 2
    # a shimmed name imported before the launcher runs (here `utils`, from a decoy-free directory
    # of its own) must make run.main refuse instead of mixing two resolutions; in a fresh process
    (tmp_path / "pre").mkdir()
    (tmp_path / "pre" / "utils.py").write_text("X = 1\n")
    (tmp_path / "s.py").write_text("pass\n")
    probe = textwrap.dedent(f"""
        import sys
        sys.path[:0] = [{str(tmp_path / "pre")!r}, {DROPIN!r}]
        import utils, run
        try:
            run.main([{str(tmp_path / "s.py")!r}])
        except RuntimeError as e:
            print("REFUSED", e)
    """)
    r = _run(["-c", probe], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "REFUSED" in r.stdout and "'utils'" in r.stdout, r.stdout
    # the path order, checked in this process without leaving `run` imported
    sys.path.insert(0, DROPIN)
    try:
        import importlib
        run = importlib.import_module("run")
        assert run.resolve_path("/x/y", ["", "/x/y", "/a"])[:4] == [DROPIN, ROOT, "/x/y", "/a"]
    finally:
        sys.path.remove(DROPIN)
        sys.modules.pop("run", None)


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="the reference checkout is only in the build container")
def test_reference_training_script_binds_to_this_package(tmp_path):
    """The reference's own train_speech_embedder.py, run unchanged through the launcher from a
    checkout-like CWD: its train() builds this package's dataset (no GPU here, so it stops at the
    first I/O -- the missing training directory -- inside this package's data_load.py)."""
    cwd = tmp_path / "run"
    (cwd / "config").mkdir(parents=True)
    cfg = open(os.path.join(PKG, "config", "config.yaml")).read()
    (cwd / "config" / "config.yaml").write_text(cfg)
    r = _run([os.path.join(DROPIN, "run.py"), os.path.join(REFERENCE, "train_speech_embedder.py")], cwd=str(cwd))
    assert r.returncode != 0
    tb = r.stderr
    assert os.path.join(REFERENCE, "train_speech_embedder.py") in tb, tb[-3000:]
    assert os.path.join("pytorch_speaker_verification_amd", "data_load.py") in tb, tb[-3000:]
    assert "FileNotFoundError" in tb, tb[-3000:]
    assert os.path.join(REFERENCE, "data_load.py") not in tb
