#!/usr/bin/env python3
"""Run one of the reference's scripts, unchanged, on this package's HIP path.

    cd /path/to/reference/checkout            # config/config.yaml is read relative to the CWD
    python /path/to/this/repo/dropin/run.py train_speech_embedder.py [args...]

The reference's scripts import their siblings by bare module name (``from hparam import hparam``,
``from data_load import ...``, ``from speech_embedder_net import ...``: train_speech_embedder.py:15-17,
data_load.py:16-17, dvector_create.py:19-21).  Started as ``python script.py``, Python puts the
script's own directory at ``sys.path[0]``, AHEAD of ``PYTHONPATH``, so a shim directory on
``PYTHONPATH`` never wins and the reference's own ``nn.LSTM`` modules are imported.  This launcher
fixes the order instead: this ``dropin/`` directory first, then the repo root (the package the
shims re-export), then the script's directory (so modules that have no shim, such as
``VAD_segments``, still resolve to the reference's), then the rest of ``sys.path``.  The script then
runs as ``__main__`` with ``sys.argv`` = [script, args...], as ``python script.py args...`` would.
"""
from __future__ import annotations

import os
import runpy
import sys

DROPIN = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(DROPIN)
# the module names the reference's scripts import that this directory shadows
SHIMMED = ("hparam", "speech_embedder_net", "utils", "data_load")


def resolve_path(script_dir, path=None):
    """The launcher's ``sys.path``: dropin, repo root, the script's directory, then ``path`` with
    those three (and the empty / CWD entry when it is the script's directory) removed."""
    path = sys.path if path is None else path
    first = [DROPIN, ROOT, script_dir]
    seen = {os.path.realpath(p) for p in first}
    rest = [p for p in path if os.path.realpath(p or os.getcwd()) not in seen]
    return first + rest


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__.strip(), file=sys.stderr)
        return 2
    script = os.path.abspath(argv[0])
    if not os.path.isfile(script):
        print(f"dropin/run.py: no such script: {argv[0]}", file=sys.stderr)
        return 2
    stale = [m for m in SHIMMED if m in sys.modules]
    if stale:  # imported under other resolution rules already: refuse rather than mix two builds
        raise RuntimeError(f"modules {stale} are already imported; start the script through this launcher")
    sys.path[:] = resolve_path(os.path.dirname(script))
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
