"""Configuration singleton with the reference's surface (hparam.py:7-61).

``hparam`` is built at import time from ``config/config.yaml`` relative to the current
working directory -- as the reference does (hparam.py:49) -- and falls back to the copy
shipped in this package when the CWD has none.  Unlike the reference (which calls
``yaml.load_all`` without a Loader and fails under PyYAML >= 6) the file is
parsed with ``yaml.safe_load_all``.  Keys are the reference's (config/config.yaml:1-40);
``hp.model.hidden`` etc. are read at SpeechEmbedder construction time, so overriding them
builds a smaller net.
"""
from __future__ import annotations

import os

import yaml

_DEFAULT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config", "config.yaml")


def load_hparam(filename):
    """Merge the YAML documents of ``filename`` into one dict (hparam.py:7-14)."""
    with open(filename, "r") as stream:
        out = {}
        for doc in yaml.safe_load_all(stream):
            if doc:
                out.update(doc)
    return out


def merge_dict(user, default):
    """Recursively fill missing keys of ``user`` from ``default`` (hparam.py:17-24)."""
    if isinstance(user, dict) and isinstance(default, dict):
        for k, v in default.items():
            user[k] = merge_dict(user[k], v) if k in user else v
    return user


class Dotdict(dict):
    """dict with attribute access; nested dicts become Dotdicts (hparam.py:27-44)."""

    __getattr__ = dict.__getitem__
    __setattr__ = dict.__setitem__
    __delattr__ = dict.__delitem__

    def __init__(self, dct=None):
        super().__init__()
        for key, value in (dct or {}).items():
            self[key] = Dotdict(value) if hasattr(value, "keys") else value


class Hparam(Dotdict):
    """The configuration object (hparam.py:47-58)."""

    def __init__(self, file="config/config.yaml"):
        super().__init__()
        path = file if os.path.exists(file) else _DEFAULT
        for k, v in Dotdict(load_hparam(path)).items():
            self[k] = v
        self.__dict__["_path"] = path

    __getattr__ = Dotdict.__getitem__
    __setattr__ = Dotdict.__setitem__
    __delattr__ = Dotdict.__delitem__


hparam = Hparam()
