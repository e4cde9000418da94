"""The ctypes binding of libmpcmmd.so (``mpc-mmd_amd/optimizer/_native.py``),
loaded by file path: this package is also named ``optimizer`` (the reference
keeps two packages of that name, ``synthetic_*/optimizer`` and
``carla/optimizer``), so the static one cannot be imported by name here."""
from __future__ import annotations

import importlib.util
import os
import sys

_NAME = "mpcmmd_native"


def native():
    mod = sys.modules.get(_NAME)
    if mod is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            "optimizer", "_native.py")
        spec = importlib.util.spec_from_file_location(_NAME, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[_NAME] = mod
        spec.loader.exec_module(mod)
    return mod
