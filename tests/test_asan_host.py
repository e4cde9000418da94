"""CPU sanitizer run of the library's host-only code (VERDICT r03
item 8): `make -C mpc-mmd_amd asan` builds csrc/host_constants.cpp with
-fsanitize=address,undefined into a harness (tests/native/asan_host.cpp) that
builds every variant's constants and the dynamic-obstacle QP tracks.  The run
must be clean (any ASan / UBSan report aborts it: -fno-sanitize-recover), and
its values must equal the product library's (mpcmmd_host_constant,
mpcmmd_obs_dynamic_traj: no GPU needed)."""
import math
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpc-mmd_amd")
sys.path[:0] = [ROOT, PKG]


def _seq(v):
    s = 0.0
    a = 0.0
    for x in np.asarray(v, np.float64).tolist():
        s += x
        a += math.fabs(x)
    return s, a


@pytest.fixture(scope="module")
def asan_lines():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.run(["make", "-C", PKG, "asan"], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(PKG, "build_asan", "asan_host")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return [ln.split() for ln in r.stdout.splitlines() if ln.strip()]


def test_asan_constants_match_library(asan_lines):
    from optimizer import _native
    names = {v: k for k, v in _native.VARIANT.items()}
    seen = 0
    for tag, H, variant, name, cnt, s, a in asan_lines:
        if tag != "const" or int(variant) not in names:
            continue
        cfg = _native.make_config(4, 2, 0.1, int(H), "gaussian", 0.0, 0.0, variant=names[int(variant)])
        v = _native.host_constant(cfg, name)
        assert v.size == int(cnt), (H, variant, name)
        ls, la = _seq(v)
        assert ls == float(s) and la == float(a), (H, variant, name, ls, s)
        seen += 1
    assert seen >= 7 * 7 * 2


def test_asan_dynamic_tracks_match_library(asan_lines):
    from optimizer import _native
    O = 20
    i = np.arange(O)
    x0 = (30.0 + 5.0 * i).astype(np.float32)
    y0 = np.where(i % 2 == 1, 1.75, -1.75).astype(np.float32)
    vx0 = (np.float32(3.0) + np.float32(0.5) * i.astype(np.float32)).astype(np.float32)
    vy0 = (np.float32(0.1) * (i % 3).astype(np.float32)).astype(np.float32)
    vd = (np.float32(4.0) + np.float32(0.25) * i.astype(np.float32)).astype(np.float32)
    xt, yt = _native.obs_dynamic_traj(x0, y0, vx0, vy0, vd, -1.75)
    got = {ln[3]: (float(ln[5]), float(ln[6])) for ln in asan_lines if ln[0] == "dyn"}
    assert _seq(xt.reshape(-1)) == got["x_traj"]
    assert _seq(yt.reshape(-1)) == got["y_traj"]
