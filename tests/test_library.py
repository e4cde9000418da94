"""The C-ABI library without a GPU: it loads, exports every symbol
include/mpcmmd.h declares, validates configurations, refuses to run without a
device (no CPU fallback), and its host-built batch-invariant constants are
bit-identical to the oracle's.  CPU only (no compute calls)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle.problem import Problem

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def nat():
    from optimizer import _native
    return _native


def test_exports_every_declared_symbol(nat):
    hdr = open(os.path.join(ROOT, "include", "mpcmmd.h")).read()
    declared = set(re.findall(r"\b(mpcmmd_[a-z_]+)\s*\(", hdr))
    L = nat.lib()
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert declared == set(nat.SYMBOLS)
    assert L.mpcmmd_abi_version() == nat.ABI_VERSION


def test_no_device_means_error_not_fallback(nat):
    if nat.lib().mpcmmd_device_count() > 0:
        pytest.skip("a GPU is visible")
    cfg = nat.make_config(8, 3, 0.1, 10, "gaussian", 0.0, 0.0, num_batch=32)
    with pytest.raises(nat.NativeError):
        nat.Handle(cfg)
    from optimizer import cem
    with pytest.raises(nat.NativeError):
        cem.CEM(8, 3, 0.1, 10, "gaussian", 0.0, 0.0)


def test_config_validation(nat):
    L = nat.lib()
    h = C.c_void_p()
    for bad in (dict(num_batch=10), dict(num_prime=101), dict(num_obs=0)):
        kw = dict(num_batch=32)
        kw.update({k: v for k, v in bad.items() if k == "num_batch"})
        args = dict(num_reduced=8, num_obs=bad.get("num_obs", 3), noise_level=0.1,
                    num_prime=bad.get("num_prime", 10), noise="gaussian", acc_const_noise=0.0,
                    steer_const_noise=0.0)
        cfg = nat.make_config(**args, **kw)
        rc = L.mpcmmd_create(C.byref(cfg), C.byref(h))
        assert rc < 0 and L.mpcmmd_last_error()


@pytest.mark.parametrize("H,variant", [(10, "static"), (30, "static"), (50, "dynamic")])
def test_host_constants_bit_identical(nat, H, variant):
    cfg = nat.make_config(22, 10, 0.1, H, "gaussian", 0.0, 0.0, num_batch=1024, variant=variant)
    p = Problem(22, 10, 0.1, H, "gaussian", 0.0, 0.0, num_batch=1024, variant=variant)
    pairs = {
        "P": p.P.astype(np.float64), "Pdot": p.Pdot.astype(np.float64), "Pddot": p.Pddot.astype(np.float64),
        "P64": p.P64, "Pdot64": p.Pd64, "Pddot64": p.Pdd64, "P_prime": p.P_prime.astype(np.float64),
        "guess_kinv_x": p.guess_kinv_x, "guess_kinv_y": p.guess_kinv_y,
        "proj_kinv_x": p.proj_kinv_x, "proj_kinv_y": p.proj_kinv_y, "fit": p.fit,
    }
    for name, ref in pairs.items():
        got = nat.host_constant(cfg, name)
        assert got.size == ref.size, name
        assert np.array_equal(got, ref.reshape(-1)), f"{name}: max diff {np.abs(got - ref.reshape(-1)).max()}"


def test_drop_in_package_imports_without_jax():
    import optimizer
    from optimizer import cem, cem_helper  # noqa: F401
    assert hasattr(cem, "CEM")
    import sys
    assert "jax" not in sys.modules


@pytest.mark.parametrize("O,variant", [(3, "carla_town05"), (7, "carla_town10hd")])
def test_det_kkt_inverse_bit_identical(nat, O, variant):
    """compute_cem_det's projection KKT (carla/optimizer/projection_det.py:
    149-160: + rho_obs A_obs^T A_obs, A_obs = tile(P, (O, 1))), host-built,
    bit-identical to the oracle's."""
    cfg = nat.make_config(10, O, 0.1, 60, "gaussian", 0.0, 0.0, num_batch=100, variant=variant)
    p = Problem(10, O, 0.1, 60, "gaussian", 0.0, 0.0, num_batch=100, variant=variant)
    kx, ky = p.det_kinv()
    assert np.array_equal(nat.host_constant(cfg, "det_kinv_x"), kx.reshape(-1))
    assert np.array_equal(nat.host_constant(cfg, "det_kinv_y"), ky.reshape(-1))
    # the obstacle rows change the system: not the plain projection's inverse
    assert not np.array_equal(kx, p.proj_kinv_x)

