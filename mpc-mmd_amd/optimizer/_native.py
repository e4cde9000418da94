"""ctypes binding of libmpcmmd.so (include/mpcmmd.h).

The library is built in-tree (``mpc-mmd_amd/libmpcmmd.so``, see
``__graft_entry__.build``).  There is no fallback: if the library is missing,
or no GPU is visible when a handle is created, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPCMMD_LIB", os.path.join(os.path.dirname(_HERE), "libmpcmmd.so"))

COST = {"mmd_opt": 0, "mmd_random": 1, "cvar": 2, "saa": 3, "det": 4}  # det: CARLA handles (compute_cem_det)
NOISE = {"gaussian": 0, "beta": 1}
VARIANT = {"static": 0, "dynamic": 1, "carla_town05": 2, "carla_town10hd": 3}
RESULT_STRIDE_BETA_MAX = 32
ABI_VERSION = 4

SYMBOLS = (
    "mpcmmd_abi_version", "mpcmmd_last_error", "mpcmmd_device_count", "mpcmmd_create",
    "mpcmmd_destroy", "mpcmmd_set_stream", "mpcmmd_get_stream", "mpcmmd_solve", "mpcmmd_begin",
    "mpcmmd_iterate", "mpcmmd_finish", "mpcmmd_sync", "mpcmmd_profile", "mpcmmd_kernel_times",
    "mpcmmd_kernel_name", "mpcmmd_buffer_info", "mpcmmd_read", "mpcmmd_write", "mpcmmd_run_stage",
    "mpcmmd_host_constant", "mpcmmd_obs_dynamic_traj", "mpcmmd_validate", "mpcmmd_create_batch",
    "mpcmmd_max_configs", "mpcmmd_solve_batch", "mpcmmd_begin_batch", "mpcmmd_finish_batch",
    "mpcmmd_carla_begin", "mpcmmd_carla_solve", "mpcmmd_path_smoothing", "mpcmmd_path_parameters",
    "mpcmmd_global_to_frenet", "mpcmmd_set_graphs", "mpcmmd_handle_info",
)


class Config(C.Structure):
    _fields_ = [("num_reduced", C.c_int32), ("num_obs", C.c_int32), ("noise_level", C.c_float),
                ("num_prime", C.c_int32), ("noise", C.c_int32), ("acc_const_noise", C.c_float),
                ("steer_const_noise", C.c_float), ("num_batch", C.c_int32), ("variant", C.c_int32),
                ("maxiter_cem", C.c_int32), ("device", C.c_int32), ("seed", C.c_uint32)]


class Draws(C.Structure):
    _fields_ = [("pop0", C.POINTER(C.c_float)), ("roll", C.POINTER(C.c_float)),
                ("resample", C.POINTER(C.c_float)), ("beta_z0", C.POINTER(C.c_float)),
                ("beta_z", C.POINTER(C.c_float)), ("init_eps", C.POINTER(C.c_float))]


class Result(C.Structure):
    _fields_ = [("cx", C.c_float * 11), ("cy", C.c_float * 11), ("cost_lane", C.c_float),
                ("cost_obs", C.c_float), ("sigma", C.c_float), ("res_beta", C.c_float * 20),
                ("beta", C.POINTER(C.c_float)), ("elite_proj", C.POINTER(C.c_int32)),
                ("elite_obs", C.POINTER(C.c_int32)), ("elite_cem", C.POINTER(C.c_int32)),
                ("steering", C.POINTER(C.c_float)), ("v_best", C.POINTER(C.c_float)),
                ("mean_param", C.c_float * 8)]


class Path(C.Structure):
    _fields_ = [("num_path", C.c_int32), ("x_path", C.POINTER(C.c_float)), ("y_path", C.POINTER(C.c_float)),
                ("arc_vec", C.POINTER(C.c_float)), ("Fx_dot", C.POINTER(C.c_float)),
                ("Fy_dot", C.POINTER(C.c_float)), ("kappa", C.POINTER(C.c_float))]

PATH_KEYS = ("x_path", "y_path", "arc_vec", "Fx_dot", "Fy_dot", "kappa")


class ValidateArgs(C.Structure):
    _fields_ = [("num_cfg", C.c_int32), ("num_obs", C.c_int32), ("num_prime", C.c_int32),
                ("num_rollouts", C.c_int32), ("noise", C.c_int32), ("variant", C.c_int32),
                ("noise_level", C.c_double), ("acc_const_noise", C.c_double), ("steer_const_noise", C.c_double),
                ("seed", C.c_uint32), ("device", C.c_int32),
                ("cx", C.POINTER(C.c_double)), ("cy", C.POINTER(C.c_double)),
                ("init_state", C.POINTER(C.c_double)), ("x_obs", C.POINTER(C.c_float)),
                ("y_obs", C.POINTER(C.c_float)), ("draws", C.POINTER(C.c_double)),
                ("keys", C.POINTER(C.c_uint32)), ("count", C.POINTER(C.c_int32)),
                ("count_lane", C.POINTER(C.c_int32))]


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libmpcmmd.so once (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (or `make -C mpc-mmd_amd`)")
    L = C.CDLL(LIB_PATH)
    fp = C.POINTER(C.c_float)
    vp = C.c_void_p
    L.mpcmmd_abi_version.restype = C.c_int32
    L.mpcmmd_last_error.restype = C.c_char_p
    L.mpcmmd_device_count.restype = C.c_int32
    L.mpcmmd_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
    L.mpcmmd_create_batch.argtypes = [C.POINTER(Config), C.c_int32, C.POINTER(vp)]
    L.mpcmmd_max_configs.argtypes = [vp]
    L.mpcmmd_max_configs.restype = C.c_int32
    L.mpcmmd_handle_info.argtypes = [vp, C.c_char_p, C.POINTER(C.c_int64)]
    ip = C.POINTER(C.c_int32)
    bargs = [vp, C.c_int32, C.c_int32, ip, fp, fp, fp, fp, fp, fp]
    L.mpcmmd_solve_batch.argtypes = bargs + [C.POINTER(Result)]
    L.mpcmmd_begin_batch.argtypes = bargs
    L.mpcmmd_finish_batch.argtypes = [vp, C.c_int32, C.POINTER(Result)]
    L.mpcmmd_destroy.argtypes = [vp]
    L.mpcmmd_destroy.restype = None
    L.mpcmmd_set_stream.argtypes = [vp, vp]
    L.mpcmmd_get_stream.argtypes = [vp]
    L.mpcmmd_get_stream.restype = vp
    args = [vp, C.c_int32, C.c_int32, fp, fp, fp, fp, fp, C.c_float, C.POINTER(Draws)]
    L.mpcmmd_solve.argtypes = args + [C.POINTER(Result)]
    L.mpcmmd_begin.argtypes = args
    L.mpcmmd_iterate.argtypes = [vp, C.c_int32, C.c_int32]
    L.mpcmmd_finish.argtypes = [vp, C.POINTER(Result)]
    L.mpcmmd_sync.argtypes = [vp]
    L.mpcmmd_profile.argtypes = [vp, C.c_int32]
    L.mpcmmd_kernel_times.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_int32]
    L.mpcmmd_kernel_name.argtypes = [C.c_int32]
    L.mpcmmd_kernel_name.restype = C.c_char_p
    L.mpcmmd_buffer_info.argtypes = [vp, C.c_char_p, C.POINTER(C.c_size_t)]
    L.mpcmmd_read.argtypes = [vp, C.c_char_p, vp, C.c_size_t]
    L.mpcmmd_write.argtypes = [vp, C.c_char_p, vp, C.c_size_t]
    L.mpcmmd_run_stage.argtypes = [vp, C.c_int32, C.c_int32]
    L.mpcmmd_host_constant.argtypes = [C.POINTER(Config), C.c_char_p, C.POINTER(C.c_double), C.c_size_t]
    L.mpcmmd_validate.argtypes = [C.POINTER(ValidateArgs)]
    L.mpcmmd_obs_dynamic_traj.argtypes = [C.c_int32, fp, fp, fp, fp, fp, C.c_float, fp, fp]
    cargs = [vp, C.c_int32, C.c_int32, fp, fp, fp, fp, fp, C.c_float, C.POINTER(Path), C.POINTER(Draws)]
    L.mpcmmd_set_graphs.argtypes = [vp, C.c_int32]
    L.mpcmmd_carla_begin.argtypes = cargs
    L.mpcmmd_carla_solve.argtypes = cargs + [C.POINTER(Result)]
    L.mpcmmd_path_smoothing.argtypes = [C.c_int32, fp, fp, C.c_float, fp, fp]
    L.mpcmmd_path_parameters.argtypes = [C.c_int32, fp, fp, fp, fp, fp, fp, fp, fp, fp]
    L.mpcmmd_global_to_frenet.argtypes = [C.POINTER(Path), C.c_int32, fp, fp, fp, fp, fp, fp, fp]
    if L.mpcmmd_abi_version() != ABI_VERSION:
        raise NativeError("libmpcmmd ABI version mismatch")
    _lib = L
    return L


def check(rc):
    if rc < 0:
        raise NativeError(f"libmpcmmd error {rc}: {lib().mpcmmd_last_error().decode()}")
    return rc


def make_config(num_reduced, num_obs, noise_level, num_prime, noise, acc_const_noise, steer_const_noise,
                num_batch=100, variant="static", maxiter_cem=20, device=0, seed=0):
    return Config(int(num_reduced), int(num_obs), float(noise_level), int(num_prime), NOISE[noise],
                  float(acc_const_noise), float(steer_const_noise), int(num_batch), VARIANT[variant],
                  int(maxiter_cem), int(device), int(seed) & 0xFFFFFFFF)


def host_constant(cfg, name):
    L = lib()
    n = check(L.mpcmmd_host_constant(C.byref(cfg), name.encode(), None, 0))
    out = np.empty(n, np.float64)
    check(L.mpcmmd_host_constant(C.byref(cfg), name.encode(), out.ctypes.data_as(C.POINTER(C.c_double)), n))
    return out


def obs_dynamic_traj(x0, y0, vx0, vy0, v_des, y_des=-1.75):
    """mpcmmd_obs_dynamic_traj: per-obstacle QP trajectories [O][100] x 2
    (obs_data.compute_obs_guess, obs_data_generate_dynamic.py:73-109)."""
    a = [np.ascontiguousarray(np.asarray(v, np.float32).reshape(-1)) for v in (x0, y0, vx0, vy0, v_des)]
    O = a[0].size
    if any(v.size != O for v in a):
        raise ValueError("obstacle arrays differ in length")
    xt = np.empty((O, 100), np.float32)
    yt = np.empty((O, 100), np.float32)
    check(lib().mpcmmd_obs_dynamic_traj(O, *[_fptr(v) for v in a], float(y_des), _fptr(xt), _fptr(yt)))
    return xt, yt


def validate(cx, cy, init_state, x_obs, y_obs, keys, num_prime, noise, noise_level, acc_const_noise=0.0,
             steer_const_noise=0.0, num_rollouts=1000, variant="static", draws=None, seed=0, device=0):
    """mpcmmd_validate over K configurations: (count [K], count_lane [K])
    (S/validation.py compute_stats :134-171).  cx, cy [K,11]; init_state
    [K,6]; x_obs, y_obs [K,O,100] obstacle tracks; keys [K]; draws
    [K,3,R,H] fp64 or None (internal Philox)."""
    d = lambda a, *shape: np.ascontiguousarray(np.asarray(a, np.float64).reshape(*shape))
    cx = np.atleast_2d(np.asarray(cx, np.float64))
    K = cx.shape[0]
    cx, cy = d(cx, K, 11), d(cy, K, 11)
    st = d(init_state, K, 6)
    xo = np.ascontiguousarray(np.asarray(x_obs, np.float32).reshape(K, -1, 100))
    yo = np.ascontiguousarray(np.asarray(y_obs, np.float32).reshape(K, -1, 100))
    O = xo.shape[1]
    ks = np.ascontiguousarray(np.asarray(keys, np.int64).reshape(K).astype(np.uint32))
    dr = None if draws is None else d(draws, K, 3, num_rollouts, num_prime)
    cnt = np.zeros(K, np.int32)
    cl = np.zeros(K, np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    args = ValidateArgs(K, O, int(num_prime), int(num_rollouts), NOISE[noise], VARIANT[variant], float(noise_level),
                        float(acc_const_noise), float(steer_const_noise), int(seed) & 0xFFFFFFFF, int(device),
                        dp(cx), dp(cy), dp(st), _fptr(xo), _fptr(yo), None if dr is None else dp(dr),
                        ks.ctypes.data_as(C.POINTER(C.c_uint32)), cnt.ctypes.data_as(C.POINTER(C.c_int32)),
                        cl.ctypes.data_as(C.POINTER(C.c_int32)))
    check(lib().mpcmmd_validate(C.byref(args)))
    return cnt, cl


def _fptr(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


def make_path(path):
    """mpcmmd_path from a dict of the six arrays (PATH_KEYS); returns
    (Path, keep) - keep holds the contiguous fp32 copies alive."""
    keep = {k: np.ascontiguousarray(np.asarray(path[k], np.float32).reshape(-1)) for k in PATH_KEYS}
    P = keep["x_path"].size
    if any(v.size != P for v in keep.values()):
        raise ValueError("path arrays differ in length")
    return Path(P, *(_fptr(keep[k]) for k in PATH_KEYS)), keep


def path_smoothing(x_wp, y_wp, threshold):
    """mpcmmd_path_smoothing (Helper.custom_path_smoothing, carla/optimizer/cem_helper.py:391-410)."""
    xw = np.ascontiguousarray(np.asarray(x_wp, np.float32).reshape(-1))
    yw = np.ascontiguousarray(np.asarray(y_wp, np.float32).reshape(-1))
    xo = np.empty_like(xw)
    yo = np.empty_like(yw)
    check(lib().mpcmmd_path_smoothing(xw.size, _fptr(xw), _fptr(yw), float(threshold), _fptr(xo), _fptr(yo)))
    return xo, yo


def path_parameters(x_path, y_path):
    """mpcmmd_path_parameters (Helper.compute_path_parameters, cem_helper.py:321-345):
    Fx_dot, Fy_dot, Fx_ddot, Fy_ddot, arc_vec, kappa, arc_length."""
    x = np.ascontiguousarray(np.asarray(x_path, np.float32).reshape(-1))
    y = np.ascontiguousarray(np.asarray(y_path, np.float32).reshape(-1))
    outs = [np.empty_like(x) for _ in range(6)]
    al = C.c_float()
    check(lib().mpcmmd_path_parameters(x.size, _fptr(x), _fptr(y), *[_fptr(o) for o in outs], C.byref(al)))
    return (*outs, np.float32(al.value))


def global_to_frenet(path, x, y, v, vdot, psi, psidot):
    """mpcmmd_global_to_frenet (Helper.global_to_frenet, cem_helper.py:348-388) of
    arrays of states: (x, y, vx, vy, ax, ay, psi) in the Frenet frame."""
    a = [np.ascontiguousarray(np.asarray(u, np.float32).reshape(-1)) for u in (x, y, v, vdot, psi, psidot)]
    n = a[0].size
    a = [np.ascontiguousarray(np.broadcast_to(u, (n,))) for u in a]
    out = np.empty((n, 7), np.float32)
    pth, keep = make_path(path)
    check(lib().mpcmmd_global_to_frenet(C.byref(pth), n, *[_fptr(u) for u in a], _fptr(out)))
    return tuple(out[:, k] for k in range(7))


class Handle:
    """Owns one mpcmmd_handle (one device, one stream).  ``max_configs`` > 1
    sizes it for ``solve_batch`` (that many configurations per launch)."""

    def __init__(self, cfg, max_configs=1):
        self.cfg = cfg
        self.max_configs = int(max_configs)
        self._L = lib()
        if self._L.mpcmmd_device_count() < 1:
            raise NativeError("no HIP device visible: libmpcmmd needs an MI355X (gfx950)")
        h = C.c_void_p()
        check(self._L.mpcmmd_create_batch(C.byref(cfg), self.max_configs, C.byref(h)))
        self._h = h
        self._keep = []

    def close(self):
        if getattr(self, "_h", None):
            self._L.mpcmmd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- solve ----------------------------------------------------------------
    def _inputs(self, init_state, mean, cov, x_obs, y_obs, draws):
        f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float32))
        ins = dict(init_state=f(init_state).reshape(6), mean=f(mean).reshape(8), cov=f(cov).reshape(64),
                   x_obs=f(x_obs), y_obs=f(y_obs))
        if ins["x_obs"].shape != (self.cfg.num_obs, 100) or ins["y_obs"].shape != (self.cfg.num_obs, 100):
            raise ValueError(f"x_obs_traj / y_obs_traj must be [{self.cfg.num_obs}, 100]")
        d = None
        if draws is not None:
            keep = {}
            names = ("pop0", "roll", "resample", "beta_z0", "beta_z", "init_eps")
            for k in names:
                a = getattr(draws, k, None)
                keep[k] = None if a is None else np.ascontiguousarray(a, dtype=np.float32)
            d = Draws(*(_fptr(keep[k]) for k in names))
            ins["_draws_keep"] = keep
        ins["draws"] = d
        return ins

    def begin(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, draws=None):
        ins = self._inputs(init_state, mean, cov, x_obs, y_obs, draws)
        self._keep = [ins]
        d = ins["draws"]
        check(self._L.mpcmmd_begin(self._h, COST[cost], int(idx_mpc), _fptr(ins["init_state"]),
                                   _fptr(ins["mean"]), _fptr(ins["cov"]), _fptr(ins["x_obs"]),
                                   _fptr(ins["y_obs"]), float(v_des), None if d is None else C.byref(d)))

    def carla_begin(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws=None):
        """mpcmmd_carla_begin: compute_cem_mmd / compute_cem_cvar / compute_cem_det
        of the CARLA optimizer (carla/optimizer/cem.py:217-790; cost "mmd_opt",
        "cvar", "det"); path: dict of PATH_KEYS."""
        ins = self._inputs(init_state, mean, cov, x_obs, y_obs, draws)
        pth, keep = make_path(path)
        ins["_path"] = (pth, keep)
        self._keep = [ins]
        d = ins["draws"]
        check(self._L.mpcmmd_carla_begin(self._h, COST[cost], int(idx_mpc), _fptr(ins["init_state"]),
                                         _fptr(ins["mean"]), _fptr(ins["cov"]), _fptr(ins["x_obs"]),
                                         _fptr(ins["y_obs"]), float(v_des), C.byref(pth),
                                         None if d is None else C.byref(d)))

    def carla_solve(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws=None, trace=False):
        self.carla_begin(cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, path, draws)
        self.iterate(0, self.cfg.maxiter_cem)
        return self.finish(trace)

    def iterate(self, t_begin, count):
        check(self._L.mpcmmd_iterate(self._h, int(t_begin), int(count)))

    def sync(self):
        check(self._L.mpcmmd_sync(self._h))

    def finish(self, trace=False):
        r = Result()
        beta = np.zeros(max(self.cfg.num_reduced, 1), np.float32)
        r.beta = _fptr(beta)
        steer = np.zeros(100, np.float32)
        vbest = np.zeros(100, np.float32)
        r.steering = _fptr(steer)
        r.v_best = _fptr(vbest)
        T, B = self.cfg.maxiter_cem, self.cfg.num_batch
        tr = None
        if trace:
            tr = dict(elite_proj=np.zeros((T, B), np.int32), elite_obs=np.zeros((T, 20), np.int32),
                      elite_cem=np.zeros((T, 5), np.int32))
            for k, v in tr.items():
                setattr(r, k, v.ctypes.data_as(C.POINTER(C.c_int32)))
        check(self._L.mpcmmd_finish(self._h, C.byref(r)))
        out = dict(cx=np.array(r.cx, np.float32), cy=np.array(r.cy, np.float32),
                   cost_lane=np.float32(r.cost_lane), cost_obs=np.float32(r.cost_obs),
                   sigma=np.float32(r.sigma), res_beta=np.array(r.res_beta, np.float32), beta=beta)
        if self.cfg.variant >= 2:
            out.update(steering=steer, v_best=vbest, mean_param=np.array(r.mean_param, np.float32))
        if tr is not None:
            out.update(tr)
        return out

    def _batch_inputs(self, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des):
        G = len(idx_mpc)
        if G > self.max_configs:
            raise ValueError(f"{G} configurations > max_configs {self.max_configs}")
        f = lambda a, *sh: np.ascontiguousarray(np.broadcast_to(np.asarray(a, np.float32), sh))
        O = self.cfg.num_obs
        ins = dict(idx=np.ascontiguousarray(np.asarray(idx_mpc, np.int64).astype(np.int32)),
                   init=f(init_state, G, 6) if np.ndim(init_state) == 2 else f(np.asarray(init_state).reshape(6), G, 6),
                   mean=f(mean, G, 8) if np.ndim(mean) == 2 else f(np.asarray(mean).reshape(8), G, 8),
                   cov=f(np.asarray(cov, np.float32).reshape(-1, 64), G, 64),
                   xo=f(np.asarray(x_obs, np.float32).reshape(G, O, 100), G, O, 100),
                   yo=f(np.asarray(y_obs, np.float32).reshape(G, O, 100), G, O, 100),
                   vd=f(np.asarray(v_des, np.float32).reshape(-1), G))
        args = (ins["idx"].ctypes.data_as(C.POINTER(C.c_int32)), _fptr(ins["init"]), _fptr(ins["mean"]),
                _fptr(ins["cov"]), _fptr(ins["xo"]), _fptr(ins["yo"]), _fptr(ins["vd"]))
        return G, ins, args

    def begin_batch(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des):
        """mpcmmd_begin_batch (then iterate / finish_batch)."""
        G, ins, args = self._batch_inputs(idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des)
        self._keep = [ins]
        check(self._L.mpcmmd_begin_batch(self._h, G, COST[cost], *args))
        self._G = G

    def finish_batch(self):
        G = self._G
        rs = (Result * G)()
        betas = [np.zeros(max(self.cfg.num_reduced, 1), np.float32) for _ in range(G)]
        for g in range(G):
            rs[g].beta = _fptr(betas[g])
        check(self._L.mpcmmd_finish_batch(self._h, G, rs))
        return [dict(cx=np.array(r.cx, np.float32), cy=np.array(r.cy, np.float32),
                     cost_lane=np.float32(r.cost_lane), cost_obs=np.float32(r.cost_obs), sigma=np.float32(r.sigma),
                     res_beta=np.array(r.res_beta, np.float32), beta=betas[g]) for g, r in enumerate(rs)]

    def solve_batch(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des):
        """mpcmmd_solve_batch: len(idx_mpc) configurations in one batch.
        init_state / mean / cov / v_des may be shared (one value) or per
        configuration; x_obs, y_obs [G, O, 100].  Returns one result dict
        per configuration (the keys of finish())."""
        self.begin_batch(cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des)
        self.iterate(0, self.cfg.maxiter_cem)
        return self.finish_batch()

    def solve(self, cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, draws=None, trace=False):
        self.begin(cost, idx_mpc, init_state, mean, cov, x_obs, y_obs, v_des, draws)
        self.iterate(0, self.cfg.maxiter_cem)
        return self.finish(trace)

    # -- stage access (parity tests) -------------------------------------------
    def buffer_bytes(self, name):
        n = C.c_size_t()
        check(self._L.mpcmmd_buffer_info(self._h, name.encode(), C.byref(n)))
        return n.value

    def read(self, name, dtype=np.float32, shape=None):
        nb = self.buffer_bytes(name)
        out = np.empty(nb // np.dtype(dtype).itemsize, dtype)
        check(self._L.mpcmmd_read(self._h, name.encode(), out.ctypes.data, out.nbytes))
        return out if shape is None else out[: int(np.prod(shape))].reshape(shape)

    def write(self, name, arr):
        arr = np.ascontiguousarray(arr)
        check(self._L.mpcmmd_write(self._h, name.encode(), arr.ctypes.data, arr.nbytes))

    def run_stage(self, stage, t):
        check(self._L.mpcmmd_run_stage(self._h, int(stage), int(t)))

    def info(self, name):
        """mpcmmd_handle_info: the handle's implementation choices ("gen_wave",
        "select_prep", "fused_small", "groups", "capacity")."""
        v = C.c_int64()
        check(self._L.mpcmmd_handle_info(self._h, name.encode(), C.byref(v)))
        return v.value

    # -- streams / profiling -----------------------------------------------------
    def set_stream(self, stream_ptr):
        check(self._L.mpcmmd_set_stream(self._h, C.c_void_p(stream_ptr)))

    def set_graphs(self, enable):
        """mpcmmd_set_graphs: replay whole solves as captured HIP graphs."""
        check(self._L.mpcmmd_set_graphs(self._h, 1 if enable else 0))

    def profile(self, enable):
        check(self._L.mpcmmd_profile(self._h, 1 if enable else 0))

    def kernel_times(self):
        n = 64
        la = (C.c_int32 * n)()
        ms = (C.c_double * n)()
        k = min(n, check(self._L.mpcmmd_kernel_times(self._h, la, ms, n)))
        return {self._L.mpcmmd_kernel_name(i).decode(): (la[i], ms[i]) for i in range(k)}
