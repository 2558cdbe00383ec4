"""ctypes bindings of ``librocket_hip.so`` (C-ABI declared in ``include/rocket_hip.h``).

There is no CPU fallback: if the HIP library is missing, every entry point of the
package raises.  ``torch`` is imported first so that the process has ONE HIP
runtime (torch's bundled ``libamdhip64.so`` carries the same soname,
``libamdhip64.so.7``, as the one ``librocket_hip.so`` links against; the dynamic
loader reuses the already-loaded copy).
"""
import ctypes
import os
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RR_LIB_PATH") or os.path.join(HERE, "librocket_hip.so")  # override: diagnostics only
HEADER = os.path.join(os.path.dirname(HERE), "include", "rocket_hip.h")

ABI_VERSION = 12

RR_OK, RR_EINVAL, RR_EHIP, RR_ENOMEM = 0, -1, -2, -3
RR_MODEL_3DOF, RR_MODEL_6DOF = 3, 6
RR_INT_RK4, RR_INT_EULER, RR_INT_DOPRI5 = 0, 1, 2
RR_FLAG_AUTO_RESET = 0x1
RR_FLAG_EPISODE_STATS = 0x2
RR_FLAG_REWARD_ANNEALING = 0x4
RR_FLAG_ACTION_SOA = 0x8
RR_FLAG_SCIPY_H0_CLAMP = 0x10
RR_FLAG_HOST_STATE = 0x20
RR_MAX_STATE = 14
RR_POLICY_FP32, RR_POLICY_BF16, RR_POLICY_FP16X3 = 0, 1, 2

_d3 = ctypes.c_double * 3
_f14 = ctypes.c_float * RR_MAX_STATE
_d14 = ctypes.c_double * RR_MAX_STATE


class RrParams(ctypes.Structure):
    """Mirror of ``rr_params`` (include/rocket_hip.h)."""

    _fields_ = [
        ("model", ctypes.c_int32),
        ("integrator", ctypes.c_int32),
        ("max_episode_steps", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("dt", ctypes.c_double),
        ("ic_low", _f14),
        ("ic_high", _f14),
        ("normalizer", _d14),
        ("bounds_low", _d3),
        ("bounds_high", _d3),
        ("max_gimbal", ctypes.c_double),
        ("max_thrust", ctypes.c_double),
        ("alfa", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("eta", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("delta", ctypes.c_double),
        ("kappa", ctypes.c_double),
        ("xi", ctypes.c_double),
        ("waypoint", ctypes.c_double),
        ("landing_radius", ctypes.c_double),
        ("max_velocity", ctypes.c_double),
        ("att_limit", _d3),
        ("land_att_limit", _d3),
        ("omega_lim", _d3),
    ]


class RrBuffers(ctypes.Structure):
    """Mirror of ``rr_buffers``."""

    _fields_ = [
        ("state", ctypes.c_void_p),
        ("v0", ctypes.c_void_p),
        ("elapsed", ctypes.c_void_p),
        ("ep_return", ctypes.c_void_p),
        ("done_bits", ctypes.c_void_p),
        ("terminal_obs", ctypes.c_void_p),
        ("terminal_return", ctypes.c_void_p),
        ("terminal_len", ctypes.c_void_p),
    ]


# symbol -> (restype, argtypes); the test suite checks this against include/rocket_hip.h
_P = ctypes.c_void_p
SIGNATURES = {
    "rr_abi_version": (ctypes.c_int, []),
    "rr_last_error": (ctypes.c_char_p, []),
    "rr_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(RrParams), ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_int]),
    "rr_destroy": (ctypes.c_int, [_P]),
    "rr_num_envs": (ctypes.c_int64, [_P]),
    "rr_state_dim": (ctypes.c_int, [_P]),
    "rr_action_dim": (ctypes.c_int, [_P]),
    "rr_seed": (ctypes.c_int, [_P, ctypes.c_uint64, _P]),
    "rr_reset": (ctypes.c_int, [_P, _P, _P, _P]),
    "rr_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "rr_step_rows": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "rr_step_repeat": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.c_int64, _P, _P, _P, _P, _P, _P]),
    "rr_set_state": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "rr_get_state": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "rr_set_state64": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "rr_get_state64": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "rr_counter_bits": (ctypes.c_int, [_P]),
    "rr_get_aux": (ctypes.c_int, [_P, _P, _P, _P]),
    "rr_set_aux": (ctypes.c_int, [_P, _P, _P, _P]),
    "rr_get_buffers": (ctypes.c_int, [_P, ctypes.POINTER(RrBuffers)]),
    "rr_host_alloc": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int64]),
    "rr_host_free": (ctypes.c_int, [_P]),
    "rr_fetch_done": (ctypes.c_int64, [_P, ctypes.c_int64, _P, _P, _P, _P, _P]),
    "rr_copy_terminal": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "rr_gather_rows": (ctypes.c_int64, [_P, _P, _P, _P, _P, _P, ctypes.c_int64, _P, _P, _P, _P, _P, _P]),
    "rr_policy_layout": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    "rr_policy_pack": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P]),
    "rr_policy_act": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, _P,
                                     ctypes.c_uint64, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P,
                                     ctypes.c_float, _P, _P, _P, _P]),
    "rr_policy_bootstrap": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _P, _P, _P,
                                           ctypes.c_float, _P, _P, _P, _P]),
    "rr_rollout_step": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_uint64, _P, ctypes.c_int, ctypes.c_float,
                                       _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rr_rollout_collect": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_uint64, _P, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_float] + [_P] * 17),
    "rr_gae": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, _P, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, _P,
                              _P, _P]),
    "rr_clip_adam_workspace_size": (ctypes.c_int, [ctypes.c_int64, _P]),
    "rr_clip_adam": (ctypes.c_int, [ctypes.c_int, _P, _P, _P, _P, _P, _P, ctypes.c_float, _P, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_float, _P, ctypes.c_int64, _P]),
    "rr_ppo_workspace_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _P]),
    "rr_ppo_grad": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int64,
                                   ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, ctypes.c_int64, _P]),
    "rr_ppo_update_workspace_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _P]),
    "rr_ppo_update": (ctypes.c_int, [ctypes.c_int, ctypes.c_int] + [_P] * 11 + [ctypes.c_int64, _P, ctypes.c_int64,
                                     ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_float, _P, ctypes.c_uint32, _P,
                                     ctypes.c_int64, _P]),
}

_LIB = None


class RocketHipError(RuntimeError):
    pass


def load(require_torch=True):
    """Load librocket_hip.so (raises if it has not been built: no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if require_torch:
        import torch  # noqa: F401  (one HIP runtime per process, see module doc)
    if not os.path.exists(LIB_PATH):
        raise RocketHipError(
            "librocket_hip.so is not built (expected at %s). Build it with "
            "`python -m rl_rocket_amd.build` (hipcc, gfx950). There is no CPU fallback." % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    override = bool(os.environ.get("RR_LIB_PATH"))
    missing = []
    for name, (res, args) in SIGNATURES.items():
        if override and not hasattr(lib, name):
            missing.append(name)  # an older diagnostic build (tools/ab_kernel.py) may lack newer entry points
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    abi = lib.rr_abi_version()
    if abi != ABI_VERSION:
        if not override:
            raise RocketHipError("librocket_hip.so ABI %d != expected %d" % (abi, ABI_VERSION))
        # diagnostic builds may be older: say so now rather than as a wrong counter decoding later
        warnings.warn("RR_LIB_PATH=%s has ABI %d, this package expects %d%s" % (
            LIB_PATH, abi, ABI_VERSION, (" (missing: %s)" % ", ".join(missing)) if missing else ""),
            RuntimeWarning, stacklevel=2)
    for name in missing:  # a call of a missing entry point raises a clear error at the call site
        setattr(lib, name, _missing(name))
    _LIB = lib
    return lib


def _missing(name):
    def call(*a, **k):
        raise RocketHipError("%s is not exported by the RR_LIB_PATH library %s (ABI mismatch)" % (name, LIB_PATH))
    return call


def check(rc, what="rocket_hip"):
    if rc < 0:
        msg = load().rr_last_error()
        raise RocketHipError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))
    return rc
