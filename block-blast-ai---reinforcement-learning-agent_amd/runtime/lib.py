"""ctypes binding of ``include/bbvec.h`` (libbbvec.so, gfx950).

This is the only way the product reaches its kernels.  There is no CPU
fallback: if the library is missing or no HIP device is present, the first
call raises ``BBNativeError`` with the reason.

``load_host()`` binds the env half of the same ABI from libbbvec_host.so, the
host backend (csrc/bb_host.cpp) that ``DeviceEnvBatch(device="cpu")`` selects
explicitly; nothing falls back to it.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("BBVEC_LIB", os.path.join(PKG_DIR, "libbbvec.so"))
HOST_LIB_PATH = os.path.join(PKG_DIR, "libbbvec_host.so")

BB_OK = 0
BB_ACTIONS = 192
BB_NUM_PIECES = 37


class BBNativeError(RuntimeError):
    """Raised when the HIP library is unavailable or a C-ABI call fails."""


class RewardCfg(C.Structure):
    _fields_ = [
        ("line_clear_base", C.c_double),
        ("block_placed", C.c_double),
        ("game_over_penalty", C.c_double),
        ("hole_penalty", C.c_double),
        ("center_bonus", C.c_double),
        ("combo_multiplier_bonus", C.c_double),
        ("survival_bonus", C.c_double),
    ]


class Info(C.Structure):
    _fields_ = [
        ("score", C.c_int64),
        ("score_gained", C.c_int64),
        ("term_board", C.c_uint64),
        ("moves", C.c_int32),
        ("lines", C.c_int32),
        ("max_combo", C.c_int32),
        ("blocks", C.c_int32),
        ("term_hand", C.c_uint32),
        ("holes", C.c_uint8),
        ("filled", C.c_uint8),
        ("flags", C.c_uint8),
        ("last_blocks", C.c_uint8),
        ("last_lines", C.c_uint8),
        ("last_cm", C.c_uint8),
        ("pad", C.c_uint8 * 2),
    ]


ABI_VERSION = 8  # include/bbvec.h BB_ABI_VERSION
INFO_BYTES = C.sizeof(Info)  # 56, matches sizeof(bb_info)


class StepOut(C.Structure):
    _fields_ = [
        ("reward", C.c_void_p),
        ("terminated", C.c_void_p),
        ("reward_f64", C.c_void_p),
        ("mask", C.c_void_p),
        ("lines", C.c_void_p),
        ("info", C.c_void_p),
        ("next_action", C.c_void_p),
        ("policy_seed", C.c_uint64),
        ("policy_step", C.c_uint64),
        ("env_offset", C.c_uint64),
        ("final_score", C.c_void_p),
        ("final_moves", C.c_void_p),
    ]


class RolloutOut(C.Structure):
    _fields_ = [
        ("reward", C.c_void_p),
        ("terminated", C.c_void_p),
        ("lines", C.c_void_p),
        ("actions", C.c_void_p),
        ("mask", C.c_void_p),
        ("next_action", C.c_void_p),
        ("policy_seed", C.c_uint64),
        ("policy_step0", C.c_uint64),
        ("env_offset", C.c_uint64),
    ]


class StateView(C.Structure):
    _fields_ = [
        ("board", C.c_void_p),
        ("hand", C.c_void_p),
        ("score", C.c_void_p),
        ("combo", C.c_void_p),
        ("max_combo", C.c_void_p),
        ("moves", C.c_void_p),
        ("lines", C.c_void_p),
        ("blocks", C.c_void_p),
        ("prev_holes", C.c_void_p),
        ("prev_center", C.c_void_p),
        ("rng", C.c_void_p),
    ]


_P = C.c_void_p
_I32 = C.c_int32
_U64 = C.c_uint64
_F = C.c_float

# name -> (restype, argtypes); exactly the entry points of include/bbvec.h
SIGNATURES = {
    "bb_abi_version": (C.c_int, []),
    "bb_build_id": (C.c_char_p, []),
    "bb_create": (C.c_int, [_I32, _I32, C.POINTER(RewardCfg), _I32, C.POINTER(_P)]),
    "bb_destroy": (None, [_P]),
    "bb_last_error": (C.c_char_p, [_P]),
    "bb_num_envs": (_I32, [_P]),
    "bb_pcg64_seed": (C.c_int, [_U64, C.POINTER(_U64)]),
    "bb_seed": (C.c_int, [_P, _P, _P, _P]),
    "bb_reset": (C.c_int, [_P, _P, _P]),
    "bb_step": (C.c_int, [_P, _P, C.POINTER(StepOut), _P]),
    "bb_rollout": (C.c_int, [_P, _I32, _P, C.POINTER(RolloutOut), _P]),
    "bb_sync": (C.c_int, [_P, _P]),
    "bb_obs": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "bb_device_ptrs": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P)]),
    "bb_snapshot": (C.c_int, [_P, _P, _P, _P, _P]),
    "bb_get_state": (C.c_int, [_P, C.POINTER(StateView)]),
    "bb_set_state": (C.c_int, [_P, C.POINTER(StateView)]),
    "bb_debug_counters": (C.c_int, [_P, _P]),
    "bb_random_actions": (C.c_int, [_P, _I32, _U64, _U64, _U64, _P, _P]),
    "bb_masked_sample": (C.c_int, [_P, _P, _I32, _P, _U64, _U64, _U64, _I32, _P, _P, _P, _P, _P]),
    "bb_masked_sample_dstep": (C.c_int, [_P, _P, _I32, _U64, _P, _U64, _U64, _I32, _P, _P, _P, _P]),
    "bb_gae": (C.c_int, [_P, _P, _P, _P, _I32, _I32, _F, _F, _P, _P, _P]),
    "bb_gather_obs": (C.c_int, [_P, _P, _P, _P, _I32, _P, _P, _P]),
    "bb_bn_workspace_bytes": (C.c_int64, [_I32, _I32, _I32, _I32, _I32]),
    "bb_bn_forward": (C.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _F, _I32, _P, _P, _P, _P, _P, _F, _P, _P,
                                _P]),
    "bb_bn_forward_res": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _F, _I32, _P, _P, _P, _P, _P,
                                    _F, _P, _P, _P]),
    "bb_bn_backward_part": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P,
                                      _P, _P, _I32, _I32, _I32, _I32, _P, _P, _I32, _P]),
    "bb_bn_forward_part": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _F, _I32, _P, _P, _P, _P, _P,
                                     _F, _P, _P, _P, _I32, _P]),
    "bb_bn_backward": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P,
                                 _P]),
    "bb_bn_backward_red": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P,
                                     _P, _I32, _I32, _I32, _I32, _P, _P]),
    "bb_bn_backward_res": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                     _P, _P, _I32, _I32, _I32, _I32, _P, _P]),
    "bb_conv3x3_workspace_bytes": (C.c_int64, [_I32, _I32, _I32]),
    "bb_conv3x3_prep": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "bb_conv3x3_prep_multi": (C.c_int, [_I32, _P, _P, _P, _P, _P, _P, _P]),
    "bb_conv3x3_forward": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "bb_conv3x3_forward_add": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P, _P]),
    "bb_conv3x3_stats_blocks": (C.c_int32, [_I32, _I32]),
    "bb_conv3x3_forward_stats": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P, _P]),
    "bb_conv3x3_forward_bstats": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _I32, _P, _P]),
    "bb_conv3x3_wgrad": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _I32, _P, _P]),
    "bb_conv3x3_wgrad_chunks": (C.c_int32, [_I32, _I32, _I32]),
    "bb_conv3x3_wgrad_partial": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "bb_conv3x3_wgrad_reduce": (C.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P]),
    "bb_conv3x3_f32_prep": (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "bb_conv3x3_f32_forward": (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    "bb_linear_f32": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _P, _P]),
    "bb_ppo_loss_workspace_bytes": (C.c_int64, [_I32]),
    "bb_ppo_loss_forward": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _F, _F, _F, _P, _P, _P, _P, _P]),
    "bb_ppo_loss_backward": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _F, _F, _F, _P, _P, _P, _P]),
    "bb_ppo_loss_forward_bf16": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _F, _F, _F, _P, _P, _P, _P, _P]),
    "bb_ppo_loss_fused": (C.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _I32, _F, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P]),
    "bb_ppo_loss_backward_bf16": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _F, _F, _F, _P, _P, _P, _P]),
    "bb_adam_clip_workspace_bytes": (C.c_int64, [_I32, _P]),
    "bb_adam_clip_step": (C.c_int, [_I32, _P, _P, _P, _P, _P, _P, C.c_double, C.c_double, C.c_double, C.c_double, _F,
                                    _P, _P, _P]),
    "bb_cast_multi": (C.c_int, [_I32, _I32, _P, _P, _P, _P, _P, _P]),
    "bb_dropout_forward": (C.c_int, [_P, C.c_int64, _F, _P, _P]),
    "bb_conv_in_wgrad_workspace_bytes": (C.c_int64, [_I32]),
    "bb_conv_in_forward": (C.c_int, [_P, _I32, _P, _I32, _I32, _P, _P]),
    "bb_conv_in_wgrad": (C.c_int, [_P, _I32, _P, _I32, _P, _I32, _P, _P]),
    "bb_conv_in_forward_prep": (C.c_int, [_P, _I32, _P, _I32, _I32, _P, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "bb_linear_n1_workspace_bytes": (C.c_int64, [_I32, _I32]),
    "bb_linear_n1_counters": (C.c_int32, [_I32]),
    "bb_linear_n1_forward": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _P, _P]),
    "bb_linear_n1_backward": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "bb_linear_wgrad_workspace_bytes": (C.c_int64, [_I32, _I32, _I32]),
    "bb_linear_wgrad_counters": (C.c_int32, [_I32, _I32]),
    "bb_linear_wgrad": (C.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P]),
    "bb_linear_bgrad_workspace_bytes": (C.c_int64, [_I32, _I32]),
    "bb_linear_bgrad_counters": (C.c_int32, [_I32]),
    "bb_linear_bgrad": (C.c_int, [_P, _P, _I32, _I32, _F, _P, _P, _P, _P, _P]),
    "bb_linear_bgrad2": (C.c_int, [_P, _P, _I32, _P, _I32, _I32, _F, _P, _P, _P, _P, _P]),
}

# the env entry points, which the host backend (libbbvec_host.so) exports too
HOST_SYMBOLS = ("bb_abi_version", "bb_build_id", "bb_create", "bb_destroy", "bb_last_error", "bb_num_envs", "bb_pcg64_seed",
                "bb_seed", "bb_reset", "bb_step", "bb_rollout", "bb_sync", "bb_obs", "bb_device_ptrs", "bb_snapshot",
                "bb_get_state", "bb_set_state", "bb_random_actions")

_lib = None
_host = None
_lock = threading.Lock()


def load(path: str | None = None):
    """Load libbbvec.so (once) and bind every symbol of bbvec.h."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise BBNativeError(
                f"HIP library not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
            )
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError == missing export
            fn.restype = res
            fn.argtypes = args
        v = lib.bb_abi_version()
        if v != ABI_VERSION:
            raise BBNativeError(f"libbbvec ABI version mismatch ({v}, expected {ABI_VERSION})")
        if path is None and "BBVEC_LIB" not in os.environ:
            _check_build_id(lib, p, host=False)
        if path is None:
            _lib = lib
        return lib


def _check_build_id(lib, p: str, host: bool) -> None:
    """Refuse a library that was not built from the sources beside it (bb_build_id against
    runtime/build.py's hash of csrc/, include/bbvec.h and the flags).  Explicit variant builds
    (load(path), BBVEC_LIB) are diagnostics and skip the check."""
    from . import build as B

    want = B.host_source_id() if host else B.source_id()
    have = lib.bb_build_id().decode()
    if have != want:
        raise BBNativeError(
            f"{os.path.basename(p)} was built from other sources (build id {have}, these sources {want}); "
            "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")


def build_id(host: bool = False) -> str:
    """The loaded library's build id (bb_build_id)."""
    return (load_host() if host else load()).bb_build_id().decode()


def load_host():
    """Load libbbvec_host.so (once), the host backend of the env entry points."""
    global _host
    with _lock:
        if _host is not None:
            return _host
        if not os.path.exists(HOST_LIB_PATH):
            raise BBNativeError(f"host backend not found at {HOST_LIB_PATH}; build it with "
                                "`python -c 'import __graft_entry__ as g; g.build()'`")
        lib = C.CDLL(HOST_LIB_PATH)
        for name in HOST_SYMBOLS:
            res, args = SIGNATURES[name]
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.bb_abi_version() != ABI_VERSION:
            raise BBNativeError("libbbvec_host ABI version mismatch")
        _check_build_id(lib, HOST_LIB_PATH, host=True)
        _host = lib
        return lib


def last_error(handle=None, lib=None) -> str:
    msg = (lib or load()).bb_last_error(handle)
    return msg.decode() if msg else ""


def check(rc: int, what: str, handle=None, lib=None) -> None:
    if rc != BB_OK:
        raise BBNativeError(f"{what} failed ({rc}): {last_error(handle, lib)}")


def pcg64_seed(seed: int):
    """numpy-exact default_rng(seed) PCG64 words {state_hi, state_lo, inc_hi, inc_lo}."""
    out = (_U64 * 4)()
    check(load().bb_pcg64_seed(seed, out), "bb_pcg64_seed")
    return [int(x) for x in out]


def reward_cfg(rewards: dict) -> RewardCfg:
    cfg = RewardCfg()
    for name, _ in RewardCfg._fields_:
        setattr(cfg, name, float(rewards[name]))
    return cfg
