"""ctypes binding of libmadigan_hip.so (the C ABI in include/madigan_amd.h).

The shared library is built in-tree by ``madigan_amd.build`` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library or a GPU is
missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmadigan_hip.so")
MAX_ASSETS = 64
ABI_VERSION = 10
SRC_PARAMS = 64
AUX_WIDTH = 24
MAX_NSTEP = 256

# status codes -> the reference's exception types (DataTypes.h:36-46, pybind11)
OK, ERR_CONFIG, ERR_INDEX, ERR_LENGTH, ERR_DEVICE, ERR_ARG = range(6)

GREEN, INSUFF_MARGIN, MARGIN_CALL, BLOWN_OUT = range(4)
(SRC_EXTERNAL, SRC_SINE, SRC_OU, SRC_TRENDOU, SRC_REPLAY, SRC_SIMPLETREND, SRC_TRENDYOU, SRC_GAUSSIAN,
 SRC_SAWTOOTH, SRC_TRIANGLE, SRC_OUPAIR, SRC_SINEADDER, SRC_SINEDYNAMIC, SRC_SINEDYNTREND) = range(14)
(SHAPER_NONE, SHAPER_DSR, SHAPER_DDR, SHAPER_PPC, SHAPER_SHARPE, SHAPER_SORTINO_A,
 SHAPER_SORTINO_B) = range(7)
NSTEP_POP_EXACT, NSTEP_POP_RUNNING = 0, 1  # mgn_config.nstep_pop (ABI 9)
REWARD_ENV_LOG, REWARD_AGENT_SUM, REWARD_AGENT_PER_ASSET = range(3)
(NORM_NONE, NORM_LOG, NORM_LOOKBACK, NORM_STANDARD_NORMAL, NORM_LOOKBACK_LOG,
 NORM_LOG_STANDARD_NORMAL) = range(6)
RING_PLAIN, RING_PAIR_RATIO = range(2)
STEP_NONE, STEP_UNITS, STEP_SINGLE = range(3)
SCHED_AUTO, SCHED_SINGLE, SCHED_DUO, SCHED_TRIO = range(4)
OP_BROKER_UNITS, OP_BROKER_SINGLE, OP_BROKER_CLOSE, OP_PORT_TXN, OP_PORT_CLOSE, OP_CHECK_ORDER = range(6)


class MadiganError(RuntimeError):
    """HIP runtime failure inside the extension."""


class AssetSource(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad_", C.c_int32), ("p", C.c_double * SRC_PARAMS)]


class Config(C.Structure):
    _fields_ = [
        ("n_envs", C.c_int32), ("n_assets", C.c_int32), ("env_offset", C.c_int64),
        ("seed", C.c_uint64), ("init_cash", C.c_double), ("required_margin", C.c_double),
        ("maintenance_margin", C.c_double), ("slippage_rel", C.c_double),
        ("slippage_abs", C.c_double), ("tc_rel", C.c_double), ("tc_abs", C.c_double),
        ("shaper", C.c_int32), ("reward_mode", C.c_int32), ("adaptation_rate", C.c_double),
        ("cosine_temp", C.c_double), ("desired_portfolio", C.c_double * (MAX_ASSETS + 1)),
        ("window", C.c_int32), ("norm_type", C.c_int32), ("auto_reset", C.c_int32),
        ("action_atoms", C.c_int32), ("unit_size", C.c_double),
        ("nstep", C.c_int32), ("nstep_pop", C.c_int32), ("discount", C.c_double),
        ("n_feats", C.c_int32), ("pad3_", C.c_int32), ("sortino_exp", C.c_double),
        ("aux", C.c_int32), ("pad4_", C.c_int32),
    ]


TRAJ_FIELDS = ("reward", "agent_reward", "shaped", "done", "obs_price", "obs_port", "timestamp",
               "tprice", "tunits", "tcost", "risk", "margin_call", "n_shaped", "data_end")


class Traj(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in TRAJ_FIELDS]


VIEW_PTR_FIELDS = ("ledger", "mean_entry", "borrowed", "prices", "sine_x", "ou_mean", "trend_dy",
                   "trend_len", "trend_flags", "cash", "timestamp", "shaper_a", "shaper_b",
                   "ep_stats", "episode_stats", "ext_prices", "units", "asset_idx", "ring",
                   "ring_ts", "ring_head", "ring_len", "win_price", "win_port", "win_ts",
                   "reset_mask", "nstep_ring", "nstep_len", "nstep_head", "replay_cursor",
                   "aux", "draw_skip")


class Views(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in VIEW_PTR_FIELDS] + [
        ("out", Traj), ("n_envs", C.c_int32), ("n_assets", C.c_int32), ("window", C.c_int32),
        ("reward_dim", C.c_int32), ("nstep", C.c_int32), ("n_feats", C.c_int32)]


class ReplayTape(C.Structure):
    _fields_ = [("price", C.c_void_p), ("feats", C.c_void_p), ("ts", C.c_void_p),
                ("data_end", C.c_void_p), ("rows", C.c_int64), ("stride", C.c_int64)]


class HistView(C.Structure):  # mgn_hist_view
    _fields_ = [("hist", C.c_void_p), ("hist_ts", C.c_void_p), ("hend", C.c_void_p), ("hlen", C.c_void_p),
                ("rows", C.c_int32), ("cols", C.c_int32), ("k_steps", C.c_int32), ("window", C.c_int32),
                ("n_feats", C.c_int32), ("pad_", C.c_int32)]


class Ring(C.Structure):
    _fields_ = [("n_envs", C.c_int32), ("n_price", C.c_int32), ("n_port", C.c_int32),
                ("window", C.c_int32), ("norm_type", C.c_int32), ("transform", C.c_int32),
                ("ring", C.c_void_p), ("ring_ts", C.c_void_p), ("head", C.c_void_p),
                ("len", C.c_void_p), ("out_stride", C.c_int32), ("out_offset", C.c_int32)]


SYMBOLS = {
    # name: (restype, argtypes)
    "mgn_abi_version": (C.c_int, []),
    "mgn_arena_bytes": (C.c_size_t, [C.POINTER(Config)]),
    "mgn_create": (C.c_int, [C.POINTER(Config), C.POINTER(AssetSource), C.c_void_p, C.c_void_p,
                             C.c_size_t, C.POINTER(C.c_void_p)]),
    "mgn_destroy": (C.c_int, [C.c_void_p]),
    "mgn_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_get_views": (C.c_int, [C.c_void_p, C.POINTER(Views)]),
    "mgn_reset": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "mgn_rollout": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(Traj)]),
    "mgn_rollout_units": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(Traj)]),
    "mgn_set_prices": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_set_sources": (C.c_int, [C.c_void_p, C.POINTER(AssetSource), C.c_void_p]),
    "mgn_stats_allgather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "mgn_state_bytes": (C.c_size_t, [C.c_void_p]),
    "mgn_save_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "mgn_load_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "mgn_attach_replay": (C.c_int, [C.c_void_p, C.POINTER(ReplayTape)]),
    "mgn_window_push": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mgn_window_clear": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_window": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mgn_rollout_hist": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(Traj)]),
    "mgn_window_hist": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mgn_set_window_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_set_timing": (C.c_int, [C.c_void_p, C.c_int32]),
    "mgn_get_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "mgn_rollout_window": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(Traj),
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]),
    "mgn_generate_actions": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_uint64]),
    "mgn_valuation": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mgn_set_broker": (C.c_int, [C.c_void_p] + [C.c_double] * 6),
    "mgn_ring_push": (C.c_int, [C.POINTER(Ring), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mgn_ring_clear": (C.c_int, [C.POINTER(Ring), C.c_void_p, C.c_void_p]),
    "mgn_ring_gather": (C.c_int, [C.POINTER(Ring), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mgn_feat_diff": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]),
    "mgn_set_layout": (C.c_int, [C.c_void_p, C.c_int32]),
    "mgn_get_layout": (C.c_int, [C.c_void_p]),
    "mgn_set_schedule": (C.c_int, [C.c_void_p, C.c_int32]),
    "mgn_get_schedule": (C.c_int, [C.c_void_p]),
    "mgn_window_hist_view": (C.c_int, [C.c_void_p, C.POINTER(HistView)]),
    "mgn_ledger_op": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.POINTER(Traj)]),
    "mgn_bandwidth_probe": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32, C.c_void_p,
                                      C.POINTER(C.c_double)]),
    "mgn_synchronize": (C.c_int, [C.c_void_p]),
    "mgn_synchronize_spin": (C.c_int, [C.c_void_p]),
    "mgn_last_error": (C.c_char_p, [C.c_void_p]),
    "mgn_global_error": (C.c_char_p, []),
}

# exported by the diagnostic builds only (timing ablations; never in the product ABI)
DIAG_SYMBOLS = {
    "mgn_set_ablation": (C.c_int, [C.c_void_p, C.c_int32]),
}

_lib = None
_hip = None


def hip():
    """The process's HIP runtime (the instance torch loaded), for the few
    stream-ordered copies the host wrappers issue directly."""
    global _hip
    if _hip is None:
        h = C.CDLL("libamdhip64.so")
        h.hipMemcpyAsync.restype = C.c_int
        h.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        h.hipStreamSynchronize.restype = C.c_int
        h.hipStreamSynchronize.argtypes = [C.c_void_p]
        h.hipPointerGetAttributes.restype = C.c_int
        h.hipPointerGetAttributes.argtypes = [C.c_void_p, C.c_void_p]
        _hip = h
    return _hip


class _PtrAttr(C.Structure):  # hipPointerAttribute_t (hip_runtime_api.h)
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


def device_view(host_ptr: int) -> int:
    """The device address of pinned host memory the kernels may read in place
    (hipHostMalloc memory is mapped into the device address space), or 0 when
    the runtime reports none."""
    a = _PtrAttr()
    if hip().hipPointerGetAttributes(C.byref(a), C.c_void_p(host_ptr)) != 0:
        return 0
    return int(a.devicePointer or 0)


def load(path: str = ""):
    """Load the HIP extension (no GPU needed to load it).  MADIGAN_LIB_PATH
    selects a diagnostic build of the same sources (tools/build_variant.py)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MADIGAN_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -m madigan_amd.build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = C.CDLL(path)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # diagnostic builds only (tools/build_variant.py defines MGN_DIAG)
    for name, (res, args) in DIAG_SYMBOLS.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype = res
            fn.argtypes = args
    if lib.mgn_abi_version() != ABI_VERSION:
        raise ImportError("libmadigan_hip.so ABI version mismatch; rebuild the extension")
    _lib = lib
    return lib


_pycall = None


def pycall():
    """The CPython binding of mgn_rollout (`_mgn_pycall`, csrc/mgn_pycall.c,
    linked against the in-tree libmadigan_hip.so), or None when the loaded
    library is another build (MADIGAN_LIB_PATH) or the binding is not built:
    the launcher then calls through ctypes."""
    global _pycall
    if _pycall is None:
        lib = load()
        mod = False
        if os.path.realpath(lib._name) == os.path.realpath(LIB_PATH):
            try:
                from . import _mgn_pycall as mod
            except ImportError:
                mod = False
        _pycall = mod
    return _pycall or None


def check(status: int, handle=None) -> None:
    if status == OK:
        return
    lib = load()
    msg = (lib.mgn_last_error(handle) if handle else lib.mgn_global_error()) or b""
    msg = msg.decode(errors="replace")
    if status == ERR_CONFIG:
        raise RuntimeError(msg)
    if status == ERR_INDEX:
        raise IndexError(msg)
    if status == ERR_LENGTH:
        raise ValueError(msg)
    if status == ERR_ARG:
        raise TypeError(msg)
    raise MadiganError(msg)
