"""ctypes binding of libdmt.so (include/dmt.h).

The product path has no CPU fallback: if the HIP library is missing, importing this
module raises; if no GPU is present, ``dmt_create`` fails with DMT_ERR_HIP.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# DMT_LIB_PATH: alternative build of the same library (kernel-variant experiments)
LIB_PATH = os.environ.get("DMT_LIB_PATH") or os.path.join(HERE, "libdmt.so")
INCLUDE_H = os.path.join(os.path.dirname(HERE), "include", "dmt.h")

# ---- constants (mirror include/dmt.h) ----
OK, ERR_INVALID, ERR_HIP, ERR_OOM, ERR_STATE, ERR_COMM = 0, 1, 2, 3, 4, 5
MODEL_OU, MODEL_FHN, MODEL_LORENZ = 0, 1, 2
F64, F32 = 0, 1
MAP_AUTO, MAP_LANE, MAP_WAVE = 0, 1, 2
U, UPROP = 0, 1
PATH_X, PATH_W, PATH_DW = 0, 1, 2  # dmt_download_paths `what`
LAW_PP, LAW_PPB = 0, 1
SWAP_XX, SWAP_WW, SWAP_PP, SWAP_LL = 1, 2, 4, 8
BLK_LL, BLK_LLPROP, BLK_LL_HIST, BLK_LLPROP_HIST, BLK_ACC_HIST = 0, 1, 2, 3, 4
K_DRAW, K_ACCEPT, K_PATHLL, K_RECOMPUTE, K_REDUCE = 0, 1, 2, 3, 4
# device random streams (include/dmt.h): salt = RNG_AUTO draws from the handle's counter
RNG_AUTO = 0xFFFFFFFF
SALT_LIMIT = 0x40000000
LAW_STRIDE = 64
LAW_AUXTD = 15  # DMT_LAW_AUXTD: time-dependent auxiliary law (dmt_upload_aux)
LAW_GSTALE = 14  # DMT_LAW_GSTALE: u°'s guiding term left stale by critical_change = false
LAW_THETA, LAW_SIGMA, LAW_A, LAW_BT, LAW_BETA, LAW_DA, LAW_C0, LAW_TRACE = 0, 16, 25, 31, 40, 43, 49, 50
LAW_SIGINV = 51
LAW_ANCHOR = 60
LAW_AUXLIN = 63
# set_proposal_law! parameter names (include/dmt.h DMT_PAR_*)
# (ASCII and DiffusionDefinition's own symbols, e.g. :γ)
PAR_FHN = {"eps": 0, "s": 1, "gamma": 2, "beta": 3, "sigma": 4, "ϵ": 0, "γ": 2, "β": 3, "σ": 4}
PAR_LORENZ = {"s": 0, "r": 1, "beta": 2, "β": 2}

# exported symbols (checked against include/dmt.h by tests/test_abi.py)
SYMBOLS = [
    "dmt_create", "dmt_destroy", "dmt_upload_grid", "dmt_upload_law", "dmt_set_paths",
    "dmt_download_paths", "dmt_draw_unit", "dmt_create_layout", "dmt_layout_size",
    "dmt_draw_proposal", "dmt_accept_reject", "dmt_loglikhd", "dmt_recompute_path", "dmt_find_W_for_X", "dmt_upload_obs", "dmt_set_obs",
    "dmt_recompute_guiding_term", "dmt_set_proposal_law", "dmt_download_law", "dmt_swap",
    "dmt_save_ll", "dmt_set_accepted", "dmt_get_block_state", "dmt_set_block_state",
    "dmt_fetch_ll", "dmt_mcmc_step", "dmt_mcmc_run", "dmt_guiding_linear", "dmt_guiding_linear_td", "dmt_upload_aux", "dmt_comm_unique_id", "dmt_comm_init", "dmt_set_shard", "dmt_sync",
    "dmt_set_timing", "dmt_get_timing", "dmt_memory_bytes", "dmt_debug_philox", "dmt_recent_kernels",
    "dmt_debug_normals", "dmt_last_error", "dmt_version", "dmt_snapshot_reserve",
    "dmt_snapshot_take", "dmt_snapshot_download", "dmt_snapshot_write", "dmt_set_ll",
    "dmt_fetch_ll_local", "dmt_comm_size", "dmt_rng_counter", "dmt_set_rng_counter",
    "dmt_set_run_snapshots", "dmt_mcmc_step_local", "dmt_mcmc_run_local", "dmt_draw_success",
    "dmt_rng_state", "dmt_set_rng_state", "dmt_combine_rank_partials",
    "dmt_set_service", "dmt_service_stats", "dmt_set_proposal_law_cc", "dmt_upload_aux_a",
    "dmt_guiding_linear_tda",
]


class DMTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libdmt error {code}: {msg}")
        self.code = code


class dmt_model(C.Structure):
    _fields_ = [("model", C.c_int32), ("precision", C.c_int32), ("d", C.c_int32), ("m", C.c_int32)]


class dmt_structure(C.Structure):
    _fields_ = [("n_recordings", C.c_int64), ("n_segments", C.POINTER(C.c_int32)),
                ("n_points", C.POINTER(C.c_int32))]


class dmt_config(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("device", C.c_int32), ("grid_shared", C.c_int32),
                ("mapping", C.c_int32)]


if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
        "(make -C diffusionmcmctools.jl_amd/csrc). There is no CPU fallback.")

lib = C.CDLL(LIB_PATH)

_P = C.c_void_p
_pd = C.POINTER(C.c_double)
_pu8 = C.POINTER(C.c_uint8)
_pi32 = C.POINTER(C.c_int32)
_pi64 = C.POINTER(C.c_int64)
_pu32 = C.POINTER(C.c_uint32)
_i32, _i64, _u32, _u64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64

_SIGS = {
    "dmt_create": [C.POINTER(_P), C.POINTER(dmt_model), C.POINTER(dmt_structure), C.POINTER(dmt_config)],
    "dmt_destroy": [_P],
    "dmt_upload_grid": [_P, _pd],
    "dmt_upload_law": [_P, _i32, _i32, _pd, _i32, _pd, _pd],
    "dmt_set_paths": [_P, _i32, _pd, _pd],
    "dmt_download_paths": [_P, _i32, _i32, _pd],
    "dmt_draw_unit": [_P, _i32, _i64, _i64, _pd, _i64, _u32, _pd, _pu8],
    "dmt_create_layout": [_P, _pi32, _pi32, _pi32, _pu8, _pd, _i64, _pi32],
    "dmt_layout_size": [_P, _i32, _pi64],
    "dmt_draw_proposal": [_P, _i32, _i64, _i64, _pd, _i64, _u32, _pu8],
    "dmt_accept_reject": [_P, _i32, _i64, _i64, _pd, _i64, _u32, _pu8],
    "dmt_loglikhd": [_P, _i32, _i32, _i64, _i64],
    "dmt_recompute_path": [_P, _i32, _i64, _i64, _i32, _pu8],
    "dmt_find_W_for_X": [_P, _i32, _i64, _i64],
    "dmt_upload_obs": [_P, _pd, _pd, _pd, C.c_double],
    "dmt_set_obs": [_P, _i32, _i64, _i64],
    "dmt_download_law": [_P, _i32, _i32, _pd, _pd, _pd],
    "dmt_recompute_guiding_term": [_P, _i32, _i64, _i64, _i32],
    "dmt_set_proposal_law": [_P, _i32, _i64, _i64, _i32, _P, _P, _i32, _P, _P],
    "dmt_swap": [_P, _i32, _i32, _i64, _i64],
    "dmt_save_ll": [_P, _i32, _i64, _i64, _i64],
    "dmt_set_accepted": [_P, _i32, _i64, _i64, _i64, _pu8],
    "dmt_get_block_state": [_P, _i32, _i32, _i64, _i64, _P],
    "dmt_set_block_state": [_P, _i32, _i32, _i64, _i64, _P],
    "dmt_fetch_ll": [_P, _i32, _i64, _i64, _i64, _pd, _pd, _pi64],
    "dmt_mcmc_step": [_P, _i32, _i64, _i64, _i64, _u32, _pd, _pd, _pi64],
    "dmt_guiding_linear": [_i32, _pd, _pd, _pd, _i32, _pd, _pd, _pd, C.c_double, _pd, _pd, _pd],
    "dmt_guiding_linear_td": [_i32, _pd, _pd, _i32, _pd, _pd, _pd, C.c_double, _pd, _pd, _pd],
    "dmt_upload_aux": [_P, _i32, _pd],
    "dmt_upload_aux_a": [_P, _i32, _pd, _i32],
    "dmt_guiding_linear_tda": [_i32, _pd, _i32, _pd, _pd, _pd, C.c_double, _pd, _pd, _pd],
    "dmt_comm_unique_id": [_pu8],
    "dmt_comm_init": [_P, _i32, _i32, _pu8],
    "dmt_mcmc_run": [_P, _i32, _i64, _i64, _i64, _i64, _u32, _pd],
    "dmt_mcmc_step_local": [_P, _i32, _i64, _i64, _i64, _u32, _pd, _pd, _pi64],
    "dmt_mcmc_run_local": [_P, _i32, _i64, _i64, _i64, _i64, _u32, _pd],
    "dmt_set_shard": [_P, _i64],
    "dmt_sync": [_P],
    "dmt_set_timing": [_P, _i32],
    "dmt_get_timing": [_P, _i32, _pd, _pi64],
    "dmt_memory_bytes": [_P, _pi64],
    "dmt_debug_philox": [_i32, _u64, _pu32, _i64, _pu32],
    "dmt_debug_normals": [_i32, _u64, _pu32, _i64, _pd],
    "dmt_snapshot_reserve": [_P, _i32, _i64],
    "dmt_snapshot_take": [_P, _i32, _i64, _i64],
    "dmt_set_run_snapshots": [_P, _i64, _i64],
    "dmt_snapshot_download": [_P, _i32, _i64, _pd, _pi64],
    "dmt_snapshot_write": [_P, C.c_char_p, _i64, _i64],
    "dmt_set_ll": [_P, _i32, _i32, _i64, _i64, _i64, _pd],
    "dmt_fetch_ll_local": [_P, _i32, _i64, _i64, _i64, _pd, _pd, _pi64],
    "dmt_comm_size": [_P, _pi32],
    "dmt_rng_counter": [_P, C.POINTER(_u64)],
    "dmt_set_rng_counter": [_P, _u64],
    "dmt_draw_success": [_P, _i32, _i64, _i64, _pu8],
    "dmt_rng_state": [_P, C.POINTER(_u64), C.POINTER(_u64), _pu8],
    "dmt_set_rng_state": [_P, _u64, _u64, C.c_uint8],
    "dmt_combine_rank_partials": [_pd, _i32, _i64, _pd],
    "dmt_set_service": [_P, _i32, C.c_double],
    "dmt_set_proposal_law_cc": [_P, _i32, _i64, _i64, _i32, _P, _P, _i32, _i32, _P, _P],
    "dmt_service_stats": [_P, C.POINTER(_u64)],
    "dmt_recent_kernels": [C.c_char_p, _i64],
}
for _name, _args in _SIGS.items():
    _f = getattr(lib, _name)
    _f.argtypes = _args
    _f.restype = C.c_int32
lib.dmt_last_error.restype = C.c_char_p
lib.dmt_last_error.argtypes = []
lib.dmt_version.restype = C.c_char_p
lib.dmt_version.argtypes = []


# Hot-path entry points with untyped pointer arguments: the caller passes integer addresses it
# computed once (a numpy array's .ctypes.data), which ctypes forwards without building pointer
# objects — ≈ 1 µs per call instead of ≈ 9 µs through call() + f64p() (dmt_mcmc_run, dmt_sync:
# the per-call host time of the driver's 20-iteration command)
_FAST = {
    "dmt_mcmc_run": [_P, _i32, _i64, _i64, _i64, _i64, _u32, _P],
    "dmt_mcmc_run_local": [_P, _i32, _i64, _i64, _i64, _i64, _u32, _P],
    "dmt_sync": [_P],
}
fast = {}
for _name, _args in _FAST.items():
    fast[_name] = C.CFUNCTYPE(C.c_int32, *_args)((_name, lib))


def recent_kernels() -> list:
    """Demangled names of the last (≤ 8) kernels this thread launched through libdmt, most
    recent first (dmt_recent_kernels)."""
    buf = C.create_string_buffer(8192)
    check(lib.dmt_recent_kernels(buf, len(buf)))
    return [n for n in buf.value.decode(errors="replace").split("\n") if n]


def check(status: int) -> None:
    if status != OK:
        raise DMTError(status, lib.dmt_last_error().decode(errors="replace"))


def call(name: str, *args) -> None:
    check(getattr(lib, name)(*args))


# ---- array helpers ----
def f64p(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous, "need a C-contiguous float64 array"
    return a.ctypes.data_as(_pd)


def u8p(a):
    if a is None:
        return None
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(_pu8)


def i32p(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_pi32)


def u32p(a):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(_pu32)


def version() -> str:
    return lib.dmt_version().decode()
