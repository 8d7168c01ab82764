"""ctypes binding of the C ABI (include/pathplanning_amd.h) — the same symbols a Rust host binds
through ``extern "C"``.  The shared library is built in-tree by
``__graft_entry__.build()`` into ``rs-pathplanning_amd/lib/``; there is no fallback: a missing
library or a missing GPU raises."""
from __future__ import annotations

import ctypes as C
import os
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "PP_AMD_LIB", os.path.join(os.path.dirname(PKG_DIR), "lib", "libpathplanning_amd.so"))

PP_OK = 0
PP_ERR_INVALID_ARGUMENT = -1
PP_ERR_HIP = -2
PP_ERR_NO_DEVICE = -3
PP_ERR_CAPACITY = -4
PP_ERR_STATE = -5
PP_ERR_STEER_OVERFLOW = -6
PP_ERR_REFERENCE_PANIC = -7
PP_CF_CHAIN = 18
PP_ABI_VERSION = 5

_ERR_NAMES = {
    PP_ERR_INVALID_ARGUMENT: "PP_ERR_INVALID_ARGUMENT", PP_ERR_HIP: "PP_ERR_HIP",
    PP_ERR_NO_DEVICE: "PP_ERR_NO_DEVICE", PP_ERR_CAPACITY: "PP_ERR_CAPACITY",
    PP_ERR_STATE: "PP_ERR_STATE", PP_ERR_STEER_OVERFLOW: "PP_ERR_STEER_OVERFLOW",
    PP_ERR_REFERENCE_PANIC: "PP_ERR_REFERENCE_PANIC",
}

# every symbol include/pathplanning_amd.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = [
    "pp_abi_version", "pp_last_error", "pp_device_count", "pp_create", "pp_destroy",
    "pp_synchronize", "pp_rng_u64", "pp_gen_range", "pp_mod2pi", "pp_pi_2_pi",
    "pp_dubins_path_planning_batch", "pp_dubins_path_planning_from_origin_batch",
    "pp_dubins_words_batch", "pp_create_circle", "pp_rrt_line_to_origin", "pp_rrt_optimize",
    "pp_rrt_finalize",
    "pp_space_new", "pp_space_set_grid", "pp_space_get_bounds",
    "pp_space_new_polygons", "pp_space_verify_batch",
    "pp_rrt_new",
    "pp_rrt_set_window", "pp_rrt_extend", "pp_rrt_extend_samples", "pp_rrt_tree_import",
    "pp_rrt_plan_one", "pp_rrt_tree_size",
    "pp_rrt_iteration", "pp_rrt_tree_export", "pp_rrt_get_nearest_node_batch",
    "pp_rrt_verify_node_batch", "pp_rrt_check_finish_batch", "pp_rrt_check_finish",
    "pp_rrt_plan", "pp_batch_new", "pp_batch_set_window", "pp_batch_set_finish_schedule", "pp_batch_extend", "pp_batch_state", "pp_batch_tree_export",
    "pp_batch_plan",
    "pp_star_new", "pp_star_extend", "pp_star_state", "pp_star_tree_export",
    "pp_rrt_get_stats", "pp_rrt_reset_stats", "pp_set_profiling",
]


class PPError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


class DubinsConfigC(C.Structure):
    _fields_ = [(n, C.c_double) for n in
                ("sx", "sy", "syaw", "ex", "ey", "eyaw", "turn_radius", "step_size")]


class StatsC(C.Structure):
    _fields_ = [
        ("iterations", C.c_int64), ("accepted", C.c_int64), ("windows", C.c_int64),
        ("truncations", C.c_int64), ("repair_rounds", C.c_int64), ("repairs", C.c_int64),
        ("literal_repairs", C.c_int64), ("nn_flagged", C.c_int64), ("node_evals", C.c_int64),
        ("nn_scan_ms", C.c_double), ("nn_scan_launches", C.c_int64),
        ("steer_ms", C.c_double), ("steer_launches", C.c_int64),
        ("finalize_ms", C.c_double), ("prep_ms", C.c_double), ("insert_ms", C.c_double),
        ("walk_points", C.c_int64), ("walk_arc_points", C.c_int64), ("batch_steps", C.c_int64), ("batch_passes", C.c_int64),
        ("finish_ms", C.c_double), ("finish_launches", C.c_int64), ("finish_nodes", C.c_int64),
        ("finish_edges", C.c_int64), ("finish_points", C.c_int64),
        ("finish_arc_points", C.c_int64),
        ("reserved_abi3", C.c_int64 * 8),
        ("samples_evaluated", C.c_int64), ("samples_blocked", C.c_int64),
        ("walk_tasks", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved_abi3"}


_lock = threading.Lock()
_lib = None


def lib():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise PPError(PP_ERR_STATE, f"{LIB_PATH} not built: run __graft_entry__.build()")
        # One HIP runtime per process: PyTorch (the streams / torch.distributed plumbing) ships
        # its own libamdhip64 / libhsa-runtime64; loaded first, the library binds to that one
        # instead of bringing /opt/rocm's beside it.  Measured: the config-3 batch (two sub-batch
        # streams) 320 -> 342 M it/s, a 1024-query shard 145 -> 172 M; single-stream workloads
        # unchanged.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        L.pp_abi_version.restype = C.c_int
        if L.pp_abi_version() != PP_ABI_VERSION:
            raise PPError(PP_ERR_STATE, f"{LIB_PATH}: ABI {L.pp_abi_version()}, this binding is "
                                        f"{PP_ABI_VERSION} (rebuild with __graft_entry__.build())")
        dp, ip, i64p = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
        vp = C.c_void_p
        sig = {
            "pp_abi_version": ([], C.c_int),
            "pp_last_error": ([], C.c_char_p),
            "pp_device_count": ([ip], C.c_int),
            "pp_create": ([C.c_int, C.POINTER(vp)], C.c_int),
            "pp_destroy": ([vp], C.c_int),
            "pp_synchronize": ([vp], C.c_int),
            "pp_rng_u64": ([C.c_uint64, C.c_uint64], C.c_uint64),
            "pp_gen_range": ([C.c_uint64, C.c_uint64, C.c_double, C.c_double], C.c_double),
            "pp_mod2pi": ([C.c_double], C.c_double),
            "pp_pi_2_pi": ([C.c_double], C.c_double),
            "pp_dubins_path_planning_batch": (
                [vp, C.POINTER(DubinsConfigC), C.c_int, C.c_int, dp, dp, dp, ip, ip, dp], C.c_int),
            "pp_dubins_path_planning_from_origin_batch": (
                [vp, dp, C.c_int, C.c_int, dp, dp, dp, ip, ip, dp], C.c_int),
            "pp_dubins_words_batch": ([vp, dp, C.c_int, dp, ip], C.c_int),
            "pp_create_circle": ([C.c_double, C.c_double, C.c_double, dp, C.c_int, ip], C.c_int),
            "pp_rrt_line_to_origin": ([vp, C.c_int32, dp, dp, C.c_int64, i64p], C.c_int),
            "pp_rrt_optimize": ([vp, C.c_int32, C.c_int, ip, ip], C.c_int),
            "pp_rrt_finalize": ([vp, C.c_double, C.c_double, C.c_double, C.c_int32, dp, dp,
                                 C.c_int64, i64p, C.POINTER(C.c_uint8)], C.c_int),
            "pp_space_new": ([vp] + [C.c_double] * 7 + [dp, dp, dp, C.c_int], C.c_int),
            "pp_space_set_grid": ([vp, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_double,
                                   C.c_double, C.c_double], C.c_int),
            "pp_space_get_bounds": ([vp, dp], C.c_int),
            "pp_space_new_polygons": ([vp, dp, C.c_int, dp, C.POINTER(C.c_int32), C.c_int,
                                       C.c_double, C.c_double, C.c_double], C.c_int),
            "pp_space_verify_batch": ([vp, dp, dp, C.POINTER(C.c_int64), C.c_int,
                                       C.POINTER(C.c_uint8)], C.c_int),
            "pp_rrt_new": ([vp] + [C.c_double] * 6 + [C.c_int64, C.c_double, C.c_uint64, C.c_int64],
                           C.c_int),
            "pp_rrt_set_window": ([vp, C.c_int], C.c_int),
            "pp_rrt_extend": ([vp, C.c_int64, i64p], C.c_int),
            "pp_rrt_extend_samples": ([vp, dp, dp, C.c_int64, ip, dp, C.POINTER(C.c_uint8), i64p],
                                      C.c_int),
            "pp_rrt_tree_import": ([vp, dp, dp, dp, ip, C.c_int64], C.c_int),
            "pp_rrt_plan_one": ([vp, ip], C.c_int),
            "pp_rrt_tree_size": ([vp, i64p], C.c_int),
            "pp_rrt_iteration": ([vp, i64p], C.c_int),
            "pp_rrt_tree_export": ([vp, dp, dp, dp, ip, C.c_int64, i64p], C.c_int),
            "pp_rrt_get_nearest_node_batch": ([vp, dp, dp, C.c_int, ip, dp], C.c_int),
            "pp_rrt_verify_node_batch": ([vp, dp, dp, ip, C.c_int, C.POINTER(C.c_uint8), dp],
                                         C.c_int),
            "pp_rrt_check_finish_batch": ([vp, ip, C.c_int, C.POINTER(C.c_uint8), dp, ip, ip],
                                          C.c_int),
            "pp_rrt_check_finish": ([vp, C.c_int32, C.POINTER(C.c_uint8), dp, dp, C.c_int64, i64p,
                                     dp], C.c_int),
            "pp_rrt_plan": ([vp, C.c_int64, ip, dp, i64p], C.c_int),
            "pp_batch_new": ([vp, C.c_int, dp, dp, C.POINTER(C.c_uint64), C.c_int64, C.c_double],
                             C.c_int),
            "pp_batch_set_window": ([vp, C.c_int], C.c_int),
            "pp_batch_set_finish_schedule": ([vp, C.c_int, C.c_int, C.c_int], C.c_int),
            "pp_batch_extend": ([vp, C.c_int64, i64p, i64p], C.c_int),
            "pp_batch_state": ([vp, ip, i64p, i64p], C.c_int),
            "pp_batch_tree_export": ([vp, C.c_int, dp, dp, dp, ip, C.c_int64, i64p], C.c_int),
            "pp_batch_plan": ([vp, ip, dp, ip, ip, i64p], C.c_int),
            "pp_star_new": ([vp, C.c_int, dp, C.POINTER(C.c_uint64), C.c_int64, C.c_double,
                             C.c_int, C.c_double], C.c_int),
            "pp_star_extend": ([vp, C.c_int64, i64p, i64p, i64p], C.c_int),
            "pp_star_state": ([vp, ip, i64p, i64p, i64p], C.c_int),
            "pp_star_tree_export": ([vp, C.c_int, dp, dp, dp, ip, dp, C.c_int64, i64p], C.c_int),
            "pp_rrt_get_stats": ([vp, C.POINTER(StatsC), C.c_uint64], C.c_int),
            "pp_rrt_reset_stats": ([vp], C.c_int),
            "pp_set_profiling": ([vp, C.c_int], C.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
        return L


def check(rc):
    if rc != PP_OK:
        msg = lib().pp_last_error()
        raise PPError(rc, msg.decode() if msg else "")
    return rc


def device_count() -> int:
    n = C.c_int32(0)
    check(lib().pp_device_count(C.byref(n)))
    return n.value


class Context:
    """One HIP stream + device-resident scene/tree (``pp_ctx``)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        check(lib().pp_create(device, C.byref(self._h)))
        self.device = device

    @property
    def handle(self):
        if not self._h:
            raise PPError(PP_ERR_STATE, "context destroyed")
        return self._h

    def close(self):
        if self._h:
            lib().pp_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device: int = 0) -> Context:
    with _lock:
        ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _default_ctx[device] = ctx
    return ctx
