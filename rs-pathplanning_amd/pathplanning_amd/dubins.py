"""``pathplanning::dubins`` (src/dubins.rs) on the GPU.

Mirrors the module's public API — ``Mode``, ``mod2pi``, ``pi_2_pi``, the six words ``lsl`` ..
``lrl``, ``DubinsConfig``, ``dubins_path_planning_from_origin``, ``dubins_path_planning`` — with the
words and paths computed by HIP kernels (one lane per configuration, f64, the reference's
evaluation order).  The ``*_batch`` forms take many configurations per launch.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from enum import Enum

import numpy as np

from . import _ffi


class Mode(Enum):  # dubins.rs:4-9
    L = 0
    S = 1
    R = 2


# ALL_PLANNERS order (dubins.rs:291) and each word's segment modes (dubins.rs:26-135)
WORDS = ["LSL", "RSR", "LSR", "RSL", "RLR", "LRL"]
WORD_MODES = [tuple(Mode[ch] for ch in w) for w in WORDS]


def mod2pi(theta: float) -> float:  # dubins.rs:18-20
    return _ffi.lib().pp_mod2pi(theta)


def pi_2_pi(angle: float) -> float:  # dubins.rs:22-24
    return _ffi.lib().pp_pi_2_pi(angle)


@dataclass
class DubinsConfig:  # dubins.rs:315-324
    sx: float
    sy: float
    syaw: float
    ex: float
    ey: float
    eyaw: float
    turn_radius: float
    step_size: float


def _max_points(conf: DubinsConfig) -> int:
    # n_point = trunc(total/step) + 7 with total <= 3 * 2pi + |d| / R + 2 (CSC: p <= d + 2; CCC:
    # every length < 2pi) — a safe capacity bound for the output slot
    d = np.hypot(conf.ex - conf.sx, conf.ey - conf.sy) / conf.turn_radius
    return int((3 * 2 * np.pi + d + 4.0) / conf.step_size) + 16


def dubins_path_planning_batch(confs, ctx: _ffi.Context | None = None, cap: int | None = None):
    """dubins_path_planning for every config: list of ``(px, py, pyaw, mode, cost)`` or ``None``."""
    confs = list(confs)
    n = len(confs)
    if n == 0:
        return []
    ctx = ctx or _ffi.default_context()
    if cap is None:
        cap = max(_max_points(c) for c in confs)
    arr = (_ffi.DubinsConfigC * n)(*[
        _ffi.DubinsConfigC(c.sx, c.sy, c.syaw, c.ex, c.ey, c.eyaw, c.turn_radius, c.step_size)
        for c in confs])
    px = np.zeros(n * cap)
    py = np.zeros(n * cap)
    pyaw = np.zeros(n * cap)
    npts = np.zeros(n, dtype=np.int32)
    word = np.zeros(n, dtype=np.int32)
    cost = np.zeros(n)
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int32)
    _ffi.check(_ffi.lib().pp_dubins_path_planning_batch(
        ctx.handle, arr, n, cap, px.ctypes.data_as(dp), py.ctypes.data_as(dp),
        pyaw.ctypes.data_as(dp), npts.ctypes.data_as(ip), word.ctypes.data_as(ip),
        cost.ctypes.data_as(dp)))
    out = []
    for i in range(n):
        if word[i] < 0:
            out.append(None)
            continue
        k = int(npts[i])
        s = slice(i * cap, i * cap + k)
        out.append((px[s].copy(), py[s].copy(), pyaw[s].copy(), WORD_MODES[word[i]],
                    float(cost[i])))
    return out


def dubins_path_planning(conf: DubinsConfig, ctx: _ffi.Context | None = None):
    """dubins.rs:401-428: ``(px, py, pyaw, mode, cost)`` or ``None``."""
    return dubins_path_planning_batch([conf], ctx)[0]


def dubins_path_planning_from_origin_batch(confs, ctx: _ffi.Context | None = None,
                                           cap: int | None = None):
    """dubins_path_planning_from_origin (dubins.rs:326-399) for every ``(dx, dy, eyaw, c,
    step_size)``: list of ``(px, py, pyaw, mode, cost)`` in the local frame (yaw as generated) or
    ``None``."""
    confs = np.ascontiguousarray(confs, dtype=np.float64).reshape(-1, 5)
    n = len(confs)
    if n == 0:
        return []
    ctx = ctx or _ffi.default_context()
    if cap is None:
        d = np.hypot(confs[:, 0], confs[:, 1]) * confs[:, 3]
        cap = int(np.max((3 * 2 * np.pi + d + 4.0) / confs[:, 4])) + 16
    px, py, pyaw = (np.zeros(n * cap) for _ in range(3))
    npts = np.zeros(n, dtype=np.int32)
    word = np.zeros(n, dtype=np.int32)
    cost = np.zeros(n)
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
    _ffi.check(_ffi.lib().pp_dubins_path_planning_from_origin_batch(
        ctx.handle, confs.ctypes.data_as(dp), n, cap, px.ctypes.data_as(dp),
        py.ctypes.data_as(dp), pyaw.ctypes.data_as(dp), npts.ctypes.data_as(ip),
        word.ctypes.data_as(ip), cost.ctypes.data_as(dp)))
    out = []
    for i in range(n):
        if word[i] < 0:
            out.append(None)
            continue
        s = slice(i * cap, i * cap + int(npts[i]))
        out.append((px[s].copy(), py[s].copy(), pyaw[s].copy(), WORD_MODES[word[i]],
                    float(cost[i])))
    return out


def dubins_path_planning_from_origin(dx: float, dy: float, eyaw: float, c: float,
                                     step_size: float, ctx: _ffi.Context | None = None):
    """dubins.rs:326-399: ``(px, py, pyaw, mode, cost)`` in the local frame, or ``None``."""
    return dubins_path_planning_from_origin_batch([(dx, dy, eyaw, c, step_size)], ctx)[0]


def words_batch(abd, ctx: _ffi.Context | None = None):
    """The six words of every ``(alpha, beta, d)``: arrays ``tpq[n, 6, 3]`` and ``ok[n, 6]``
    (ALL_PLANNERS order, dubins.rs:291)."""
    abd = np.ascontiguousarray(abd, dtype=np.float64).reshape(-1, 3)
    n = len(abd)
    ctx = ctx or _ffi.default_context()
    tpq = np.zeros((n, 6, 3))
    ok = np.zeros((n, 6), dtype=np.int32)
    if n:
        _ffi.check(_ffi.lib().pp_dubins_words_batch(
            ctx.handle, abd.ctypes.data_as(C.POINTER(C.c_double)), n,
            tpq.ctypes.data_as(C.POINTER(C.c_double)), ok.ctypes.data_as(C.POINTER(C.c_int32))))
    return tpq, ok


def _word(w: int, alpha: float, beta: float, d: float):
    tpq, ok = words_batch([(alpha, beta, d)])
    if not ok[0, w]:
        return (None, None, None, WORD_MODES[w])
    t, p, q = (float(v) for v in tpq[0, w])
    return (t, p, q, WORD_MODES[w])


def lsl(alpha: float, beta: float, d: float):  # dubins.rs:27-48
    return _word(0, alpha, beta, d)


def rsr(alpha: float, beta: float, d: float):  # dubins.rs:51-71
    return _word(1, alpha, beta, d)


def lsr(alpha: float, beta: float, d: float):  # dubins.rs:74-92
    return _word(2, alpha, beta, d)


def rsl(alpha: float, beta: float, d: float):  # dubins.rs:95-113
    return _word(3, alpha, beta, d)


def rlr(alpha: float, beta: float, d: float):  # dubins.rs:116-133
    return _word(4, alpha, beta, d)


def lrl(alpha: float, beta: float, d: float):  # dubins.rs:136-153
    return _word(5, alpha, beta, d)
