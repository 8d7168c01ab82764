"""``pathplanning::dubins`` (src/dubins.rs) on the GPU.

Mirrors the module's public API — ``Mode``, ``mod2pi``, ``pi_2_pi``, ``DubinsConfig``,
``dubins_path_planning`` — with the path computed by the HIP ``dubins_batch`` kernel (one lane per
configuration, f64, the reference's evaluation order).  ``dubins_path_planning_batch`` is the
batched form the extend loop is built from.
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
