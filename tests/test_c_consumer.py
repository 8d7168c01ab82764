"""CPU: a plain C99 program (tests/c_consumer/consumer.c) compiled by gcc against
include/pathplanning_amd.h and linked with the HIP library — the header is a usable C header on
its own, its struct layouts (pp_dubins_config = DubinsConfig, dubins.rs:315-324; pp_stats) are the
ones the ctypes mirror and a Rust #[repr(C)] block assume, and the host-only entry
points give the same answers through a C caller as through Python and the oracle."""
import json
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def consumer(pkg, tmp_path_factory):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not on PATH")
    libdir = os.path.dirname(pkg._ffi.LIB_PATH)
    exe = str(tmp_path_factory.mktemp("cc") / "consumer")
    subprocess.run([gcc, "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_consumer", "consumer.c"), "-o", exe,
                    "-L", libdir, "-lpathplanning_amd", "-Wl,-rpath," + libdir],
                   check=True, capture_output=True, text=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
    return json.loads(out)


def test_struct_layouts_match_the_ctypes_mirror(pkg, consumer):
    import ctypes as C

    f = pkg._ffi
    assert consumer["abi"] == f.lib().pp_abi_version()
    assert consumer["sizeof.pp_dubins_config"] == C.sizeof(f.DubinsConfigC) == 64
    assert consumer["sizeof.pp_stats"] == C.sizeof(f.StatsC)
    for T, py in (("pp_dubins_config", f.DubinsConfigC), ("pp_stats", f.StatsC)):
        for k, v in consumer.items():
            if k.startswith(T + "."):
                assert v == getattr(py, k.split(".", 1)[1]).offset, k


def test_host_entry_points_through_c(pkg, consumer):
    import dubins_py
    from pathplanning_amd import scenes

    assert consumer["rc_circle"] == consumer["ok"]
    assert consumer["rc_small"] == consumer["err"] and consumer["n_small"] == consumer["n"]
    got = np.array(consumer["xy"]).reshape(-1, 2)
    assert np.array_equal(got, scenes.create_circle_polygon((1.5, -2.0), 3.0))
    assert consumer["n"] == math.ceil(2 * math.pi * 3.0) + 1
    assert consumer["mod2pi"] == dubins_py.mod2pi(-7.25)
    assert consumer["pi_2_pi"] == dubins_py.pi_2_pi(4.0)
    assert int(consumer["rng"]) == dubins_py.rng_u64(42, 7)
    assert consumer["gen_range"] == dubins_py.gen_range(42, 7, -3.0, 5.0)
    # pp_device_count never fails on a CPU-only host (header contract)
    assert consumer["rc_dev"] == consumer["ok"] and consumer["ndev"] >= 0
