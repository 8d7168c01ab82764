"""CPU: the C-ABI library builds for gfx950, loads, exports every symbol include/*.h declares, and
its host-only functions agree with the oracle.  No compute call needs a GPU here."""
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "pathplanning_amd.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(pp_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_abi(pkg):
    syms = _declared_symbols()
    assert set(syms) == set(pkg._ffi.EXPORTED)


def test_library_exports_every_declared_symbol(pkg):
    lib_path = pkg._ffi.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(pp_[a-z0-9_]+)\b", out))
    missing = [s for s in _declared_symbols() if s not in exported]
    assert not missing, missing
    L = pkg._ffi.lib()
    for s in _declared_symbols():
        assert hasattr(L, s)


def test_library_holds_gfx950_code(pkg):
    # the offload bundle's target id names the architecture
    with open(pkg._ffi.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_abi_version(pkg):
    assert pkg._ffi.lib().pp_abi_version() == 5 == pkg._ffi.PP_ABI_VERSION


def test_rng_matches_oracle(pkg, oracle_mod):
    L = pkg._ffi.lib()
    for seed in (0, 1, 42, 2**63 + 5):
        for ctr in (0, 1, 2, 1000, 2**40 + 3):
            assert L.pp_rng_u64(seed, ctr) == oracle_mod.rng_u64(seed, ctr)
            assert L.pp_gen_range(seed, ctr, -5.5, 14.5) == oracle_mod.gen_range(seed, ctr, -5.5, 14.5)
            assert pkg.scenes.gen_range(seed, ctr, 0.5, 511.5) == oracle_mod.gen_range(seed, ctr, 0.5, 511.5)
            v = L.pp_gen_range(seed, ctr, 2.0, 8.0)
            assert 2.0 <= v < 8.0


def test_angle_helpers_match_oracle(pkg, oracle_mod):
    L = pkg._ffi.lib()
    for v in (-10.0, -4.0, -3.2, -1e-9, 0.0, 1.0, 3.14159, 6.3, 100.0):
        assert L.pp_mod2pi(v) == oracle_mod.mod2pi(v)
        assert L.pp_pi_2_pi(v) == oracle_mod.pi_2_pi(v)


def test_no_gpu_fails_loudly(pkg):
    if pkg.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(pkg.PPError) as e:
        pkg.Context(0)
    assert e.value.code == pkg._ffi.PP_ERR_NO_DEVICE


def test_product_never_touches_the_oracle():
    base = os.path.join(ROOT, "rs-pathplanning_amd")
    for dirpath, _, files in os.walk(base):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h")):
                with open(os.path.join(dirpath, fn), errors="ignore") as f:
                    txt = f.read()
                assert "import oracle" not in txt and "liboracle" not in txt and "dubins_py" not in txt, fn


def test_create_circle_is_the_crate_polygon(built):
    """pp_create_circle (rrt.rs:43-60, host arithmetic) against the expression restated in Python
    (glibc cos/sin, the Rust evaluation order), bit for bit."""
    import math

    import numpy as np
    from pathplanning_amd import scenes

    for (cx, cy, r) in [(0.0, 0.0, 1.0), (5.0, 5.0, 2.0), (-3.25, 7.5, 0.3), (100.0, 40.0, 7.9)]:
        got = scenes.create_circle_polygon((cx, cy), r)
        n = math.ceil(2.0 * math.pi * r / 1.0)
        exp = np.array([(math.cos(2.0 * math.pi / n * float(i)) * r + cx,
                         math.sin(2.0 * math.pi / n * float(i)) * r + cy)
                        for i in range(int(n + 1.0))])
        assert got.shape == exp.shape and np.array_equal(got, exp)


def test_integration_binding_declares_every_symbol():
    """INTEGRATION.md's Rust extern block (the binding a maintainer adds to the crate) names
    every entry point the header declares, and nothing the header dropped."""
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        txt = f.read()
    bound = set(re.findall(r"pub fn (pp_[a-z0-9_]+)\s*\(", txt))
    assert bound == set(_declared_symbols())
