"""bench.py's provenance block (CPU, no GPU call): the measured library's hash and build flags,
the PP_* variables a line was taken with (the library reads none), and the refusal of a PP_AMD_LIB variant build
unless --allow-variant-lib is given."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


def test_provenance_records_knobs(monkeypatch):
    bench = _bench()
    monkeypatch.delenv("PP_AMD_LIB", raising=False)
    monkeypatch.setenv("PP_SOME_KNOB", "3")
    p = bench.provenance(argparse.Namespace(allow_variant_lib=False))
    assert p["lib"].endswith("libpathplanning_amd.so") and len(p["lib_sha256_16"]) == 16
    assert "--offload-arch=gfx950" in p["hipcc_flags"] and p["variant"] is False
    assert p["env_knobs"].get("PP_SOME_KNOB") == "3"


def test_provenance_refuses_variant_lib(monkeypatch):
    bench = _bench()
    monkeypatch.setenv("PP_AMD_LIB", "/nonexistent/libpathplanning_amd.so")
    with pytest.raises(SystemExit):
        bench.provenance(argparse.Namespace(allow_variant_lib=False))
