"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer over the host-side C/C++ that never runs on
the GPU (SURVEY.md §5's sanitizer pass; host code only — GPU sanitizers are not available).

tests/sanitize/san_driver.cpp is built with gcc/g++ ``-fsanitize=address,undefined
-fno-sanitize-recover=all`` together with
  * rs-pathplanning_amd/csrc/pp_scene.cpp — the library's scene building (Space::new,
    rrt.rs:81-122: shrunken bounds, buffered obstacles, polygon rings/edges, the item-grid CSR and
    its LDS image), with the CSR recounted by brute force under every LDS budget, and
  * oracle/pp_oracle.c — extend (incremental and full re-verify), check_finish, plan, RRT* and
    the threaded query pools, built with the oracle's own numeric flags (oracle/Makefile).
Any sanitizer report aborts the driver.  Its results must also equal the unsanitized oracle
(oracle/liboracle.so) run in-process on the same scenes, so the instrumented build computes the
same thing as the one the parity tests use."""
import json
import math
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

ORACLE_FLAGS = ["-O1", "-g", "-ffp-contract=off", "-fno-fast-math", "-fno-builtin-sin",
                "-fno-builtin-cos", "-fno-builtin-sincos"]
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def _scenes():
    from pathplanning_amd import scenes

    out = []
    b6 = scenes.bench6()
    out.append(("bench6", b6, 600))
    f5 = scenes.field512()
    out.append(("field512", f5, 300))
    rng = np.random.default_rng(5)
    many = dict(f5)
    # > 4096 items: the grid-only LDS image (cull discs in L2) or no image; some discs reach
    # outside the sampling box, one covers a quarter of it
    c = np.stack([rng.uniform(-40, 552, 6000), rng.uniform(-40, 552, 6000),
                  rng.uniform(0.1, 2.0, 6000)], 1)
    c[0] = (400.0, 400.0, 90.0)
    many["circles"] = [tuple(r) for r in c]
    out.append(("field512_6000", many, 150))
    empty = dict(b6)
    empty["circles"] = []
    out.append(("empty", empty, 300))
    out.append(("transit", scenes.transit(), 300))
    out.append(("bench6_polygons", scenes.bench6_polygons(), 300))
    return out


def _write(path, items, bad):
    with open(path, "w") as f:
        for name, raw, iters in items:
            w, _, turn = raw["robot"]
            f.write(f"scene {name} ")
            if "bounds_polygon" in raw:
                b = np.asarray(raw["bounds_polygon"], dtype=np.float64).reshape(-1, 2)
                obs = [np.asarray(o, dtype=np.float64).reshape(-1, 2) for o in raw["obstacle_polygons"]]
                off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(int)
                f.write(f"polygons {w!r} {turn!r} {raw['step_size']!r} {len(b)} ")
                f.write(" ".join(repr(float(v)) for v in b.ravel()))
                f.write(f" {len(obs)} " + " ".join(str(v) for v in off) + f" {int(off[-1])} ")
                f.write(" ".join(repr(float(v)) for o in obs for v in o.ravel()))
            else:
                x0, y0, x1, y1 = raw["bounds"]
                circ = np.asarray(raw["circles"], dtype=np.float64).reshape(-1, 3)
                f.write(f"discs {x0!r} {y0!r} {x1!r} {y1!r} {w!r} {turn!r} {raw['step_size']!r} "
                        f"{len(circ)} " + " ".join(repr(float(v)) for v in circ.ravel()))
            sx, sy, syaw = raw["start"]
            gx, gy, gyaw = raw["goal"]
            f.write(f" {sx!r} {sy!r} {syaw!r} {gx!r} {gy!r} {gyaw!r} 7 {iters}\n")
        f.write(bad)


# invalid inputs: the library's argument checks must reject them without touching bad memory
BAD = (
    "scene bad_offsets polygons 1.0 1.0 0.1 4 0 0 10 0 10 10 0 10 2 0 3 1 3 1 1 2 1 2 2 "
    "0 0 0 1 1 0 7 10\n"
    "scene nan_vertex polygons 1.0 1.0 0.1 4 0 0 10 0 10 10 0 10 1 0 3 3 1 1 nan 1 2 2 "
    "0 0 0 1 1 0 7 10\n"
    "scene ring_too_small polygons 1.0 1.0 0.1 4 0 0 10 0 0 0 0 0 0 0 0 0 0 0 1 1 0 7 10\n"
    "scene empty_box discs 0 0 1 1 2.0 1.0 0.1 0 0 0 0 1 1 0 7 10\n"
    "scene inf_disc discs 0 0 10 10 1.0 1.0 0.1 1 5 inf 1 0 0 0 1 1 0 7 10\n"
)


@pytest.fixture(scope="module")
def san_run(pkg, tmp_path_factory):
    gcc, gxx = shutil.which("gcc"), shutil.which("g++")
    if gcc is None or gxx is None:
        pytest.skip("gcc/g++ not on PATH")
    d = tmp_path_factory.mktemp("san")
    objs = []
    for src, cc, extra in (
        (os.path.join(ROOT, "oracle", "pp_oracle.c"), gcc, ["-std=c11"] + ORACLE_FLAGS),
        (os.path.join(ROOT, "rs-pathplanning_amd", "csrc", "pp_scene.cpp"), gxx, ["-std=c++17", "-O1", "-g"]),
        (os.path.join(ROOT, "tests", "sanitize", "san_driver.cpp"), gxx, ["-std=c++17", "-O1", "-g"]),
    ):
        o = str(d / (os.path.basename(src) + ".o"))
        subprocess.run([cc, *extra, *SAN, "-Wall", "-c", src, "-o", o], check=True,
                       capture_output=True, text=True)
        objs.append(o)
    exe = str(d / "san_driver")
    subprocess.run([gxx, *SAN, *objs, "-o", exe, "-lm", "-pthread"], check=True,
                   capture_output=True, text=True)
    items = _scenes()
    inp = str(d / "scenes.txt")
    _write(inp, items, BAD)
    env = dict(os.environ)
    # the harness may preload its own library ahead of the ASan runtime: do not abort on that
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    p = subprocess.run([exe, inp], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    return {r["name"]: r for r in json.loads(p.stdout)}, items


def test_sanitized_scene_builder_and_oracle_run_clean(san_run):
    res, items = san_run
    for name, raw, _ in items:
        r = res[name]
        assert r["rc"] == 0, r
        # the LDS image never exceeds its budget and the grid is at most 256 x 256
        for gnx, gny, entries, lds, o_d4 in r["grids"]:
            assert 1 <= gnx <= 256 and 1 <= gny <= 256 and entries >= 0
            assert 0 <= lds <= 64 * 1024
    assert res["field512_6000"]["grids"][2][3] == 0  # zero budget: no grid-only image
    # the inside bitmap (point_blocked): cells set on a dense field, and every point a set cell
    # maps to lies inside a disc
    for name, r in res.items():
        if "inside" in r:
            assert r["inside"][1] == 0, (name, r["inside"])
    assert res["field512_6000"]["inside"][0] > 1000
    # invalid inputs are refused (PP_ERR_INVALID_ARGUMENT) with a message
    for name in ("bad_offsets", "nan_vertex", "ring_too_small", "empty_box", "inf_disc"):
        assert res[name]["rc"] == -1 and res[name]["err"], res[name]


def test_sanitized_oracle_equals_the_unsanitized_one(san_run):
    import oracle as orc

    res, items = san_run
    for name, raw, iters in items:
        r = res[name]
        S = orc.OracleScene.from_raw(raw)
        assert r["box"] == [S.minx, S.maxx, S.miny, S.maxy], name
        sx, sy, syaw = raw["start"]
        gx, gy, gyaw = raw["goal"]
        T = orc.OracleTree(raw["start"], iters + 2)
        acc, _, _ = orc.rrt_extend(S, T, 7, 0, iters)
        T2 = orc.OracleTree(raw["start"], iters + 2)
        acc2, _, _ = orc.rrt_extend(S, T2, 7, 0, iters, full_reverify=True)
        assert r["extend"] == [acc, acc2], name
        x, y, yaw, par = T.arrays()
        assert r["tree"] == [len(x), int(par.sum()), x[-1], y[-1], yaw[-1]], name
        for node, rc, n, length, nch in r["finish"]:
            cf = orc.check_finish(S, T, node, (gx, gy), gyaw)
            assert rc == int(cf["ok"]) and n == cf["n"] and nch == len(cf["chain"]), (name, node)
            if rc == 1:
                assert length == cf["length"]
        P = orc.OracleTree(raw["start"], iters + 2)
        pacc, best, blen, _ = orc.plan(S, P, 7, 0, iters, (gx, gy), gyaw)
        assert r["plan"] == [pacc, best, blen if best >= 0 else -1.0], name
        ST = orc.OracleStarTree(raw["start"], iters + 2)
        sacc, rew, _, _ = orc.star_extend(S, ST, 7, 0, iters)
        assert r["star"] == [sacc, rew], name
        x, y, yaw, par = ST.arrays()
        assert r["star_tree"] == [len(x), int(par.sum()), x[-1], y[-1], yaw[-1]], name
        starts = [raw["start"]] * 4
        seeds = [7 + 1000 * q for q in range(4)]
        qa = orc.queries(S, starts, seeds, iters // 4, threads=2)
        qs, qrw = orc.star_queries(S, starts, seeds, iters // 4, 0, 0.0, threads=2)
        assert r["queries"] == [qa, qs, qrw], name
    # the library's cull slack formula (pp_scene.cpp) is what pp_space_new installs
    assert res["bench6"]["cull_slack"] == pytest.approx(1e-3)
    assert math.isfinite(res["transit"]["cull_slack"])
