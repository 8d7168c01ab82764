#!/bin/bash
# One build → measure iteration on the GPU box (repo root): GPU parity tests, the default bench
# line, and a kernel trace of a short bench run.  Every GPU step has its own time limit and the
# script stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/iter"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep > "$OUT/trace.log" 2>&1 || exit $?
echo iter-done
