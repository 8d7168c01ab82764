#!/bin/bash
# HBM traffic of the window kernel (NN screen) at the bench size: FETCH_SIZE and WRITE_SIZE, one
# rocprofv3 counter pass each (counters never share a pass with tracing), into gpurun_out/prof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/prof"
mkdir -p "$OUT"
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex window_kernel -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex window_kernel -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 || exit $?
echo traffic-done
