#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root); summaries → scripts/prof_summary.py.
#   1. kernel trace + stats of the default bench workload (config 2)
#   2. HBM read bytes (FETCH_SIZE) of nn_scan, its own pass
#   3. HBM write bytes (WRITE_SIZE) of nn_scan, its own pass
#   4. kernel trace + stats of the config-3 query batch
# Counters never share a pass with --sys-trace / --runtime-trace (MI355X_MICROARCH.md; pool rules).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/prof"
mkdir -p "$OUT"
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex window_kernel -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex window_kernel -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace3" -o run -- python3 "$R/bench.py" --workload config3 --steps 400 > "$OUT/trace3.log" 2>&1 || exit $?
echo profile-done
