#!/bin/bash
# A/B kernel timelines: default library vs lib/variant (short default bench under rocprofv3).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/abt"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d "$OUT/a" -o run -- python3 "$R/bench.py" $A > "$OUT/a.log" 2>&1 || exit $?
echo "== A (default)"; python3 "$R/scripts/timeline.py" "$OUT/a/run_kernel_trace.csv" | tail -9
export PP_AMD_LIB="$R/rs-pathplanning_amd/lib/variant/libpathplanning_amd.so"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d "$OUT/b" -o run -- python3 "$R/bench.py" $A > "$OUT/b.log" 2>&1 || exit $?
echo "== B (variant)"; python3 "$R/scripts/timeline.py" "$OUT/b/run_kernel_trace.csv" | tail -9
echo abt-done
