#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats, no counters) of bench workloads: one run per
# workload in WLS, plus the plain bench line of the same command for comparison.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-trace}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for wl in ${WLS:-config2}; do
  case $wl in
    default) A="" ;;
    config2|config4|polygons) A="--workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep ${EXTRA:-}" ;;
    *) A="--workload $wl --warmup 3 --no-cpu-baseline ${EXTRA:-}" ;;
  esac
  timeout -k 10 400 python3 "$R/bench.py" $A > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { tail -5 "$OUT/bench_$wl.err"; exit 1; }
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/$wl" -o run -- python3 "$R/bench.py" $A > "$OUT/trace_$wl.log" 2>&1 || { tail -5 "$OUT/trace_$wl.log"; exit 1; }
  echo "ok $wl"
done
echo trace-done
