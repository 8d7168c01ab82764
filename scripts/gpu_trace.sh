#!/bin/bash
# Kernel-trace summaries (rocprofv3 --kernel-trace --stats, no counters) of bench.py workloads, one
# run each: gpurun_out/$TAG/<name>/..._kernel_stats.csv plus the bench line of the traced run.
# RUNS: "name|bench args;name|bench args;..."
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-trace}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra JOBS <<< "${RUNS:-config3|--workload config3 --no-cpu-baseline}"
for j in "${JOBS[@]}"; do
  name=${j%%|*}
  args=${j#*|}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" $args > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAILED $name"; tail -5 "$OUT/$name.err"; exit 1; }
  echo "ok $name"
done
