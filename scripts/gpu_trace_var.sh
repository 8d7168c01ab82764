#!/bin/bash
# Kernel traces of bench workloads against the in-tree library or a variant (VAR=<name>:
# rs-pathplanning_amd/lib/<name>/), one rocprofv3 --kernel-trace --stats run each.
# RUNS: "name|var|bench args;..." (var "base" = in-tree)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-tracevar}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra JOBS <<< "$RUNS"
for j in "${JOBS[@]}"; do
  IFS='|' read -r name var args <<< "$j"
  if [ "$var" = base ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" $args > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAILED $name"; tail -5 "$OUT/$name.err"; exit 1; }
  else
    PP_AMD_LIB="$R/rs-pathplanning_amd/lib/$var/libpathplanning_amd.so" timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$name" -o run -- python3 "$R/bench.py" $args --allow-variant-lib > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "FAILED $name"; tail -5 "$OUT/$name.err"; exit 1; }
  fi
  echo "ok $name"
done
