#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of one bench workload for the in-tree library
# and library variants (rs-pathplanning_amd/lib/<v>/): gpurun_out/$TAG/<v>/..._kernel_stats.csv.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-trace_ab}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset PP_AMD_LIB; EXTRA_V=""; else export PP_AMD_LIB="$R/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so"; EXTRA_V="--allow-variant-lib"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$v" -o run -- python3 "$R/bench.py" ${ARGS:---workload config3 --no-cpu-baseline} $EXTRA_V > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "FAILED $v"; tail -5 "$OUT/$v.err"; exit 1; }
  echo "ok $v"
done
