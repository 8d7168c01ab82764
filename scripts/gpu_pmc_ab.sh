#!/bin/bash
# One counter pass (PMC, its own rocprofv3 run) of one kernel under a bench workload, for the
# in-tree library and variants (rs-pathplanning_amd/lib/<v>/): gpurun_out/$TAG/<v>/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-pmc_ab}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
K=${KERNEL:-check_finish_kernel}
P=${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH}
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset PP_AMD_LIB; EXTRA_V=""; else export PP_AMD_LIB="$R/rs-pathplanning_amd/lib/$v/libpathplanning_amd.so"; EXTRA_V="--allow-variant-lib"; fi
  timeout -s KILL 300 rocprofv3 --pmc $P -T -f csv --kernel-include-regex "$K" -d "$OUT/$v" -o run -- python3 "$R/bench.py" ${ARGS:---workload config3 --no-cpu-baseline} $EXTRA_V > "$OUT/$v.log" 2>&1 || { echo "FAILED $v"; tail -5 "$OUT/$v.log"; exit 1; }
  echo "ok $v"
done
