#!/bin/bash
# Phase-A span schedule A/B of the batch plan (PP_AMD_CFB_SPAN0 / PP_AMD_CFB_SPAN): config 3 per
# SPANS entry "s0:s"; everything under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-span}"
mkdir -p "$OUT"
for sp in ${SPANS:-4:4}; do
  s0=${sp%%:*}; s1=${sp#*:}
  for rep in ${REPS:-1}; do
    PP_AMD_CFB_SPAN0=$s0 PP_AMD_CFB_SPAN=$s1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload config3 $EXTRA > "$OUT/c3_${s0}_${s1}_$rep.json" 2> "$OUT/c3_${s0}_${s1}_$rep.err" || { tail -20 "$OUT/c3_${s0}_${s1}_$rep.err"; exit 1; }
    echo "done $sp $rep"
  done
done
