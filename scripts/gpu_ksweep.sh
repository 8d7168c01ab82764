#!/bin/bash
# Batch-window sweep (bench.py --batch-window K) of config 3 at QUERIES queries, REPS runs each,
# alternating the K values; bench lines into gpurun_out/$TAG/k<K>_<rep>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-ksweep}"
mkdir -p "$OUT"
for rep in ${REPS:-1}; do
  for k in ${KS:-16 32 64}; do
    timeout -k 10 300 python -u bench.py --workload ${WL:-config3} --queries ${QUERIES:-1024} --batch-window $k --no-cpu-baseline > "$OUT/k${k}_$rep.json" 2> "$OUT/k${k}_$rep.err" || { tail -20 "$OUT/k${k}_$rep.err"; exit 1; }
    echo "done $k $rep"
  done
done
