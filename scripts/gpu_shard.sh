#!/bin/bash
# config-3 shard sweep: the 1024-query shard (and the 8192 batch) per window K and schedule, plus
# a config-2 line; everything under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-shard}"
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --warmup 3 --no-sub --no-cpu-baseline > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -20 "$OUT/c2.err"; exit 1; }
echo c2 done
for q in ${QUERIES:-1024}; do
  for sch in ${SCHEDULES:-lockstep persistent}; do
    for k in ${KS:-16 32 64}; do
      timeout -k 10 300 python -u bench.py --workload config3 --queries $q --schedule $sch --batch-window $k --no-cpu-baseline > "$OUT/c3_${q}_${sch}_k$k.json" 2> "$OUT/c3_${q}_${sch}_k$k.err" || { tail -20 "$OUT/c3_${q}_${sch}_k$k.err"; exit 1; }
      echo "done $q $sch $k"
    done
  done
done
