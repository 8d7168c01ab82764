#!/bin/bash
# HBM traffic of the batch NN kernels (config 3: mq_sample_nn, config 5: star_sample): FETCH_SIZE
# and WRITE_SIZE, one rocprofv3 counter pass each, whole-batch launches only (one stream).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/traffic"
mkdir -p "$OUT"
export PP_BATCH_STREAMS=1
for spec in "config3:mq_sample_nn" "config5:star_sample"; do
  w=${spec%%:*}; k=${spec##*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T -f csv --kernel-include-regex $k -d "$OUT/${w}_$c" -o run -- python3 "$R/bench.py" --workload $w --no-cpu-baseline > "$OUT/${w}_$c.log" 2>&1 || exit $?
  done
done
echo traffic-done
