#!/bin/bash
# Config 5 with 2, 3 (default) and 4 sub-batch streams (PP_BATCH_STREAMS), batch and shard.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/str5"
mkdir -p "$OUT"
cd "$R"
for q in 8192 1024; do
  for ns in 3 2 4; do
    PP_BATCH_STREAMS=$ns timeout -k 10 300 python3 bench.py --workload config5 --queries $q --no-cpu-baseline > "$OUT/b_${ns}_$q.json" 2> "$OUT/b_${ns}_$q.err" || { tail -20 "$OUT/b_${ns}_$q.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${ns}_$q.json')); print('streams $ns q $q', round(d['value']/1e6,2), 'M it/s', d['records_digest'])"
  done
done
echo str5-done
