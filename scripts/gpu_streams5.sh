#!/bin/bash
# Config 5 (8192 queries and a 1024-query shard) across sub-batch stream counts.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/streams5"
mkdir -p "$OUT"
cd "$R"
for n in ${NS:-2 3 4}; do
  for q in 8192 1024; do
    PP_BATCH_STREAMS=$n timeout -k 10 300 python3 bench.py --workload config5 --queries $q --no-cpu-baseline > "$OUT/b_${n}_$q.json" 2> "$OUT/b_${n}_$q.err" || { tail -20 "$OUT/b_${n}_$q.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_$q.json')); print('streams=$n q=$q', d['value'], d['nodes_total'])"
  done
done
echo streams-done
