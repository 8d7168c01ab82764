#!/bin/bash
# The 8-GPU shard on one GPU: config 3 and config 5 on 1024 queries (one rank's share of 8192).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/shards"
mkdir -p "$OUT"
cd "$R"
for w in config3 config5; do
  timeout -k 10 300 python3 bench.py --workload $w --queries 1024 --no-cpu-baseline > "$OUT/$w.json" 2> "$OUT/$w.err" || { tail -20 "$OUT/$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$w.json')); print('$w shard', round(d['value']/1e6,2), 'M it/s', d.get('records_digest'))"
done
echo shards-done
