#!/bin/bash
# RRT* graphs on/off: tests, then config 5 (8192 queries and a 1024-query shard) both ways.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/graph"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rrtstar.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for g in 0 1; do
  for q in 8192 1024; do
    if [ $g = 1 ]; then export PP_NO_GRAPH=1; else unset PP_NO_GRAPH; fi
    timeout -k 10 300 python3 bench.py --workload config5 --queries $q --no-cpu-baseline > "$OUT/b_${g}_$q.json" 2> "$OUT/b_${g}_$q.err" || { tail -20 "$OUT/b_${g}_$q.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${g}_$q.json')); print('nograph=$g q=$q', d['value'], d['nodes_total'], d['rewires_total'])"
  done
done
echo graph-done
