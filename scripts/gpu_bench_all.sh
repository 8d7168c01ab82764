#!/bin/bash
# GPU tests then the bench workloads without the CPU baselines (a quick A/B of a kernel change).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/ab"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for w in ${WORKLOADS:-config2 config5 polygons config3 config4}; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-size-sweep > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d.get('nodes_total'), d.get('rewires_total'))"
done
echo ab-done
