#!/bin/bash
# The round's record: the -m gpu suite, the default bench line, the 1024-query shard lines of
# configs 3 and 5 (with their CPU baselines); everything under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-final}"
mkdir -p "$OUT"
if [ "${TESTS:-all}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
echo bench-default-ok
timeout -k 10 300 python -u bench.py --workload config3 --queries 1024 > "$OUT/bench_config3_shard1024.json" 2> "$OUT/bench_config3_shard1024.err" || { tail -30 "$OUT/bench_config3_shard1024.err"; exit 1; }
echo shard3-ok
timeout -k 10 300 python -u bench.py --workload config5 --queries 1024 > "$OUT/bench_config5_shard1024.json" 2> "$OUT/bench_config5_shard1024.err" || { tail -30 "$OUT/bench_config5_shard1024.err"; exit 1; }
echo shard5-ok
