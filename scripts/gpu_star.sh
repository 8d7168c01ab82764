#!/bin/bash
# RRT* (config 5) on the box: parity tests, the bench line (8192 queries and a 1024-query shard),
# and a kernel trace + stats of a short run.  Every GPU step has its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/star"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rrtstar.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python3 bench.py --workload config5 ${BENCH_ARGS:-} > "$OUT/bench_config5.json" 2> "$OUT/bench_config5.err" || { tail -20 "$OUT/bench_config5.err"; exit 1; }
cat "$OUT/bench_config5.json"
timeout -k 10 300 python3 bench.py --workload config5 --queries 1024 --no-cpu-baseline > "$OUT/bench_config5_shard1024.json" 2> "$OUT/bench_config5_shard.err" || { tail -20 "$OUT/bench_config5_shard.err"; exit 1; }
cat "$OUT/bench_config5_shard1024.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace5" -o run -- python3 "$R/bench.py" --workload config5 --steps 400 --no-cpu-baseline > "$OUT/trace5.log" 2>&1 || exit $?
echo star-done
