#!/bin/bash
# Round-end evidence: every bench line (CPU baselines included where the bench has one), the
# 1024-query shards of configs 3 and 5, and rocprofv3 kernel stats of configs 3 and 5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/round"
mkdir -p "$OUT"
cd "$R"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -20 "$OUT/bench_$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); print('$n', d['value'], (d.get('cpu_baseline') or {}).get('value'))"
}
run config2
run config3 --workload config3
run config3_shard1024 --workload config3 --queries 1024 --no-cpu-baseline
run config4 --workload config4 --no-cpu-baseline
run polygons --workload polygons --no-cpu-baseline
run config5 --workload config5
run config5_shard1024 --workload config5 --queries 1024 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace3" -o run -- python3 "$R/bench.py" --workload config3 --steps 400 --no-cpu-baseline > "$OUT/trace3.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace5" -o run -- python3 "$R/bench.py" --workload config5 --steps 400 --no-cpu-baseline > "$OUT/trace5.log" 2>&1 || exit $?
echo round-done
