#!/bin/bash
# Config 3 on a 1024-query shard (the per-GPU share at 8 GPUs): bench lines for several windows
# and a kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/c3"
mkdir -p "$OUT"
cd "$R"
for k in ${KS:-0 8 32}; do
  timeout -k 10 300 python3 bench.py --workload config3 --queries 1024 --batch-window $k --no-cpu-baseline > "$OUT/bench_k$k.json" 2> "$OUT/bench_k$k.err" || { tail -20 "$OUT/bench_k$k.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k$k.json')); print('K=$k', d['value'], d['ms_per_step'], d['nodes_total'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --workload config3 --queries 1024 --steps 400 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit $?
echo c3-done
