#!/bin/bash
# Kernel trace of a short default bench run (+ the per-window timeline), optional resolve stamps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/trace"
mkdir -p "$OUT"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest.log" 2>&1; rc=$?
  tail -5 "$OUT/pytest.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python3 scripts/stamps_resolve.py > "$OUT/stamps.txt" 2>&1 || { tail -20 "$OUT/stamps.txt"; exit 1; }
  cat "$OUT/stamps.txt"
fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms/step',d['ms_per_step'],'scan ms',d['roofline']['avg_launch_ms'],'frac',d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/k" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-} > "$OUT/trace.log" 2>&1 || exit $?
python3 "$R/scripts/timeline.py" "$OUT/k/run_kernel_trace.csv"
echo trace-done
