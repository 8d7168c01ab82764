#!/bin/bash
# Full GPU check on the box (repo root): parity tests, smoke, the three bench workloads, and a
# kernel trace of config 4.  Every GPU step has its own time limit; the script stops at the first
# failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/all"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for w in config2 config4 config3; do
  timeout -k 10 400 python3 bench.py --workload $w ${BENCH_ARGS:-} > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace4" -o run -- python3 "$R/bench.py" --workload config4 --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep > "$OUT/trace4.log" 2>&1 || exit $?
echo all-done
