#!/bin/bash
# Round 2: GPU parity tests (the multi-rank test included), the default bench line (config 2 +
# sub-results, CPU baselines), then the self-launched 2-rank bench on the same GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-r02b}"
mkdir -p "$OUT"
cd "$R"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
  tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -30; exit $rc; }
fi
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -z "$NO_MULTI" ]; then
  timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu-baseline > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err" || { tail -20 "$OUT/bench_g2.err"; exit 1; }
  cat "$OUT/bench_g2.json"
fi
echo bench-done
