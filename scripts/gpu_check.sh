#!/bin/bash
# One GPU check: the -m gpu tests (or the files given in TESTS), then a bench line (BENCH_ARGS),
# each under its own time limit; everything under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT="gpurun_out/${TAG:-check}"
mkdir -p "$OUT"
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}
  [ "$T" = "all" ] && T=tests
  timeout -k 10 500 python -u -m pytest $T -x -q -m gpu --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
if [ "${BENCH_ARGS:-none}" != "none" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  echo bench-ok
fi
if [ "${BENCH2_ARGS:-none}" != "none" ]; then
  timeout -k 10 600 python -u bench.py $BENCH2_ARGS > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { tail -30 "$OUT/bench2.err"; exit 1; }
  echo bench2-ok
fi
