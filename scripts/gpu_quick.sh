#!/bin/bash
# Quick GPU iteration: parity tests, then the default bench line without the CPU baseline, then
# (optional, STAMPS=1) the resolve phase stamps.  Each GPU step has its own limit; stop on failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/quick"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1; rc=$?
tail -15 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$STAMPS" ]; then
  timeout -k 10 200 python3 scripts/stamps_resolve.py > "$OUT/stamps.txt" 2>&1 || { tail -20 "$OUT/stamps.txt"; exit 1; }
  cat "$OUT/stamps.txt"
fi
echo quick-done
