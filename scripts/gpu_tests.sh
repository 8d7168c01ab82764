#!/bin/bash
# GPU parity tests only (optionally a -k filter in PYTEST_K), one process, per-test timeout.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/tests"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" "$OUT/pytest.log" | tail -60
tail -30 "$OUT/pytest.log" | grep -v PASSED
echo "pytest rc=$rc"
exit $rc
