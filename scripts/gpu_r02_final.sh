#!/bin/bash
# Round record: GPU tests, smoke, the default bench line (what the driver runs) and its kernel
# trace (rocprofv3 --kernel-trace --stats, no counters), outputs under gpurun_out/$TAG.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-final}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
echo smoke-ok
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('value', d['value'], 'frac', d['roofline']['frac'])"
[ -n "$NO_TRACE" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace_default" -o run -- python3 "$R/bench.py" > "$OUT/trace_default.log" 2>&1 || { tail -5 "$OUT/trace_default.log"; exit 1; }
echo final-done
