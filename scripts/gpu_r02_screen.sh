#!/bin/bash
# Screen-kernel iteration: GPU parity tests, the config-2 line, a kernel trace and the SQ counter
# passes of window_kernel (each rocprofv3 pass its own run).  TAG names the output directory.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-scr}"
mkdir -p "$OUT"
cd "$R"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1; rc=$?
  tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -30; exit $rc; }
fi
A="--workload ${WL:-config2} --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep"
timeout -k 10 300 python3 bench.py $A > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; w=d.get('walk_roofline') or {}
print('value', round(d['value']/1e6,2), 'M it/s; screen', r['avg_launch_ms'], 'ms', r['frac'], '; walk', w.get('avg_launch_ms'))"
[ -n "$NO_PROF" ] && { echo scr-done; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $A > "$OUT/trace.log" 2>&1 || exit $?
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS"
i=0
for grp in "$P1" "$P2" ${PMC_TRAFFIC:+FETCH_SIZE WRITE_SIZE}; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -T -f csv --kernel-include-regex "${KERNEL:-window_kernel}" -d "$OUT/pmc/p$i" -o run -- python3 "$R/bench.py" $A > "$OUT/pmc_p$i.log" 2>&1 || { tail -5 "$OUT/pmc_p$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_kernels.py" "$OUT/pmc" 20
echo scr-done
