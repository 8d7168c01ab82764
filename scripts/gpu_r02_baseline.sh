#!/bin/bash
# Round-2 first GPU check (repo root on the box): GPU parity tests, the default bench line, a
# kernel trace of config 2 and two SQ counter passes on window_kernel (the NN screen), each pass
# its own rocprofv3 run (counters never share a pass with tracing).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/r02a"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
A="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $A > "$OUT/trace.log" 2>&1 || exit $?
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_SCA"
i=0
for grp in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -T -f csv --kernel-include-regex window_kernel -d "$OUT/pmc/p$i" -o run -- python3 "$R/bench.py" $A > "$OUT/pmc_p$i.log" 2>&1 || { tail -5 "$OUT/pmc_p$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_kernels.py" "$OUT/pmc" 20
echo r02a-done
