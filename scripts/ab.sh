#!/bin/bash
# A/B: default library vs lib/variant (same bench), plus SQ counters of nn_scan (default).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/ab"
mkdir -p "$OUT"
cd "$R"
A="--steps 30 --warmup 3 --no-cpu-baseline --no-size-sweep"
timeout -k 10 300 python3 bench.py $A > "$OUT/a.json" 2> "$OUT/a.err" || exit 1
PP_AMD_LIB="$R/rs-pathplanning_amd/lib/variant/libpathplanning_amd.so" timeout -k 10 300 python3 bench.py $A > "$OUT/b.json" 2> "$OUT/b.err" || exit 1
timeout -k 10 300 python3 bench.py $A > "$OUT/a2.json" 2> "$OUT/a2.err" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -T -f csv --kernel-include-regex nn_scan -d "$OUT/pmc" -o run -- python3 "$R/bench.py" $A > "$OUT/pmc.log" 2>&1 || exit $?
echo ab-done
