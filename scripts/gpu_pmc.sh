#!/bin/bash
# SQ / GRBM counters of one kernel (KERNEL regex, default window_kernel) over a short default
# bench, one rocprofv3 pass per counter group (counters never share a pass with tracing).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-}"
K="${KERNEL:-window_kernel}"
i=0
GROUPS=${GROUPS:-"GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES|SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU|SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM|SQ_WAIT_ANY SQ_INSTS_LDS SQ_INST_CYCLES_VMEM|FETCH_SIZE|WRITE_SIZE"}
IFS='|' read -ra GRPS <<< "$GROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -T -f csv --kernel-include-regex "$K" -d "$OUT/p$i" -o run -- python3 "$R/bench.py" $A > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_summary.py" "$OUT" "$K"
echo pmc-done
