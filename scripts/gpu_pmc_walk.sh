#!/bin/bash
# Stall-side counter passes of one kernel under a bench workload (each pass its own rocprofv3 run):
# instruction-cache traffic, wait / issue / level counters.  KERNEL, ARGS, TAG.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-pmcw}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
K=${KERNEL:-steer_walk}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH"
P2="SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
P3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_TRANS_F64"
P4="SQ_WAVES SQC_DCACHE_REQ SQC_DCACHE_MISSES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_BUSY_CYCLES SQ_IFETCH_LEVEL"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P -T -f csv --kernel-include-regex "$K" -d "$OUT/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "FAILED p$i"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "ok p$i"
done
