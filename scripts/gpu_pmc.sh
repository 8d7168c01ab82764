#!/bin/bash
# Counter passes behind the bench's rooflines (each pass its own rocprofv3 run, counters never
# beside tracing): for every (workload, kernel) the SQ instruction / wait counters and the HBM
# traffic (FETCH_SIZE, WRITE_SIZE), plus one plain bench line per workload for the normalisation
# (evals / points per launch).  Summarised by scripts/pmc_profiles.py into profiles/*.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-pmc2}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SQA="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"
SQB="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
args() {
  case $1 in
    config2|config4) echo "--workload $1 --steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep" ;;
    config3) echo "--workload $1 --warmup 3 --no-cpu-baseline --pmc-run" ;;
    config3s) echo "--workload config3 --queries 1024 --warmup 3 --no-cpu-baseline --pmc-run" ;;
    config5) echo "--workload $1 --warmup 3 --no-cpu-baseline --max-iter 600" ;;  # (PMC of 2000 steps crashed the profiler)
  esac
}
for wl in ${WLS:-config2 config4 config3 config5}; do
  timeout -k 10 300 python3 "$R/bench.py" $(args $wl) --detail "$OUT/detail_$wl.json" > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { tail -5 "$OUT/bench_$wl.err"; exit 1; }
done
job() {  # name workload kernel-regex counters...
  local name=$1 wl=$2 k=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc "$@" -T -f csv --kernel-include-regex "$k" -d "$OUT/$name" -o run -- python3 "$R/bench.py" $(args $wl) > "$OUT/$name.log" 2>&1 || { echo "FAILED $name"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "ok $name"
}
if [[ " ${WLS:-config2 config4 config3 config5} " == *" config2 "* ]]; then
  job c2_win_A config2 window_kernel $SQA
  job c2_win_B config2 window_kernel $SQB
  job c2_win_F config2 window_kernel FETCH_SIZE
  job c2_win_W config2 window_kernel WRITE_SIZE
  job c2_walk_A config2 steer_walk $SQA
  job c2_walk_B config2 steer_walk $SQB
  job c2_walk_F config2 steer_walk FETCH_SIZE
  job c2_walk_W config2 steer_walk WRITE_SIZE
fi
if [[ " ${WLS:-config2 config4 config3 config5} " == *" config4 "* ]]; then
  job c4_win_A config4 window_kernel $SQA
  job c4_win_F config4 window_kernel FETCH_SIZE
  job c4_win_W config4 window_kernel WRITE_SIZE
  job c4_walk_A config4 steer_walk $SQA
  job c4_walk_B config4 steer_walk $SQB
  job c4_walk_F config4 steer_walk FETCH_SIZE
  job c4_walk_W config4 steer_walk WRITE_SIZE
fi
if [[ " ${WLS:-config2 config4 config3 config5} " == *" config3 "* ]]; then
  job c3_walk_A config3 steer_walk $SQA
  job c3_walk_B config3 steer_walk $SQB
  job c3_walk_F config3 steer_walk FETCH_SIZE
  job c3_walk_W config3 steer_walk WRITE_SIZE
  job c3_nn_F config3 mq_sample_nn FETCH_SIZE
  job c3_nn_W config3 mq_sample_nn WRITE_SIZE
fi
if [[ " ${WLS:-config2 config4 config3 config5} " == *" config3s "* ]]; then
  job c3s_walk_A config3s steer_walk $SQA
  job c3s_walk_B config3s steer_walk $SQB
  job c3s_walk_F config3s steer_walk FETCH_SIZE
  job c3s_walk_W config3s steer_walk WRITE_SIZE
  job c3s_nn_F config3s mq_sample_nn FETCH_SIZE
  job c3s_nn_W config3s mq_sample_nn WRITE_SIZE
fi
if [[ " ${WLS:-config2 config4 config3 config5} " == *" config5 "* ]]; then
  job c5_walk_A config5 steer_walk $SQA
  job c5_walk_F config5 steer_walk FETCH_SIZE
  job c5_walk_W config5 steer_walk WRITE_SIZE
  job c5_nn_F config5 star_sample FETCH_SIZE
  job c5_nn_W config5 star_sample WRITE_SIZE
fi
echo pmc-done
