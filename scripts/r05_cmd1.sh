TAG=r05b TESTS=all BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05tr RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2split|splitres|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_trace_var.sh && \
TAG=r05ab WLS=config3 VARIANTS="base w5" REPS="1 2" bash scripts/gpu_ab.sh && \
TAG=r05ab WLS=config3 VARIANTS="base w5" REPS="1 2" EXTRA="--queries 1024" SFX=_q1024 bash scripts/gpu_ab.sh
