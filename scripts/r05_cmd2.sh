# round 5: gen-stream A/B + tests + stamps + config3 + shard trace (one GPU call)
TAG=r05c TESTS=all BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05gen WLS="config2 config4" VARIANTS="base nogen" REPS="1 2" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh && \
mkdir -p gpurun_out/r05sp3 && PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/span3/libpathplanning_amd.so timeout -k 10 300 python -u bench.py --workload config2 --no-cpu-baseline --no-size-sweep --allow-variant-lib --detail gpurun_out/r05sp3/detail.json > gpurun_out/r05sp3/c2.json 2> gpurun_out/r05sp3/c2.err && \
TAG=r05ab2 WLS=config3 VARIANTS="base" REPS="1" EXTRA="--queries 1024" SFX=_q1024 bash scripts/gpu_ab.sh && \
TAG=r05tr3 RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c2|base|--workload config2 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_trace_var.sh && \
TAG=r05pmc WLS="config2" bash scripts/gpu_pmc.sh
