# round 5: packed-FMA screen — GPU tests, then A/B against the scalar screen (config 2 / 4)
TAG=r05d TESTS=all BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05pk WLS="config2 config4" VARIANTS="base scalarscreen" REPS="1 2" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh
