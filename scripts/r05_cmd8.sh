# round 5: window kernel at 2 workgroups per CU — full GPU suite + A/B (config 2 / 4 / polygons / config 1)
TAG=r05g TESTS=all BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05wg WLS="config2 config4" VARIANTS="base pre2wg" REPS="1 2" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh && \
TAG=r05wg WLS="polygons config1" VARIANTS="base pre2wg" REPS="1" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh
