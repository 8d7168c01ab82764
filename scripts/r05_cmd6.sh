# round 5: nn_finalize pair search by sorted position — parity tests + A/B
TAG=r05e TESTS="tests/test_gpu_parity.py tests/test_gpu_fullsize.py" BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05pair WLS="config2 config4" VARIANTS="base prepair" REPS="1 2" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh
