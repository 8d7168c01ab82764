# round 5: check_finish without call frames — tests + A/B (plan, example_rrt, config-3 batch plan)
TAG=r05f TESTS="tests/test_gpu_api_surface.py tests/test_gpu_batch_plan.py tests/test_gpu_libm_flips.py tests/test_gpu_polygons.py" BENCH_ARGS=none bash scripts/gpu_check.sh && \
TAG=r05cf WLS="plan example_rrt" VARIANTS="base cfold" REPS="1 2" bash scripts/gpu_ab.sh && \
TAG=r05cf WLS="config3" VARIANTS="base cfold" REPS="1" EXTRA="--batch-window 0" bash scripts/gpu_ab.sh
