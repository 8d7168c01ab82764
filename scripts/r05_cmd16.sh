# fused window prep + walk (window_prepwalk_kernel): the -m gpu suite, then A/B against lib/sep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05pw
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r05pw REPS="1 2" WLS="config2 config4 polygons" VARIANTS="base sep" EXTRA="--no-size-sweep" bash scripts/gpu_ab.sh || exit 1
TAG=r05pw REPS="1" WLS="config1 plan example_rrt" VARIANTS="base sep" bash scripts/gpu_ab.sh
