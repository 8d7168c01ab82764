# round 6: each steer round's launches sized by a depth-histogram bound on its tasks (no empty
# second chunk, small grids in the late rounds) — batch-plan tests, then A/B against lib/pre
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06x
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch_plan.py tests/test_gpu_multirank.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06x/pytest.log 2>&1 || { tail -30 gpurun_out/r06x/pytest.log; exit 1; }
tail -2 gpurun_out/r06x/pytest.log
TAG=r06x REPS="1 2 3" RUNS="c3|base|--workload config3 --no-cpu-baseline;c3|pre|--workload config3 --no-cpu-baseline" bash scripts/gpu_runs.sh
