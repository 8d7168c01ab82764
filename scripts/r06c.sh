set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06c
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06c/pytest.log 2>&1 || { tail -40 gpurun_out/r06c/pytest.log; exit 1; }
tail -2 gpurun_out/r06c/pytest.log
TAG=r06c REPS="1 2" RUNS="c3|base|--workload config3 --no-cpu-baseline;c3|lg2048|--workload config3 --no-cpu-baseline;c3|recbig|--workload config3 --no-cpu-baseline;ex|base|--workload example_rrt --no-cpu-baseline;pl|base|--workload plan --no-cpu-baseline" bash scripts/gpu_runs.sh
