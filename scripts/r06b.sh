set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06b
timeout -k 10 120 ./scripts/micro/sincos_check > gpurun_out/r06b/sincos_check.json || { cat gpurun_out/r06b/sincos_check.json; exit 1; }
cat gpurun_out/r06b/sincos_check.json
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06b/pytest.log 2>&1 || { tail -40 gpurun_out/r06b/pytest.log; exit 1; }
tail -2 gpurun_out/r06b/pytest.log
TAG=r06b REPS="1 2" RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|ocmlsc|--workload config2 --no-cpu-baseline --no-size-sweep;c3|base|--workload config3 --no-cpu-baseline;c3|ocmlsc|--workload config3 --no-cpu-baseline;c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|ocmlsc|--workload config3 --queries 1024 --no-cpu-baseline;c5|base|--workload config5 --no-cpu-baseline;c5|ocmlsc|--workload config5 --no-cpu-baseline" bash scripts/gpu_runs.sh
