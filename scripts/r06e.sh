set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06e
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -40 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
rm -f gpurun_out/fin_stamps.txt
TAG=r06e REPS="1" RUNS="c2|finst2|--workload config2 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_runs.sh
mv gpurun_out/fin_stamps.txt gpurun_out/r06e/fin_stamps.txt
TAG=r06e REPS="1 2" RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|prevfin|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep;c4|prevfin|--workload config4 --no-cpu-baseline --no-size-sweep;c3|base|--workload config3 --no-cpu-baseline;c3|prevfin|--workload config3 --no-cpu-baseline" bash scripts/gpu_runs.sh
