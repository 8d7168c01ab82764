# round 6: dead stored-pd path and its buffers removed, list-order walk verdicts — the -m gpu
# suite, A/B against the previous library (lib/pre), the config-3 walk's WRITE_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06n2
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06n2/pytest.log 2>&1 || { tail -30 gpurun_out/r06n2/pytest.log; exit 1; }
tail -2 gpurun_out/r06n2/pytest.log
TAG=r06n2 REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|pre|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|pre|--workload config3 --no-cpu-baseline" bash scripts/gpu_runs.sh
TAG=r06npmc2 WLS="config3" bash scripts/gpu_pmc.sh
