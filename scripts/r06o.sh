# round 6: nn_finalize reads its chunk winners' f64 coordinates before the top-2 — parity files,
# then A/B against the previous library (lib/pre) on configs 2 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_libm_flips.py tests/test_gpu_api_surface.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06o/pytest.log 2>&1 || { tail -30 gpurun_out/r06o/pytest.log; exit 1; }
tail -2 gpurun_out/r06o/pytest.log
TAG=r06o REPS="1 2 3" RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|pre|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep;c4|pre|--workload config4 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_runs.sh
