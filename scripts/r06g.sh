set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06g
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch_plan.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06g/pytest_base.log 2>&1 || { tail -30 gpurun_out/r06g/pytest_base.log; exit 1; }
tail -2 gpurun_out/r06g/pytest_base.log
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/nocf/libpathplanning_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_batch_plan.py tests/test_gpu_api_surface.py tests/test_gpu_libm_flips.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06g/pytest_nocf.log 2>&1 || { tail -30 gpurun_out/r06g/pytest_nocf.log; exit 1; }
tail -2 gpurun_out/r06g/pytest_nocf.log
TAG=r06g REPS="1 2 3" RUNS="plan|nocf|--workload plan --no-cpu-baseline;plan|base|--workload plan --no-cpu-baseline;ex|nocf|--workload example_rrt --no-cpu-baseline" bash scripts/gpu_runs.sh
