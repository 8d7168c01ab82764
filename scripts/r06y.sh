# round 6: the window walk with the analytic S classes (variant lib/wks) — parity file on the
# variant, then A/B on configs 2, 4 and polygons
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06y
PP_AMD_LIB=$PWD/rs-pathplanning_amd/lib/wks/libpathplanning_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_polygons.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06y/pytest_wks.log 2>&1 || { tail -30 gpurun_out/r06y/pytest_wks.log; exit 1; }
tail -1 gpurun_out/r06y/pytest_wks.log
TAG=r06y REPS="1 2 3" RUNS="c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|wks|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep;c4|wks|--workload config4 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_runs.sh
