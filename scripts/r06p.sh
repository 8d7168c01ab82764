# round 6: long tasks first in each walk workgroup — parity files, then A/B against the previous
# library (lib/pre): the shard, config 3 (+ batch plan), config 5, config 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06p
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch_plan.py tests/test_gpu_rrtstar.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06p/pytest.log 2>&1 || { tail -30 gpurun_out/r06p/pytest.log; exit 1; }
tail -2 gpurun_out/r06p/pytest.log
TAG=r06p REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|pre|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|pre|--workload config3 --no-cpu-baseline;c5|base|--workload config5 --no-cpu-baseline;c5|pre|--workload config5 --no-cpu-baseline;c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2|pre|--workload config2 --no-cpu-baseline --no-size-sweep" bash scripts/gpu_runs.sh
