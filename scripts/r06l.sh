# round 6: s_classify's disc tests in f32 (from the cull records) — the -m gpu suite, then A/B
# against the previous library (lib/pre) on the shard, config 3 (+ its batch plan) and config 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/r06l/pytest.log 2>&1 || { tail -30 gpurun_out/r06l/pytest.log; exit 1; }
tail -2 gpurun_out/r06l/pytest.log
TAG=r06l REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|pre|--workload config3 --queries 1024 --no-cpu-baseline;c3|base|--workload config3 --no-cpu-baseline;c3|pre|--workload config3 --no-cpu-baseline;c5|base|--workload config5 --no-cpu-baseline;c5|pre|--workload config5 --no-cpu-baseline" bash scripts/gpu_runs.sh
