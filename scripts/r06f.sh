set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06f RUNS="c2b|base|--workload config2 --no-cpu-baseline --no-size-sweep;c2p|prevfin|--workload config2 --no-cpu-baseline --no-size-sweep;c3sb|base|--workload config3 --queries 1024 --no-cpu-baseline;c3sp|prevnn|--workload config3 --queries 1024 --no-cpu-baseline" bash scripts/gpu_trace_var.sh && \
TAG=r06f REPS="1 2" RUNS="c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c3s|prevnn|--workload config3 --queries 1024 --no-cpu-baseline" bash scripts/gpu_runs.sh
