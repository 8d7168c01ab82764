# round 6: counter passes at the final library, part 1 (the batch workloads incl. the shard)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06pmcF WLS="config3 config3s config5" bash scripts/gpu_pmc.sh
