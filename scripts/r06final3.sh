# round 6, final: the record at the final library (the -m gpu suite, the default line, the shards,
# per-workload traces); the counter passes follow in scripts/r06pmcG.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
FTAG=r06final3 TTAG=r06final3_trace bash scripts/gpu_record.sh
