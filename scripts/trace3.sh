#!/bin/bash
# kernel trace of the config-3 bench (short run)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/trace3"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --workload config3 --steps 400 > "$OUT/trace.log" 2>&1 || exit $?
echo trace3-done
