#!/bin/bash
# A/B of runtime knobs: for each VARIANT ("NAME=VALUE[,NAME=VALUE...]" or "base"), the bench workloads in
# WORKLOADS (default: config2 config3), one line each.  Usage on the box:
#   VARIANTS="base PP_WALK_PER_CU=2 PP_WALK_PER_CU=3" bash scripts/gpu_ab_env.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
cd "$R"
for v0 in ${VARIANTS:-base}; do
  v=$(echo "$v0" | sed 's#.*/v_\([^/]*\)/lib[^,]*#\1#; s#[/=,]#_#g')
  for w in ${WORKLOADS:-config2 config3}; do
    if [ "$v0" = base ]; then envs=""; else envs="${v0//,/ }"; fi
    env $envs PP_DEBUG=1 timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-} > "$OUT/${v}_$w.json" 2> "$OUT/${v}_$w.err" || { tail -20 "$OUT/${v}_$w.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${v}_$w.json'))
r=d.get('roofline') or {}; wr=d.get('walk_roofline') or {}
print('$v $w', round(d['value']/1e6,2), 'M it/s  screen', r.get('avg_launch_ms'), ' walk', (wr or r).get('avg_launch_ms'))"
    grep "\[pp\]" "$OUT/${v}_$w.err" | sort | uniq | head -3
  done
done
echo ab-done
