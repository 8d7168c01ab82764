#!/bin/bash
# Kernel timelines of every library variant under rs-pathplanning_amd/lib/v_*/ (short default
# bench under rocprofv3, one run each; VARIANTS="a b" to restrict).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/var"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="--steps 20 --warmup 3 --no-cpu-baseline --no-size-sweep ${BENCH_ARGS:-}"
for d in "$R"/rs-pathplanning_amd/lib/v_*/; do
  v=$(basename "$d"); v=${v#v_}
  if [ -n "$VARIANTS" ] && [[ " $VARIANTS " != *" $v "* ]]; then continue; fi
  export PP_AMD_LIB="$d/libpathplanning_amd.so"
  timeout -k 10 300 python3 "$R/bench.py" $A > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v bench failed"; tail -5 "$OUT/$v.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d "$OUT/$v" -o run -- python3 "$R/bench.py" $A > "$OUT/$v.log" 2>&1 || exit $?
  echo "== $v: $(python3 -c "import json;d=json.load(open('$OUT/$v.json'));print('it/s',d['value'],'ms/win',d['ms_per_step'],'scan ms',d['roofline']['avg_launch_ms'])")"
  python3 "$R/scripts/timeline.py" "$OUT/$v/run_kernel_trace.csv" | tail -7
done
echo variants-done
