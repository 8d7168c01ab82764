#!/bin/bash
# A/B of the working tree's library against lib/v_base (the last commit's): the GPU suite on the
# new one, then the config-2 line (no sub-results, no CPU leg) alternated 3x.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/ab"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2 3; do
  for v in new base; do
    if [ $v = base ]; then export PP_AMD_LIB="$R/rs-pathplanning_amd/lib/v_base/libpathplanning_amd.so"; else unset PP_AMD_LIB; fi
    timeout -k 10 300 python3 bench.py --no-sub --no-size-sweep --no-cpu-baseline --allow-variant-lib ${BENCH_ARGS:-} > "$OUT/b_${v}_$rep.json" 2> "$OUT/b_${v}_$rep.err" || { tail -20 "$OUT/b_${v}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${v}_$rep.json')); print('$v', round(d['value']/1e6,2), 'M it/s', d['ms_per_step'], 'window_kernel', d['roofline']['avg_launch_ms'])"
  done
done
echo ab-done
