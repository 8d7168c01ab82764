#!/bin/bash
# config 5 and polygons across grid-only LDS image budgets (PP_LDS_GRID_KB)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/ldsgrid"
mkdir -p "$OUT"
cd "$R"
for kb in ${KBS:-64 40 28 16}; do
  for w in config5 polygons; do
    PP_LDS_GRID_KB=$kb timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-size-sweep > "$OUT/b_${kb}_$w.json" 2> "$OUT/b_${kb}_$w.err" || { tail -20 "$OUT/b_${kb}_$w.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${kb}_$w.json')); print('kb=$kb $w', d['value'])"
  done
done
echo lds-done
