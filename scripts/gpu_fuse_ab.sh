#!/bin/bash
# The fused insert + next-step NN (config 3): batch parity tests, then bench lines with the fusion
# on and off (PP_MQ_FUSE=0) for the 1024-query shard and the 8192-query batch, alternated.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/fuse"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "batch or config3 or sharded" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
 for f in 1 0; do
  for q in 1024 8192; do
   PP_MQ_FUSE=$f timeout -k 10 300 python3 bench.py --workload config3 --queries $q --no-cpu-baseline > "$OUT/b_f${f}_q${q}_$rep.json" 2> "$OUT/b_f${f}_q${q}_$rep.err" || { tail -20 "$OUT/b_f${f}_q${q}_$rep.err"; exit 1; }
   python3 -c "import json; d=json.load(open('$OUT/b_f${f}_q${q}_$rep.json')); print('fuse=$f q=$q', round(d['value']/1e6,1), 'M it/s', d['records_digest'], d['nodes_total'])"
  done
 done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" --workload config3 --queries 1024 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit $?
echo fuse-done
