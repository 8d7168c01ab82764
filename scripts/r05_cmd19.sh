# batch window re-check with the active-task list: the shard at K = 16 / 32 / 64, the batch at 16 / 32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05kw
mkdir -p $OUT
for rep in 1 2; do
  for k in 16 32 64; do
    timeout -k 10 300 python -u bench.py --workload config3 --queries 1024 --batch-window $k --no-cpu-baseline > $OUT/shard_k${k}_$rep.json 2> $OUT/shard_k${k}_$rep.err || { tail -20 $OUT/shard_k${k}_$rep.err; exit 1; }
  done
  for k in 16 32; do
    timeout -k 10 300 python -u bench.py --workload config3 --batch-window $k --no-cpu-baseline > $OUT/full_k${k}_$rep.json 2> $OUT/full_k${k}_$rep.err || { tail -20 $OUT/full_k${k}_$rep.err; exit 1; }
  done
  echo rep $rep
done
# (second use, after the default became 32: the full batch at K = 64)
