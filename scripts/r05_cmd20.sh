# the full batch at K = 64 against the new automatic 32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05kw2
mkdir -p $OUT
for rep in 1 2; do
  for k in 32 64; do
    timeout -k 10 300 python -u bench.py --workload config3 --batch-window $k --no-cpu-baseline > $OUT/full_k${k}_$rep.json 2> $OUT/full_k${k}_$rep.err || { tail -20 $OUT/full_k${k}_$rep.err; exit 1; }
  done
done
