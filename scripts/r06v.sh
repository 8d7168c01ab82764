# round 6: the shard lines at the final library, now with their counter traffic (config3_q1024)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06v
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload config3 --queries 1024 --detail $OUT/detail_c3s.json > $OUT/bench_config3_shard1024.json 2> $OUT/c3s.err || { tail -30 $OUT/c3s.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload config5 --queries 1024 --detail $OUT/detail_c5s.json > $OUT/bench_config5_shard1024.json 2> $OUT/c5s.err || { tail -30 $OUT/c5s.err; exit 1; }
echo shards-ok
