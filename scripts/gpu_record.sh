# the round record (part A): the -m gpu suite, the default line (+ detail), the 1024-query shards,
# then per-workload kernel traces at the same library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${FTAG:-record}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --detail $OUT/detail_default.json > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -30 $OUT/bench_default.err; exit 1; }
echo default-ok
timeout -k 10 300 python -u bench.py --workload config3 --queries 1024 --detail $OUT/detail_c3s.json > $OUT/bench_config3_shard1024.json 2> $OUT/c3s.err || { tail -30 $OUT/c3s.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload config5 --queries 1024 --detail $OUT/detail_c5s.json > $OUT/bench_config5_shard1024.json 2> $OUT/c5s.err || { tail -30 $OUT/c5s.err; exit 1; }
echo shards-ok
TAG=${TTAG:-record_trace} RUNS="def|base|;c2|base|--workload config2 --no-cpu-baseline --no-size-sweep;c4|base|--workload config4 --no-cpu-baseline --no-size-sweep;c3|base|--workload config3 --no-cpu-baseline;c3s|base|--workload config3 --queries 1024 --no-cpu-baseline;c5|base|--workload config5 --no-cpu-baseline;ex|base|--workload example_rrt --no-cpu-baseline;pl|base|--workload plan --no-cpu-baseline" bash scripts/gpu_trace_var.sh
# per-kernel durations at the benched sizes (the last N dispatches of each kernel), then drop the
# per-dispatch trace CSVs (gpurun brings back at most 64 MiB); the --stats summaries stay
T="gpurun_out/${TTAG:-record_trace}"
python3 scripts/trace_summary.py "$T" def:20 c2:20 c4:20 c3:146 c3s:176 c5:6000 ex:207 pl:189 > "$T/kernel_durations.json"
find "$T" -name "*kernel_trace.csv" -delete
