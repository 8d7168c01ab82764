set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1 || { tail -30 gpurun_out/r03a/pytest.log; exit 1; }
tail -3 gpurun_out/r03a/pytest.log
timeout -k 10 500 python -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { tail -30 gpurun_out/r03a/bench.err; exit 1; }
echo bench-ok
