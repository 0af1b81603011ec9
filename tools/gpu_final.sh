# the driver's round-end sequence on one box: GPU parity suite, smoke(), default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest_final.log | head -20; tail -30 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_final.err; exit 1; }
python tools/bench_summary.py gpurun_out/bench_final.json
