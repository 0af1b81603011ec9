# Round-end check at HEAD (run via gpurun from the repo root): the whole -m gpu
# suite, smoke(), then the default bench -- the driver's own sequence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
tail -n 1 gpurun_out/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json || true
