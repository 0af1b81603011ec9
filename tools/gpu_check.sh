# GPU check: parity tests, then the benchmark (run via gpurun from the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -2
if [ "${NOBENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
