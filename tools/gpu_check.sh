# GPU check: parity tests (a named subset first when given), then the benchmark
# (run via gpurun from the repo root):  bash tools/gpu_check.sh [first-test-file]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 300 python -u -m pytest $1 -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_first.log 2>&1 || { echo PYTEST_FIRST_FAIL; tail -40 gpurun_out/pytest_first.log; exit 1; }
  tail -1 gpurun_out/pytest_first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -2
if [ "${NOBENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json || true
