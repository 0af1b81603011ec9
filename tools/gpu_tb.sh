# GPU parity suite, then the full benchmark (all legs) with its summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/bench.json
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
for k,v in d['configs'].items(): print(k, {a: round(b,4) for a,b in v['kernel_ms'].items()})"
