# round-2: GPU parity suite, then a quick bench A/B of the P-256 key table budget (W = 26 vs 24)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
Q="--no-cpu --no-e2e --no-configs --no-ab --no-rs256"
for gb in 110 32; do
  timeout -k 10 300 python -u bench.py $Q --table-budget-gb $gb > gpurun_out/bench_tb$gb.json 2> gpurun_out/bench_tb$gb.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_tb$gb.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_tb$gb.json')); print('budget=$gb', d['config']['p256_key_comb_w'], round(d['value']/1e6,1), 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), {k: round(v,4) for k,v in d['kernel_ms'].items()})"
done
