# P-384 key comb W = 24 tier: GPU parity suite, configs[3] A/B (default budget: W = 24; 1.5 GiB: W = 20), full bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
for v in w24 w20 w24 w20; do
  if [ $v = w20 ]; then export CAPJWT_TABLE_BUDGET_GB=1.5; else unset CAPJWT_TABLE_BUDGET_GB; fi
  timeout -k 10 300 python -u tools/config_probe.py eddsa_es384 > gpurun_out/p384_$v.json 2> gpurun_out/p384_$v.err || { echo PROBE_FAIL $v; tail -20 gpurun_out/p384_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/p384_$v.json)"
done
unset CAPJWT_TABLE_BUDGET_GB
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/bench.json
