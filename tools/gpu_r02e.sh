# round-2: GPU parity suite, then a quick ES256 bench A/B (CAPJWT_MIDSTATE on / off), then the e2e probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
Q="--no-cpu --no-e2e --no-configs --no-ab"
timeout -k 10 300 python -u bench.py $Q > gpurun_out/bench_mid1.json 2> gpurun_out/bench_mid1.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_mid1.err; exit 1; }
CAPJWT_MIDSTATE=0 timeout -k 10 300 python -u bench.py $Q > gpurun_out/bench_mid0.json 2> gpurun_out/bench_mid0.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_mid0.err; exit 1; }
for f in gpurun_out/bench_mid1.json gpurun_out/bench_mid0.json; do python -c "
import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e6,1), {k: round(v,4) for k,v in d['kernel_ms'].items()}, 'rs256', round(d['rs256']['value']/1e6,1), d['rs256'].get('kernel_ms'))"; done
timeout -k 10 300 python -u tools/e2e_probe.py > gpurun_out/e2e_probe.log 2>&1 || { echo PROBE_FAIL; tail -30 gpurun_out/e2e_probe.log; exit 1; }
tail -1 gpurun_out/e2e_probe.log
