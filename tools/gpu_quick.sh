set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench.json'))
print('es256',d['value']/1e6, d['kernel_ms']); print('rs256',d['rs256']['value']/1e6,d['rs256']['kernel_ms'],d['rs256']['roofline']['frac'])
for k,v in d['configs'].items(): print(k, v['value']/1e6, {a:b for a,b in v['kernel_ms'].items() if 'modexp' in a})
"
