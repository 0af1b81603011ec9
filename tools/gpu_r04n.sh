# Round-4 session N: host batch-array block cache -- keyset / validator GPU
# tests, then the e2e leg twice (bench.py with the other lines off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_keyset.py tests/test_gpu_edges.py tests/test_oidc_hash.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_n.log; exit 1; }
tail -n 1 gpurun_out/pytest_n.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-rs256 --no-configs --no-cpu --no-ab > gpurun_out/e2e_$i.json 2> gpurun_out/e2e_$i.err || { echo BENCH_FAIL; tail -20 gpurun_out/e2e_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_$i.json').read().strip().splitlines()[-1]); e=d['e2e']; print(round(e['value']/1e6,2), e['phases_ms_last_pass'])"
done
