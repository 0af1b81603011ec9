# round-2 check: environment probe, GPU parity suite, bench with the e2e trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{ echo "nproc $(nproc)"; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null | sed 's/^/cpu.max /'; lscpu | grep -E "Model name|^CPU\(s\)|Socket|Thread";
  (go version 2>&1 || true); free -g | head -2; } > gpurun_out/env.txt 2>&1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -2
CAPJWT_TRACE=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench.json'))
print('es256',d['value']/1e6, d['kernel_ms']); print('pcie', json.dumps(d['pcie'])); print('e2e', json.dumps(d['e2e']))
print('rs256',d['rs256']['value']/1e6)
for k,v in d['configs'].items(): print(k, v['value']/1e6, v.get('error'))
"
