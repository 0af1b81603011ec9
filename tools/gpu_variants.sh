# A/B: bench the RS256 leg of each library variant given as args (paths under cap_amd/); parity tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for V in "$@"; do
  export CAPJWT_LIB=$PWD/cap_amd/$V
  [ "${NOTEST:-0}" = 1 ] || timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$V.log 2>&1 || { echo "PYTEST_FAIL $V"; tail -30 gpurun_out/pytest_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/pytest_$V.log)"
  timeout -k 10 200 python -u bench.py --no-e2e --no-cpu $([ "${CONFIGS:-0}" = 1 ] || echo --no-configs) > gpurun_out/bench_$V.json 2> gpurun_out/bench_$V.err || { echo "BENCH_FAIL $V"; tail -30 gpurun_out/bench_$V.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/bench_$V.json'))
print('$V es256',round(d['value']/1e6,1),'rs256',round(d['rs256']['value']/1e6,1),d['rs256']['kernel_ms'])
for k,c in d.get('configs',{}).items(): print('  ',k,round(c['value']/1e6,2),{a:round(b,3) for a,b in c['kernel_ms'].items() if 'modexp' in a})"
done
