# point-kernel prefetch: GPU parity suite on the default build, then bench A/B of library variants
# (base = no prefetch, pf3 = prefetch at 3 waves/SIMD, default = prefetch forced to 4 waves/SIMD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -1
Q="--no-cpu --no-e2e --no-configs --no-ab --no-rs256 --steps 20"
for v in base pf3 default base pf3 default; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u bench.py $Q > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo BENCH_FAIL $v; tail -30 gpurun_out/bench_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$v.json')); print('$v', round(d['value']/1e6,1), 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), {k: round(v,4) for k,v in d['kernel_ms'].items()})"
done
