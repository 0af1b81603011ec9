# Ed25519 finish occupancy A/B on configs[3] (default = 3 waves/SIMD, edf2 = compiler's 2), plus the GPU Ed tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_edf.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_edf.log; exit 1; }
tail -1 gpurun_out/pytest_edf.log
for v in default edf2 default edf2; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u tools/config_probe.py eddsa_es384 > gpurun_out/edf_$v.json 2> gpurun_out/edf_$v.err || { echo PROBE_FAIL $v; tail -20 gpurun_out/edf_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/edf_$v.json')); print('$v', round(d['value']/1e6,1), {k: round(v,4) for k,v in d['kernel_ms'].items() if 'ed' in k})"
done
