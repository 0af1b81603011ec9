# RSA-3K modexp occupancy A/B (default = k_rsa_modexp_3k at 3 waves/SIMD, r3kw2 = compiler's 2), then the GPU RSA suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rsa.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r3k.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_r3k.log; exit 1; }
tail -1 gpurun_out/pytest_r3k.log
for v in default r3kw2 default r3kw2; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u tools/config_probe.py rs256_3072 > gpurun_out/r3k_$v.json 2> gpurun_out/r3k_$v.err || { echo PROBE_FAIL $v; tail -20 gpurun_out/r3k_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r3k_$v.json)"
done
