# Ed25519 prep occupancy A/B on BASELINE configs[3] (default = k_prep_ed at 3 waves/SIMD, edw2 = compiler's 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ed.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_ed.log; exit 1; }
tail -1 gpurun_out/pytest_ed.log
for v in default edw2 default edw2; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u tools/config_probe.py eddsa_es384 > gpurun_out/ed_$v.json 2> gpurun_out/ed_$v.err || { echo PROBE_FAIL $v; tail -20 gpurun_out/ed_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/ed_$v.json)"
done
