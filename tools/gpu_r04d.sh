# Round-4 session D (run via gpurun from the repo root): the whole -m gpu
# suite at HEAD (2-lane RSA-3K, deferred exact kernels, plan fill on the
# least-loaded group lane), the configs[4] stream A/B (plan-fill stream,
# zero-copy plans), and the RSA-3K layout / occupancy A/B by class cost.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
tail -n 1 gpurun_out/pytest.log
echo "[stream A/B] $(date +%T)"
timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/st_least.json 4 524288 262144 z0 > gpurun_out/st_least.txt 2>&1 || { echo ST_FAIL; tail -30 gpurun_out/st_least.txt; exit 1; }
cat gpurun_out/st_least.txt
CAPJWT_GROUP_CTRL=join timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/st_join.json 4 524288 262144 > gpurun_out/st_join.txt 2>&1 || { echo ST_FAIL; tail -30 gpurun_out/st_join.txt; exit 1; }
echo "join:"; cat gpurun_out/st_join.txt
CAPJWT_GROUP_CTRL=copy timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/st_copy.json 4 524288 262144 > gpurun_out/st_copy.txt 2>&1 || { echo ST_FAIL; tail -30 gpurun_out/st_copy.txt; exit 1; }
echo "copy:"; cat gpurun_out/st_copy.txt
echo "[rsa3k] $(date +%T)"
for v in base r3k_g4 r3k_g2w1; do
  if [ $v = base ]; then lib=""; else lib="CAPJWT_LIB=$PWD/cap_amd/ab_$v.so"; fi
  env $lib timeout -k 10 300 python3 -u tools/class_costs.py gpurun_out/r3k_$v.json rsa3072 > gpurun_out/r3k_$v.txt 2>&1 || { echo "R3K_FAIL $v"; tail -20 gpurun_out/r3k_$v.txt; exit 1; }
  echo "$v: $(tr '\n' ' ' < gpurun_out/r3k_$v.txt)"
done
