# Round-4 session H: blocked plan fill -- runtime / keyset / edge tests, then
# the configs[4] stream and the ES256 pipelined line with the blocked and the
# one-level (CAPJWT_PLAN_FILL=wave) plan fill.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_keyset.py tests/test_gpu_edges.py tests/test_gpu_keyload.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_h.log; exit 1; }
tail -n 1 gpurun_out/pytest_h.log
for m in blocked wave blocked; do
  CAPJWT_PLAN_FILL=$m timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/pf_$m.json 4 524288 262144 > gpurun_out/pf_$m.txt 2>&1 || { echo ST_FAIL; tail -30 gpurun_out/pf_$m.txt; exit 1; }
  echo "$m:"; cat gpurun_out/pf_$m.txt
done
