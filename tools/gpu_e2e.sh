# host-layer change check: KeySet/Validator GPU parity, then the e2e phase probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_keyset.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_e2e.log; exit 1; }
tail -1 gpurun_out/pytest_e2e.log
timeout -k 10 300 python -u tools/e2e_probe.py > gpurun_out/e2e_probe.log 2>&1 || { echo PROBE_FAIL; tail -30 gpurun_out/e2e_probe.log; exit 1; }
grep -v "^\[capjwt\] verify \(plan\|pack\|gpu\|verdicts\) .* 0\.\|^\[capjwt\] .*  0\.[0-9][0-9] ms" gpurun_out/e2e_probe.log | tail -40
