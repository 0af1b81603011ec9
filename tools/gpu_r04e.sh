# Round-4 session E: ECDSA parity after the scalar stage's one-token-ahead
# loads, then the ES256 A/B (prefetch on / off).  Run via gpurun from the repo root.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_tables.py tests/test_gpu_prep_mid.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_e.log; exit 1; }
tail -n 1 gpurun_out/pytest_e.log
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_scalar_pf_ab.json 'pf1:' 'pf0:CAPJWT_LIB=cap_amd/ab_scpf0.so' 'pf1_b:' 'pf0_b:CAPJWT_LIB=cap_amd/ab_scpf0.so' || exit 1
