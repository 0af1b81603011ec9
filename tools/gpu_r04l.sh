# Round-4 session L: grouped resident runs (CAPJWT_RESIDENT_GROUPS=1) --
# parity modules with it on, then the config lines with it on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CAPJWT_RESIDENT_GROUPS=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_zz_lifetime.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_l.log; exit 1; }
tail -n 1 gpurun_out/pytest_l.log
timeout -k 10 700 python3 tools/ab_run.py gpurun_out/r04_resident_groups_ab.json 'conc:' 'groups:CAPJWT_RESIDENT_GROUPS=1' 'conc_b:' 'groups_b:CAPJWT_RESIDENT_GROUPS=1' -- --configs-only --steps 8 --warmup 2 --no-ab --no-refresh || exit 1
