# Round-4 session C (run via gpurun from the repo root): zero-copy gather
# plans -- runtime tests, configs[4] stream A/B -- then the whole -m gpu
# suite, the prep A/B (32-bit window bases vs the round-3 prep) on the ES256
# line and the RSA-3K 2-lane layout A/B on the config lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_zc.sh || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
tail -n 1 gpurun_out/pytest.log
echo "[prep A/B] $(date +%T)"
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_prep32_ab.json 'prep32:' 'prep_r03:CAPJWT_LIB=cap_amd/ab_prepold.so' 'prep32_b:' 'prep_r03_b:CAPJWT_LIB=cap_amd/ab_prepold.so' || exit 1
echo "[rsa3k g2 A/B on configs] $(date +%T)"
timeout -k 10 500 python3 tools/ab_run.py gpurun_out/r04_r3k_g2_ab.json 'g4:' 'g2:CAPJWT_LIB=cap_amd/ab_r3k_g2.so' -- --configs-only --steps 6 --warmup 2 --no-ab --no-refresh || exit 1
echo "[scalar occupancy A/B] $(date +%T)"
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_scalar_ab.json 'wpc8:' 'wpc12:CAPJWT_EC_WAVES_PER_CU=12' 'w4_wpc16:CAPJWT_LIB=cap_amd/ab_sc4w.so,CAPJWT_EC_WAVES_PER_CU=16' 'w4_wpc12:CAPJWT_LIB=cap_amd/ab_sc4w.so,CAPJWT_EC_WAVES_PER_CU=12' 'wpc8_b:' || exit 1
