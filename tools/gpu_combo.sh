set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "[tests] $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
echo "[ab] $(date +%T)"
timeout -k 10 600 python -u tools/ab_run.py gpurun_out/r03_s4_ab.json base: tiny:CAPJWT_LIB=cap_amd/ab_tiny.so wpc12:CAPJWT_EC_WAVES_PER_CU=12 wpc16:CAPJWT_EC_WAVES_PER_CU=16 pack64:CAPJWT_LIB=cap_amd/ab_pack64.so || { echo AB_FAIL; exit 1; }
echo "[profile] $(date +%T)"
timeout -k 10 1100 bash tools/gpu_profile_cfg.sh r03_s4_cfg
