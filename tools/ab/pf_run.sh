# Prefetching point chains (JG_EC_PF_MAX / JG_ED_PF_MAX): parity at the launch
# sizes that take them, then A/Bs against a library built with both at 0.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export AB_REPS=2 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_comb_tiers.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1 && tail -2 gpurun_out/pf_tests.log && \
AB_N=38912 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf_ed38k.json base=cap_amd/ab_pf0.so pf=cap_amd/libcapjwt.so > gpurun_out/pf.txt 2>&1 && \
AB_ALG=ES384 AB_N=62464 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf_p384_62k.json base=cap_amd/ab_pf0.so pf=cap_amd/libcapjwt.so >> gpurun_out/pf.txt 2>&1 && \
cat gpurun_out/pf.txt && \
for v in base:ab_pf0 pf:libcapjwt; do CAPJWT_LIB=$GRAFT_REPO_ROOT/cap_amd/${v#*:}.so timeout -k 10 500 python3 -u bench.py --configs-only --no-ab --no-refresh --no-cpu --no-e2e --stream-chunks 262144 --steps 10 --warmup 3 --detail gpurun_out/cfg_${v%%:*}_detail.json > gpurun_out/cfg_${v%%:*}.json 2> gpurun_out/cfg_${v%%:*}.err || exit 1; done; python3 tools/ab/cfg_compare.py base=gpurun_out/cfg_base.json pf=gpurun_out/cfg_pf.json
