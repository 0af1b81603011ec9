# Where the prefetching chain stops paying: 262 k-token ES256 / ES384
# launches, plain k_ec_point (HEAD) vs the PF chain (ab_pf0.so:
# -DJG_EC_PF_MAX=524288); then the mid-launch parity tests at HEAD
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export AB_REPS=2 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_comb_tiers.py -m gpu -x -q -k mid_launch --timeout 200 --timeout-method thread > gpurun_out/pf4_tests.log 2>&1 && tail -1 gpurun_out/pf4_tests.log && \
AB_ALG=ES256 AB_N=262144 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf4_p256.json plain=cap_amd/libcapjwt.so pf=cap_amd/ab_pf0.so > gpurun_out/pf4.txt 2>&1 && \
AB_ALG=ES384 AB_N=262144 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf4_p384.json plain=cap_amd/libcapjwt.so pf=cap_amd/ab_pf0.so >> gpurun_out/pf4.txt 2>&1; cat gpurun_out/pf4.txt
