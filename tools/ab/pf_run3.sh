# P-256 at configs[4]'s class size: two-lane prefetching split (HEAD) vs the
# one-lane prefetching chain (ab_pf0.so: -DJG_EC_SPLIT2_P256=16384)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export AB_REPS=2 && \
AB_ALG=ES256 AB_N=62464 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf3_p256_62k.json s2pf=cap_amd/libcapjwt.so s1pf=cap_amd/ab_pf0.so > gpurun_out/pf3.txt 2>&1 && \
AB_ALG=ES256 AB_N=124928 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf3_p256_125k.json s2pf=cap_amd/libcapjwt.so s1pf=cap_amd/ab_pf0.so >> gpurun_out/pf3.txt 2>&1; cat gpurun_out/pf3.txt
