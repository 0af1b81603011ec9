# Ed25519 two-lane prefetching split at configs[4]'s launch size: full GPU
# suite at HEAD, then the A/B against the one-lane prefetching kernel
# (ab_pf0.so: -DJG_ED_SPLIT2_PF_MAX=0), then the configs lines.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export AB_REPS=2 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log && \
AB_N=38912 timeout -k 10 400 python3 -u tools/ab/point_ab.py gpurun_out/pf2_ed38k.json s1pf=cap_amd/ab_pf0.so s2pf=cap_amd/libcapjwt.so > gpurun_out/pf2.txt 2>&1 && \
cat gpurun_out/pf2.txt && \
timeout -k 10 500 python3 -u bench.py --configs-only --no-ab --no-refresh --no-cpu --no-e2e --stream-chunks 262144 --steps 10 --warmup 3 --detail gpurun_out/cfg_head_detail.json > gpurun_out/cfg_head.json 2> gpurun_out/cfg_head.err && \
python3 tools/ab/cfg_compare.py head=gpurun_out/cfg_head.json
