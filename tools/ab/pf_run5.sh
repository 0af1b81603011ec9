# The prefetching loop inside the small-launch (<= 16 k tokens) split kernels:
# lone-batch latency of the chain at 256 / 4096 / 16384 tokens, HEAD vs
# ab_spf.so (-DJG_EC_SPLIT_PF=1 -DJG_ED_SPLIT_PF=1); parity of the variant first
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export SBP_SIZES=256,2048,8000 && \
true && \
for alg in ES256 EdDSA; do for v in head:libcapjwt spf:ab_spf; do echo "== $alg ${v%%:*}"; CAPJWT_LIB=$GRAFT_REPO_ROOT/cap_amd/${v#*:}.so timeout -k 10 200 python3 -u tools/small_batch_probe.py gpurun_out/pf5_${alg}_${v%%:*}.json 1 $alg 2>&1 | tail -3 || exit 1; done; done
