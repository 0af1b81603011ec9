# Multi-device leg (Context([0, 0])) with and without the prefetch in the
# small-launch split kernels, alternated twice
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
for rep in 1 2; do for v in spf:libcapjwt nospf:ab_nospf; do CAPJWT_LIB=$GRAFT_REPO_ROOT/cap_amd/${v#*:}.so timeout -k 10 400 python3 -u bench.py --steps 4 --warmup 1 --no-configs --no-rs256 --no-e2e --no-cpu --no-ab --detail gpurun_out/md_${v%%:*}_$rep.json > gpurun_out/md_${v%%:*}_$rep.out 2> gpurun_out/md_${v%%:*}_$rep.err || exit 1; python3 -c "
import json;d=json.load(open('gpurun_out/md_${v%%:*}_$rep.json'));m=d['multi_device'];p=d['pcie']
print('${v%%:*}', $rep, 'md', round(m['verify_batch']['value']/1e6,1), 'pcie', round(p['value']/1e6,1), 'single', round(d['single']['value']/1e3,1))"; done; done
