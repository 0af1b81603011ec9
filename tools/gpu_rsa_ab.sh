# RSA modexp A/B over library variants (tools/build_ab.sh): MAD asm block size 8 / 16, occupancy 1 / 2 waves per SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
Q="--no-cpu --no-e2e --no-configs --no-ab --steps 10 --warmup 3"
for v in base b16 w2b8 w2b16 base b16 w2b8 w2b16; do
  CAPJWT_LIB=cap_amd/ab_$v.so timeout -k 10 300 python -u bench.py $Q > gpurun_out/rsa_ab_$v.json 2> gpurun_out/rsa_ab_$v.err || { echo BENCH_FAIL $v; tail -30 gpurun_out/rsa_ab_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/rsa_ab_$v.json')); r=d['rs256']; print('$v', 'rs256', round(r['value']/1e6,1), 'frac', round(r['roofline']['frac'],3), {k: round(v,4) for k,v in r['kernel_ms'].items()}, 'es256', round(d['value']/1e6,1))"
done
