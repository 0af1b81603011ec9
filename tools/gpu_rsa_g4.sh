# RSA-2048 layout A/B: 2 lanes x 37 limbs at two waves/SIMD (default) vs 4 lanes x 19 limbs (152 VGPRs, three waves)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
Q="--no-cpu --no-e2e --no-configs --no-ab --steps 10 --warmup 3"
for v in default g4 default g4; do
  if [ $v = default ]; then lib=cap_amd/libcapjwt.so; else lib=cap_amd/ab_$v.so; fi
  CAPJWT_LIB=$lib timeout -k 10 300 python -u bench.py $Q > gpurun_out/g4_$v.json 2> gpurun_out/g4_$v.err || { echo BENCH_FAIL $v; tail -20 gpurun_out/g4_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/g4_$v.json')); r=d['rs256']; print('$v', 'rs256', round(r['value']/1e6,1), {k: round(v,4) for k,v in r['kernel_ms'].items()}, 'acc', r.get('accepted'))"
done
