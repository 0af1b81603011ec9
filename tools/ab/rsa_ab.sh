# RS256 (+ PS512 configs[2] via --configs-only is too long): bench.py's rs256
# leg per library variant, alternated 3 times.  usage: bash tools/ab/rsa_ab.sh name=lib.so ...
cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    CAPJWT_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-configs --no-e2e --no-cpu --no-ab --md-devices none --detail gpurun_out/rsa_ab_detail.json > gpurun_out/rsa_ab_line.json 2> gpurun_out/rsa_ab.err || { echo "FAIL $name"; tail -5 gpurun_out/rsa_ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/rsa_ab_detail.json')); r=d['rs256']
print('$name', $rep, 'es256', round(d['value']/1e6,1), 'rs256', round(r['value']/1e6,1), 'modexp_ms', round(r['kernel_ms']['rsa2048_modexp'],4), 'frac', round(r['roofline']['frac'],4), 'acc', r['accepted'])"
  done
done
