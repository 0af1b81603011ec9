# A/B (run via gpurun from the repo root): EdDSA small-batch latency with the
# Ed25519 split kernel and without (ab_edno.so), then configs[2..4] with the
# P-256 two-lane split for mid-size launches (ab_p256s2.so) and without.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/q
mkdir -p $O
cp cap_amd/libcapjwt.so /tmp/lib_base.so
for v in base edno; do
  [ $v = edno ] && cp cap_amd/ab_edno.so cap_amd/libcapjwt.so
  echo "== small EdDSA $v $(date +%T)"
  timeout -k 10 200 python3 -u tools/small_batch_probe.py $O/small_ed_$v.json 1 EdDSA > $O/small_ed_$v.txt 2>&1 || { echo SMALL_FAIL; tail -5 $O/small_ed_$v.txt; exit 1; }
  cat $O/small_ed_$v.txt
  cp /tmp/lib_base.so cap_amd/libcapjwt.so
done
for v in p256s2 base p256s2b; do
  [ $v != base ] && cp cap_amd/ab_p256s2.so cap_amd/libcapjwt.so
  echo "== c5 $v $(date +%T)"
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$v.json 2> $O/c5_$v.err || { echo C5_FAIL; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {k: round(x['frac'],3) for k,x in d['mixed_10alg_32kid']['roofline'].items() if 'point' in k})"
  cp /tmp/lib_base.so cap_amd/libcapjwt.so
done
