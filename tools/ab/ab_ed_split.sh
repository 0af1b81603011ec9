# Ed25519 split-kernel A/B (run via gpurun from the repo root): parity tests
# with the split path, then configs[2..4] with it and without it
# (cap_amd/ab_edno.so copied over libcapjwt.so for the second run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ed
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_fe25519.py tests/test_gpu_runtime.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp cap_amd/libcapjwt.so /tmp/lib_edsplit.so
for v in edsplit edno edsplit2; do
  [ $v = edno ] && cp cap_amd/ab_edno.so cap_amd/libcapjwt.so
  [ $v != edno ] && cp /tmp/lib_edsplit.so cap_amd/libcapjwt.so
  echo "== $v $(date +%T)"
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$v.json 2> $O/c5_$v.err || { echo C5_FAIL; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {k: round(x['frac'],3) for k,x in d['mixed_10alg_32kid']['roofline'].items() if 'point' in k})"
done
cp /tmp/lib_edsplit.so cap_amd/libcapjwt.so
