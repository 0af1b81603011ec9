# A/B: one-wave scalar blocks for small ECDSA launches (JG_EC_SCALAR_SOLO_MAX)
# vs the shared four-wave inversion at every size; parity tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/solo
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_concurrency.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp cap_amd/libcapjwt.so /tmp/lib_solo.so
for v in solo solo0 solo_b solo0_b; do
  case $v in solo|solo_b) cp /tmp/lib_solo.so cap_amd/libcapjwt.so ;; *) cp cap_amd/ab_solo0.so cap_amd/libcapjwt.so ;; esac
  echo "== $v $(date +%T)"
  timeout -k 10 200 python3 -u tools/small_batch_probe.py $O/small_$v.json 1 > $O/small_$v.txt 2>&1 || { echo SMALL_FAIL; tail -5 $O/small_$v.txt; exit 1; }
  cat $O/small_$v.txt
  PROBE_CALLERS=16,64 timeout -k 10 200 python3 -u tools/single_probe.py $O/single_$v.json 4,0 > $O/single_$v.txt 2>&1 || { echo SINGLE_FAIL; tail -5 $O/single_$v.txt; exit 1; }
  grep callers $O/single_$v.txt
done
cp /tmp/lib_solo.so cap_amd/libcapjwt.so
timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5.json 2> $O/c5.err || { echo C5_FAIL; tail -5 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {k: round(x['frac'],3) for k,x in d['mixed_10alg_32kid']['roofline'].items() if 'point' in k})"
