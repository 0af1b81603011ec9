set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_runtime.py tests/test_gpu_concurrency.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp cap_amd/libcapjwt.so /tmp/lib_split2.so
for v in split2 nosplit split4; do
  [ $v = split2 ] && cp /tmp/lib_split2.so cap_amd/libcapjwt.so
  [ $v != split2 ] && cp cap_amd/ab_$v.so cap_amd/libcapjwt.so
  echo "== $v $(date +%T)"
  timeout -k 10 200 python3 -u tools/small_batch_probe.py $O/small_$v.json 1 > $O/small_$v.txt 2>&1 || { echo SMALL_FAIL; tail -5 $O/small_$v.txt; exit 1; }
  cat $O/small_$v.txt
  PROBE_CALLERS=16,64 timeout -k 10 200 python3 -u tools/single_probe.py $O/single_$v.json 4,0 > $O/single_$v.txt 2>&1 || { echo SINGLE_FAIL; tail -5 $O/single_$v.txt; exit 1; }
  grep callers $O/single_$v.txt
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$v.json 2> $O/c5_$v.err || { echo C5_FAIL; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {k: round(x['frac'],3) for k,x in d['mixed_10alg_32kid']['roofline'].items() if 'point' in k})"
done
cp /tmp/lib_split2.so cap_amd/libcapjwt.so
