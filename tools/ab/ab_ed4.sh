# Ed25519 four-lane split A/B (run via gpurun from the repo root): parity tests
# with the default library (2 lanes up to 16 k tokens) and with ab_ed4sm
# (4 lanes up to 64 k tokens), then lone EdDSA batches and configs[2..4] for
# the default, ab_ed4s (4 lanes up to 16 k) and ab_ed4m (2 lanes up to 16 k,
# 4 lanes up to 64 k).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ed4
mkdir -p $O
T="tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_fe25519.py tests/test_gpu_concurrency.py"
cp cap_amd/libcapjwt.so /tmp/lib_ed2.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp cap_amd/ab_ed4sm.so cap_amd/libcapjwt.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $O/pytest_ed4sm.log 2>&1 || { echo PYTEST4_FAIL; tail -30 $O/pytest_ed4sm.log; cp /tmp/lib_ed2.so cap_amd/libcapjwt.so; exit 1; }
tail -1 $O/pytest_ed4sm.log
for v in ed2 ed4s ed4m ed2_b ed4m_b; do
  case $v in ed2|ed2_b) cp /tmp/lib_ed2.so cap_amd/libcapjwt.so ;; *) cp cap_amd/ab_${v%_b}.so cap_amd/libcapjwt.so ;; esac
  echo "== $v $(date +%T)"
  timeout -k 10 200 python3 -u tools/small_batch_probe.py $O/small_$v.json 1 EdDSA > $O/small_$v.txt 2>&1 || { echo SMALL_FAIL; tail -5 $O/small_$v.txt; exit 1; }
  cat $O/small_$v.txt
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$v.json 2> $O/c5_$v.err || { echo C5_FAIL; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {c: {k: round(x['frac'],3) for k,x in d[c]['roofline'].items() if 'point' in k} for c in ('mixed_10alg_32kid','eddsa_es384_mixed')}, 'ed_ms', round(d['mixed_10alg_32kid']['kernel_ms']['ed25519_point'],4))"
done
cp /tmp/lib_ed2.so cap_amd/libcapjwt.so
