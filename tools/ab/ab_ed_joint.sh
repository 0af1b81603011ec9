# Ed25519 joint-load A/B (run via gpurun from the repo root): parity tests
# with the joint k_ed_point, then configs[1..4] with it (3 waves per SIMD),
# capped at 4 waves (ab_edj4), and the branchy per-entry loads (ab_edbase).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/edj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_comb_tiers.py tests/test_gpu_fe25519.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp cap_amd/libcapjwt.so /tmp/lib_joint.so
for v in joint edbase edj4 joint_b; do
  case $v in joint|joint_b) cp /tmp/lib_joint.so cap_amd/libcapjwt.so ;; *) cp cap_amd/ab_$v.so cap_amd/libcapjwt.so ;; esac
  echo "== $v $(date +%T)"
  timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$v.json 2> $O/c5_$v.err || { echo C5_FAIL; tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2), {c: {k: round(x['frac'],3) for k,x in d[c]['roofline'].items() if 'point' in k} for c in ('mixed_10alg_32kid','eddsa_es384_mixed')})"
done
cp /tmp/lib_joint.so cap_amd/libcapjwt.so
