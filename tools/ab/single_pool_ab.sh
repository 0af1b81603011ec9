# coalesced single-token path: the probe's 65 k-token pool (each token called
# twice) vs the bench's 262 k unique tokens called once each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/spool
mkdir -p $O
for v in p65k p262k p65k_b p262k_b; do
  echo "== $v $(date +%T)"
  case $v in p262k*) export PROBE_POOL_N=262144 PROBE_TOTAL=262144 ;; *) export PROBE_POOL_N=65536 PROBE_TOTAL=131072 ;; esac
  PROBE_CALLERS=16,64 timeout -k 10 300 python3 -u tools/single_probe.py $O/single_$v.json 4,0 > $O/single_$v.txt 2>&1 || { echo PROBE_FAIL; tail -5 $O/single_$v.txt; exit 1; }
  grep callers $O/single_$v.txt
done
