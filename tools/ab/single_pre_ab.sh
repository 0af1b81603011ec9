# coalesced single-token path, fresh process vs after the bench's headline
# leg (W = 26 tables built, a 1 M batch, context closed) in the same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/spre
mkdir -p $O
for v in fresh headline fresh_b headline_b; do
  echo "== $v $(date +%T)"
  case $v in headline*) export PROBE_PRE=headline ;; *) unset PROBE_PRE ;; esac
  PROBE_CALLERS=16,64 timeout -k 10 300 python3 -u tools/single_probe.py $O/single_$v.json 4,0 > $O/single_$v.txt 2>&1 || { echo PROBE_FAIL; tail -5 $O/single_$v.txt; exit 1; }
  grep callers $O/single_$v.txt
done
