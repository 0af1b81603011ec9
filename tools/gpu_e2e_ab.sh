# e2e A/B over glibc malloc settings (is the host layer allocation/page-fault bound?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in "" "glibc.malloc.trim_threshold=4294967296:glibc.malloc.top_pad=268435456" "glibc.malloc.hugetlb=1:glibc.malloc.trim_threshold=4294967296"; do
  echo "== GLIBC_TUNABLES=$t"
  GLIBC_TUNABLES=$t timeout -k 10 200 python -u tools/e2e_probe.py > gpurun_out/e2e_ab.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/e2e_ab.log; exit 1; }
  grep -E "payload-json|blob validate|verify parse|free-toks|blob release" gpurun_out/e2e_ab.log | tail -6
  grep -o "'value': [0-9.]*" gpurun_out/e2e_ab.log
done
