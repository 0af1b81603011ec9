# e2e host-thread sweep (cgroup CPU quota: does leaving headroom help?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in 16 12 14 16; do
  CAPJWT_HOST_THREADS=$t timeout -k 10 200 python -u tools/e2e_probe.py > gpurun_out/e2e_t$t.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/e2e_t$t.log; exit 1; }
  echo "threads=$t $(grep -o "'ms_per_batch': [0-9.]*" gpurun_out/e2e_t$t.log) $(grep -E 'blob (split|validate|release)|payload-json' gpurun_out/e2e_t$t.log | tail -4 | tr -s ' ' | tr '\n' ' ')"
done
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
