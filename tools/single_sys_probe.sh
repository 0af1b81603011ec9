# The coalesced single-token path at many concurrent callers under malloc /
# CPU-placement variants (system time per call: which host mechanism costs it).
# Run via gpurun from the repo root: bash tools/single_sys_probe.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sys
mkdir -p $O
export PROBE_CALLERS=256,1024
run() {
  name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 240 "$@" python3 -u tools/single_probe.py $O/$name.json 4,0 > $O/$name.txt 2>&1 || { echo FAIL; tail -5 $O/$name.txt; exit 1; }
  cat $O/$name.txt
}
run base env
run arena2 env MALLOC_ARENA_MAX=2
run cpus16 taskset -c "$(python3 -c 'import os; print(",".join(map(str, sorted(os.sched_getaffinity(0))[:16])))')"
