# e2e Validator.ValidateBatch A/B on one box (run via gpurun from the repo root):
# HEAD as the bench runs it, HEAD with synchronous comb-table builds
# (CAPJWT_TABLES_SYNC=1: no background widening during the timed passes), and the
# round-2 build (e491d0a, in build_e2e_ab/e491, built here), each in its own process
# with CAPJWT_TRACE=1 phase times.  usage: bash tools/e2e_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2e_ab
O=gpurun_out/e2e_ab
run() {  # tag dir [env...]
  local tag=$1 dir=$2; shift 2
  echo "[$tag] $(date +%T)"
  (cd "$dir" && env "$@" timeout -k 10 240 python3 -u tools/e2e_probe.py > "$GRAFT_REPO_ROOT/$O/$tag.out" 2> "$GRAFT_REPO_ROOT/$O/$tag.err") || { echo "FAIL $tag"; tail -20 "$O/$tag.err"; exit 1; }
  tail -1 "$O/$tag.out" | cut -c1-200
}
run head_a . CAPJWT_X=0
run head_sync . CAPJWT_TABLES_SYNC=1
run r02 build_e2e_ab/e491 CAPJWT_X=0
run head_b . CAPJWT_X=0
run r02_b build_e2e_ab/e491 CAPJWT_X=0
run head_sync_b . CAPJWT_TABLES_SYNC=1
