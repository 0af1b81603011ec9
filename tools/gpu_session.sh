# One GPU call: named test files first, the whole -m gpu suite, the default
# bench, then optional probes (run via gpurun from the repo root):
#   bash tools/gpu_session.sh "<first test files>" [probe ...]
# probes: e2e_ab (tools/e2e_ab.sh), keyload (tools/keyload_trace.py),
#   pmc_int (tools/gpu_pmc_int.sh), zc (tools/ubench/zc_read), smoke
#   (__graft_entry__.smoke()), prof:TAG (tools/gpu_profile_r03.sh: headline
#   kernel trace + FETCH/WRITE + SQ passes), profcfg:TAG (tools/gpu_profile_cfg.sh); "-" as the first
#   argument skips the tests and the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FIRST=$1; shift
if [ "$FIRST" = "-" ]; then SKIP=1; FIRST=""; fi
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_first.log 2>&1 || { echo PYTEST_FIRST_FAIL; tail -40 gpurun_out/pytest_first.log; exit 1; }
  tail -1 gpurun_out/pytest_first.log
fi
[ -z "$SKIP" ] && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -2
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json || true; }
for p in "$@"; do
  case $p in
    e2e_ab) bash tools/e2e_ab.sh || exit 1 ;;
    boxinfo) bash tools/boxinfo.sh > gpurun_out/boxinfo.txt 2>&1; cat gpurun_out/boxinfo.txt ;;
    pmc_int) bash tools/gpu_pmc_int.sh int || exit 1 ;;
    zc) timeout -k 10 180 ./tools/ubench/zc_read > gpurun_out/zc_read.txt 2>&1 || { echo ZC_FAIL; cat gpurun_out/zc_read.txt; exit 1; }; cat gpurun_out/zc_read.txt ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }; tail -3 gpurun_out/smoke.log ;;
    prof:*) bash tools/gpu_profile_r03.sh "${p#prof:}" || exit 1 ;;
    profcfg:*) bash tools/gpu_profile_cfg.sh "${p#profcfg:}" || exit 1 ;;
    keyload) timeout -k 10 300 python -u tools/keyload_trace.py > gpurun_out/keyload.log 2>&1 || { echo KEYLOAD_FAIL; tail -20 gpurun_out/keyload.log; exit 1; }; cat gpurun_out/keyload.log ;;
  esac
done
