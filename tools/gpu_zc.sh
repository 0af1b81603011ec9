# Zero-copy class-major plans: runtime tests, then the configs[4] stream A/B
# (chunked DMA vs zero-copy plans, prep feed on / off), then optional extra
# probes by name (pmc_int).  Run via gpurun from the repo root:
#   bash tools/gpu_zc.sh [pmc_int]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_zc.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_zc.log; exit 1; }
tail -1 gpurun_out/pytest_zc.log
timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/zc_feed1.json 4 524288 z0 z655360 > gpurun_out/zc_feed1.txt 2>&1 || { echo PROBE1_FAIL; tail -30 gpurun_out/zc_feed1.txt; exit 1; }
cat gpurun_out/zc_feed1.txt
CAPJWT_ZC_FEED=0 timeout -k 10 400 python -u tools/c5_stream_probe.py gpurun_out/zc_feed0.json 4 z0 > gpurun_out/zc_feed0.txt 2>&1 || { echo PROBE0_FAIL; tail -30 gpurun_out/zc_feed0.txt; exit 1; }
cat gpurun_out/zc_feed0.txt
for p in "$@"; do
  case $p in
    pmc_int) bash tools/gpu_pmc_int.sh int || exit 1 ;;
  esac
done
