# Round-4 session J: early arena DMA -- runtime / keyset / edge tests, then
# the configs[4] stream over class groupings, plan-fill streams and early DMA.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp2
timeout -k 10 500 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_keyset.py tests/test_gpu_edges.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_j.log; exit 1; }
tail -n 1 gpurun_out/pytest_j.log
for spec in 0012222:least:1 0012222:least:0 0102122:copy:1 0011022:least:1 0011022:copy:1 1012220:least:1 1012220:copy:1 0102122:copy:0; do
  IFS=: read g c e <<< "$spec"
  CAPJWT_CLASS_GROUP=$g CAPJWT_GROUP_CTRL=$c CAPJWT_EARLY_DMA=$e timeout -k 10 300 python -u tools/c5_stream_probe.py gpurun_out/grp2/${g}_${c}_$e.json 4 524288 262144 > gpurun_out/grp2/${g}_${c}_$e.txt 2>&1 || { echo "ST_FAIL $spec"; tail -30 gpurun_out/grp2/${g}_${c}_$e.txt; exit 1; }
  echo "$spec: $(tr '\n' ' ' < gpurun_out/grp2/${g}_${c}_$e.txt)"
done
