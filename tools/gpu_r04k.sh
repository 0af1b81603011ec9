# Round-4 session K: early arena DMA issued after the previous chunk's copies.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grp3
timeout -k 10 500 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_edges.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -n 1 gpurun_out/pytest_k.log
for spec in 0102122:copy:1 0102122:copy:0 0012222:least:1 0012222:least:0 0102122:least:1 0102122:copy:1; do
  IFS=: read g c e <<< "$spec"
  CAPJWT_CLASS_GROUP=$g CAPJWT_GROUP_CTRL=$c CAPJWT_EARLY_DMA=$e timeout -k 10 300 python -u tools/c5_stream_probe.py gpurun_out/grp3/${g}_${c}_$e.json 4 524288 262144 131072 > gpurun_out/grp3/${g}_${c}_$e.txt 2>&1 || { echo "ST_FAIL $spec"; tail -30 gpurun_out/grp3/${g}_${c}_$e.txt; exit 1; }
  echo "$spec: $(tr '\n' ' ' < gpurun_out/grp3/${g}_${c}_$e.txt)"
done
