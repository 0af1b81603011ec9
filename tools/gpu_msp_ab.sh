# mixed-config stream: per-class fan-out streams vs in-order classes per chunk, two chunk sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for ch in 65536 262144; do
  for fo in 0 1; do
    echo "fanout=$fo" >> gpurun_out/msp_ab.log
    CAPJWT_FANOUT=$fo timeout -k 10 200 python -u tools/mixed_stream_probe.py $ch >> gpurun_out/msp_ab.log 2>&1 || { tail gpurun_out/msp_ab.log; exit 1; }
  done
done
cat gpurun_out/msp_ab.log
