# mixed-config stream (10M/8 tokens, 10 algs, 32 kids): in-order classes per chunk vs per-class fan-out, larger chunks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/msp_ab2.log
for ch in 262144 524288 1310720; do
  for fo in 0 1; do
    echo "fanout=$fo chunk=$ch" >> gpurun_out/msp_ab2.log
    CAPJWT_FANOUT=$fo timeout -k 10 200 python -u tools/mixed_stream_probe.py $ch >> gpurun_out/msp_ab2.log 2>&1 || { tail gpurun_out/msp_ab2.log; exit 1; }
  done
done
grep -E "fanout|chunk" gpurun_out/msp_ab2.log
