set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/mixed_stream_probe.py ${CHUNK:-65536} > gpurun_out/msp.log 2>&1 || { tail gpurun_out/msp.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/msp_kt -o kt --output-format csv -- python3 tools/mixed_stream_probe.py ${CHUNK:-65536} >> gpurun_out/msp.log 2>&1 || { tail gpurun_out/msp.log; exit 1; }
cat gpurun_out/msp.log | grep chunk
