# Kernel timeline of the configs[4] stream: zero-copy plans vs 524k chunks
# (rocprofv3 kernel trace + CAPJWT_PIPE_TRACE host timings).  Run via gpurun
# from the repo root:  bash tools/gpu_zctrace.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/zctrace
CAPJWT_PIPE_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/zctrace/kt -o kt --output-format csv -- python3 -u tools/c5_stream_probe.py gpurun_out/zctrace/probe.json 2 z0 524288 > gpurun_out/zctrace/probe.txt 2> gpurun_out/zctrace/probe.err || { echo TRACE_FAIL; tail -30 gpurun_out/zctrace/probe.err; exit 1; }
cat gpurun_out/zctrace/probe.txt
grep "\[pipe\]" gpurun_out/zctrace/probe.err | tail -20
