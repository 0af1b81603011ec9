# Kernel timeline of the configs[4] stream (rocprofv3 kernel trace +
# CAPJWT_PIPE_TRACE host timings), by default zero-copy plans vs 524k chunks.
# Run via gpurun from the repo root:  bash tools/gpu_zctrace.sh [tag] [mode ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-zctrace}; shift
MODES=${*:-z0 524288}
O=gpurun_out/$T
mkdir -p $O
CAPJWT_PIPE_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 -u tools/c5_stream_probe.py $O/probe.json 2 $MODES > $O/probe.txt 2> $O/probe.err || { echo TRACE_FAIL; tail -30 $O/probe.err; exit 1; }
cat $O/probe.txt
grep "\[pipe\]" $O/probe.err | tail -20
