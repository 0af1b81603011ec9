# Kernel trace of small jg_verify_batch calls (tools/small_batch_probe.py, one
# thread): which kernels and gaps make up a small batch's device round trip.
# Run via gpurun from the repo root: bash tools/small_batch_trace.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/small_trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 -u tools/small_batch_probe.py $O/probe.json 1 > $O/probe.txt 2> $O/probe.err || { echo TRACE_FAIL; tail -20 $O/probe.err; exit 1; }
cat $O/probe.txt
