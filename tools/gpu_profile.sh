# rocprofv3 evidence for bench.py (run via gpurun from the repo root):
#   1. --kernel-trace --stats over a short bench run (per-kernel durations)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE (HBM traffic per launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 3 --warmup 1 --no-cpu --no-e2e --no-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_kt.json 2> gpurun_out/prof_kt.err || { echo KT_FAIL; tail -20 gpurun_out/prof_kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o f --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_fetch.json 2> gpurun_out/prof_fetch.err || { echo FETCH_FAIL; tail -20 gpurun_out/prof_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o w --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_write.json 2> gpurun_out/prof_write.err || { echo WRITE_FAIL; tail -20 gpurun_out/prof_write.err; exit 1; }
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write -name "*.csv" | head -20
