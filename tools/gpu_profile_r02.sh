# round-2 rocprofv3 evidence (run via gpurun from the repo root):
#   kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes, the SQ issue/stall
#   pass over a short bench run, and the FETCH_SIZE calibration of the point
#   kernel's 80-byte gather pattern (tools/ubench/gather_cal)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 3 --warmup 1 --no-cpu --no-e2e --no-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_kt.json 2> gpurun_out/prof_kt.err || { echo KT_FAIL; tail -20 gpurun_out/prof_kt.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o f --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_fetch.json 2> gpurun_out/prof_fetch.err || { echo FETCH_FAIL; tail -20 gpurun_out/prof_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o w --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_write.json 2> gpurun_out/prof_write.err || { echo WRITE_FAIL; tail -20 gpurun_out/prof_write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_cal -o c --output-format csv -- ./tools/ubench/gather_cal > gpurun_out/prof_cal.json 2> gpurun_out/prof_cal.err || { echo CAL_FAIL; tail -20 gpurun_out/prof_cal.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err || { echo SQ_FAIL; tail -20 gpurun_out/pmc_sq.err; exit 1; }
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_cal gpurun_out/pmc_sq -name "*.csv" | head -30
