# SQ counters (issue / stall breakdown) for the bench kernels: one rocprofv3 --pmc pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu --no-e2e --no-configs"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err || { echo SQ_FAIL; tail -20 gpurun_out/pmc_sq.err; exit 1; }
find gpurun_out/pmc_sq -name "*.csv"
