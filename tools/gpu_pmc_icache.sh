# Instruction-fetch counters for the bench kernels (I-cache pressure of the unrolled modexp): one rocprofv3 --pmc pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu --no-e2e --no-configs"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS -d gpurun_out/pmc_ic -o ic --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_ic.json 2> gpurun_out/pmc_ic.err || { echo IC_FAIL; tail -20 gpurun_out/pmc_ic.err; exit 1; }
find gpurun_out/pmc_ic -name "*.csv"
