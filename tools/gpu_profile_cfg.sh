# rocprofv3 evidence for BASELINE configs[2..4] (PS512 RSA-4096, EdDSA + ES384,
# the 10-alg 32-kid mix): one bench pass of the config lines alone, then a
# kernel trace, FETCH_SIZE / WRITE_SIZE passes and an SQ issue/stall pass of
# the same command.  Run via gpurun from the repo root:
#   gpurun --timeout 1200 -- bash tools/gpu_profile_cfg.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-cfg}
O=gpurun_out/$TAG
mkdir -p "$O"
ARGS="--configs-only --steps 4 --warmup 1 --no-ab --no-refresh"
echo "[0/5] class costs $(date +%T)"
timeout -k 10 300 python3 tools/class_costs.py "$O/class_costs.json" > "$O/class_costs.log" 2>&1 || { echo COSTS_FAIL; tail -20 "$O/class_costs.log"; exit 1; }
echo "[1/5] bench configs $(date +%T)"
timeout -k 10 300 python3 bench.py --configs-only --steps 8 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" || { echo BENCH_FAIL; tail -20 "$O/bench.err"; exit 1; }
echo "[2/5] kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$O/kt.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
echo "[3/5] FETCH_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o f --output-format csv -- python3 bench.py $ARGS > "$O/fetch.json" 2> "$O/fetch.err" || { echo FETCH_FAIL; tail -20 "$O/fetch.err"; exit 1; }
echo "[4/5] WRITE_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o w --output-format csv -- python3 bench.py $ARGS > "$O/write.json" 2> "$O/write.err" || { echo WRITE_FAIL; tail -20 "$O/write.err"; exit 1; }
echo "[5/5] SQ $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$O/sq" -o sq --output-format csv -- python3 bench.py $ARGS > "$O/sq.json" 2> "$O/sq.err" || { echo SQ_FAIL; tail -20 "$O/sq.err"; exit 1; }
echo "[6/6] roofline check $(date +%T)"
python3 tools/cfg_roofline_check.py "$O" "$O/roofline_check.json" || { echo CHECK_FAIL; exit 1; }
echo "done $(date +%T)"
find "$O" -name "*.csv" | head -40
