# round-3 rocprofv3 evidence for the headline (run via gpurun from the repo root):
#   kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes, the SQ issue/stall
#   pass over a short bench run (ES256 + RS256 lines), and the FETCH_SIZE
#   calibration run of tools/ubench/gather_cal; then the config passes of
#   tools/gpu_profile_cfg.sh.  usage: bash tools/gpu_profile_r03.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p "$O"
ARGS="--steps 4 --warmup 1 --no-cpu --no-e2e --no-configs --no-ab"
echo "[1/5] kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python3 bench.py $ARGS > "$O/kt.json" 2> "$O/kt.err" || { echo KT_FAIL; tail -20 "$O/kt.err"; exit 1; }
echo "[2/5] FETCH_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o f --output-format csv -- python3 bench.py $ARGS > "$O/fetch.json" 2> "$O/fetch.err" || { echo FETCH_FAIL; tail -20 "$O/fetch.err"; exit 1; }
echo "[3/5] WRITE_SIZE $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o w --output-format csv -- python3 bench.py $ARGS > "$O/write.json" 2> "$O/write.err" || { echo WRITE_FAIL; tail -20 "$O/write.err"; exit 1; }
echo "[4/5] gather calibration $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/cal" -o c --output-format csv -- ./tools/ubench/gather_cal > "$O/cal.json" 2> "$O/cal.err" || { echo CAL_FAIL; tail -20 "$O/cal.err"; exit 1; }
echo "[5/5] SQ $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$O/sq" -o sq --output-format csv -- python3 bench.py $ARGS > "$O/sq.json" 2> "$O/sq.err" || { echo SQ_FAIL; tail -20 "$O/sq.err"; exit 1; }
find "$O" -name "*.csv" | head -30
echo "done $(date +%T)"
