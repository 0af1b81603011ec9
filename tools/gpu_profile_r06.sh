# Round-6 rocprofv3 evidence (run via gpurun from the repo root): the headline
# (ES256 + RS256 lines) kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes,
# the SQ issue pass and the gather calibration, then the configs[2..4] kernel
# trace.  Each bench run writes its full result beside its stdout line
# (--detail), which tools/headline_roofline_check.py and cfg_roofline_check.py read.
#   usage: bash tools/gpu_profile_r06.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06}
O=gpurun_out/$TAG
mkdir -p "$O"
ARGS="--steps 4 --warmup 1 --no-cpu --no-e2e --no-configs --no-ab --md-devices none"
# SKIP_HEAD=1: only the calibration and configs passes (a rerun after the headline passes)
run() {  # name, rocprof args...
  local n=$1; shift
  echo "[$n] $(date +%T)"
  timeout -s KILL 300 rocprofv3 "$@" -d "$O/$n" -o "$n" --output-format csv -- python3 bench.py $ARGS --detail "$O/${n}_detail.json" > "$O/$n.json" 2> "$O/$n.err" || { echo "${n}_FAIL"; tail -20 "$O/$n.err"; exit 1; }
}
if [ -z "$SKIP_HEAD" ]; then
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
fi
# (the calibration binary is built by `make -C tools/ubench gather_cal`)
echo "[cal] $(date +%T)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/cal" -o c --output-format csv -- ./tools/ubench/gather_cal > "$O/cal.json" 2> "$O/cal.err" || { echo CAL_FAIL; tail -20 "$O/cal.err"; exit 1; }
echo "[cfg] $(date +%T)"
mkdir -p "$O/cfg"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/cfg/kt" -o kt --output-format csv -- python3 bench.py --configs-only --steps 4 --warmup 1 --no-ab --no-refresh --detail "$O/cfg/kt_detail.json" > "$O/cfg/kt.json" 2> "$O/cfg/kt.err" || { echo CFG_FAIL; tail -20 "$O/cfg/kt.err"; exit 1; }
python3 tools/headline_roofline_check.py "$O" "$O/headline_roofline_check.json" && python3 tools/cfg_roofline_check.py "$O/cfg" "$O/cfg_roofline_check.json" || echo CHECK_FAIL
find "$O" -name "*stats.csv" | head
echo "done $(date +%T)"
