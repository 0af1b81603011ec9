# round-2: the remaining PMC passes (gather calibration, SQ issue/stall) and an e2e host-thread sweep
# under the box's cgroup CPU quota (nr_throttled before/after each run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu --no-e2e --no-configs"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_cal -o c --output-format csv -- ./tools/ubench/gather_cal > gpurun_out/prof_cal.json 2> gpurun_out/prof_cal.err || { echo CAL_FAIL; tail -20 gpurun_out/prof_cal.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err || { echo SQ_FAIL; tail -20 gpurun_out/pmc_sq.err; exit 1; }
for t in 16 15 14 16 15 14; do
  a=$(grep nr_throttled /sys/fs/cgroup/cpu.stat | head -1 | awk '{print $2}')
  CAPJWT_HOST_THREADS=$t timeout -k 10 200 python -u tools/e2e_probe.py > gpurun_out/e2e_t$t.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/e2e_t$t.log; exit 1; }
  b=$(grep nr_throttled /sys/fs/cgroup/cpu.stat | head -1 | awk '{print $2}')
  echo "threads=$t throttled_periods=$((b-a)) $(grep -o "'ms_per_batch': [0-9.]*" gpurun_out/e2e_t$t.log) $(grep -E 'blob (split|validate)|payload-json|verify parse' gpurun_out/e2e_t$t.log | tail -4 | tr -s ' ' | tr '\n' ' ')"
done
