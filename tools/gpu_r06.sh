# Round-6 GPU session (run via gpurun from the repo root):
#   bash tools/gpu_r06.sh "<test files or ->" [bench|full|smoke] ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FIRST=$1; shift
if [ "$FIRST" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_first.log 2>&1 || { echo PYTEST_FIRST_FAIL; tail -40 gpurun_out/pytest_first.log; exit 1; }
  tail -1 gpurun_out/pytest_first.log
fi
for p in "$@"; do
  case $p in
    full) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
          tail -1 gpurun_out/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }; tail -1 gpurun_out/smoke.log ;;
    bench) timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
           wc -c gpurun_out/bench.json; cat gpurun_out/bench.json ;;
    bench:*) timeout -k 10 600 python3 -u bench.py ${p#bench:} > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err || { echo BENCHX_FAIL; tail -30 gpurun_out/bench_x.err; exit 1; }
           cat gpurun_out/bench_x.json ;;
    py:*) timeout -k 10 600 python3 -u ${p#py:} > gpurun_out/py.log 2>&1 || { echo PY_FAIL; tail -30 gpurun_out/py.log; exit 1; }; tail -30 gpurun_out/py.log ;;
  esac
done
