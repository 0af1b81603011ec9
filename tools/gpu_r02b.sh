# round-2: GPU parity suite, then the pipeline probe with its trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|error" gpurun_out/pytest.log | head -20; tail -30 gpurun_out/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest.log | tail -2
CAPJWT_PIPE_TRACE=1 timeout -k 10 300 python -u tools/pipe_probe.py 32768 65536 131072 > gpurun_out/pipe.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/pipe.log; exit 1; }
grep -E "^chunk" gpurun_out/pipe.log
