# Round-4 session O: decoded payloads in one cached block per batch -- keyset /
# validator GPU tests, then the e2e leg alternating the new host module and the
# previous one (ab_host/cap_amd_old, CAPJWT_HOST_EXT_DIR) on the same box, and
# the new one with glibc's heap trimming off (tun: freed heap stays mapped).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_keyset.py tests/test_gpu_edges.py tests/test_oidc_hash.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_o.log; exit 1; }
tail -n 1 gpurun_out/pytest_o.log
for v in new old tun new old tun; do
  if [ $v = old ]; then export CAPJWT_HOST_EXT_DIR="$GRAFT_REPO_ROOT/ab_host/cap_amd_old"; else unset CAPJWT_HOST_EXT_DIR; fi
  if [ $v = tun ]; then export GLIBC_TUNABLES=glibc.malloc.trim_threshold=4294967296:glibc.malloc.mmap_threshold=33554432; else unset GLIBC_TUNABLES; fi
  timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-rs256 --no-configs --no-cpu --no-ab > gpurun_out/e2e_o_$v.json 2> gpurun_out/e2e_o_$v.err || { echo BENCH_FAIL; tail -20 gpurun_out/e2e_o_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_o_$v.json').read().strip().splitlines()[-1]); e=d['e2e']; print('$v', round(e['value']/1e6,2), e['phases_ms_last_pass'])" | tee -a gpurun_out/e2e_o_summary.txt
done
