# A/B measurements of one GPU call (run via gpurun from the repo root), each
# step under its own time limit; results under gpurun_out/ab/.
#   bash tools/ab/ab_session.sh STEP ...
# steps:
#   cfg3:NAME[:LIB]      tools/config_probe.py eddsa_es384 (LIB: a cap_amd/ab_*.so, or VAR=VALUE)
#   cfg2:NAME[:LIB]      tools/config_probe.py ps512
#   c5:NAME[:LIB]        bench.py --configs-only (configs[2..4] lines, no refresh / e2e)
#   es256:NAME[:LIB]     bench.py ES256 line only
#   small:THREADS        tools/small_batch_probe.py
#   single[:S+S...]      tools/single_probe.py (S = inflight,window_us)
#   ktrace               tools/small_batch_trace.sh (small-batch kernel trace)
#   valu                 tools/microbench/valu_rates (VALU instruction issue rates)
#   sys                  tools/single_sys_probe.sh (single-token path at many callers)
#   trace:CHUNK          tools/gpu_zctrace.sh (configs[4] stream kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
for step in "$@"; do
  IFS=: read -r kind name lib <<< "$step"
  envs=()
  case "$lib" in
    "") ;;
    *=*) envs=("$lib") ;;                        # an environment assignment
    *) envs=(CAPJWT_LIB="$GRAFT_REPO_ROOT/cap_amd/$lib") ;;
  esac
  echo "== $step $(date +%T)"
  case $kind in
    cfg3) env "${envs[@]}" timeout -k 10 300 python3 -u tools/config_probe.py eddsa_es384 > $O/cfg3_$name.json 2> $O/cfg3_$name.err || { echo FAIL; tail -5 $O/cfg3_$name.err; exit 1; }; cat $O/cfg3_$name.json ;;
    cfg2) env "${envs[@]}" timeout -k 10 300 python3 -u tools/config_probe.py ps512 > $O/cfg2_$name.json 2> $O/cfg2_$name.err || { echo FAIL; tail -5 $O/cfg2_$name.err; exit 1; }; cat $O/cfg2_$name.json ;;
    c5) env "${envs[@]}" timeout -k 10 400 python3 -u bench.py --configs-only --no-refresh --no-e2e --no-ab --steps 10 --warmup 3 > $O/c5_$name.json 2> $O/c5_$name.err || { echo FAIL; tail -5 $O/c5_$name.err; exit 1; }; python3 -c "import json,sys; d=json.load(open('$O/c5_$name.json'))['configs']; print({k: round(v['value']/1e6,2) for k,v in d.items()}, 'stream', round(d['mixed_10alg_32kid'].get('stream',{}).get('value',0)/1e6,2))" ;;
    es256) env "${envs[@]}" timeout -k 10 300 python3 -u bench.py --no-rs256 --no-configs --no-e2e --no-cpu --no-ab --steps 10 --warmup 3 > $O/es256_$name.json 2> $O/es256_$name.err || { echo FAIL; tail -5 $O/es256_$name.err; exit 1; }; python3 -c "import json; d=json.load(open('$O/es256_$name.json')); print(round(d['value']/1e6,1), d['kernel_ms'])" ;;
    small) timeout -k 10 300 python3 -u tools/small_batch_probe.py $O/small_$name.json $name > $O/small_$name.txt 2>&1 || { echo FAIL; tail -5 $O/small_$name.txt; exit 1; }; cat $O/small_$name.txt ;;
    single) timeout -k 10 400 python3 -u tools/single_probe.py $O/single.json ${name//+/ } > $O/single.txt 2>&1 || { echo FAIL; tail -5 $O/single.txt; exit 1; }; cat $O/single.txt ;;
    ktrace) bash tools/small_batch_trace.sh || exit 1 ;;
    valu) timeout -k 10 120 tools/microbench/valu_rates > $O/valu.txt 2>&1 || { echo FAIL; cat $O/valu.txt; exit 1; }; cat $O/valu.txt ;;
    sys) bash tools/single_sys_probe.sh || exit 1 ;;
    trace) bash tools/gpu_zctrace.sh ab/trace_$name $name || exit 1 ;;
  esac
done
