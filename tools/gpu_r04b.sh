# Round-4 session B (run via gpurun from the repo root): zero-copy runtime
# tests + configs[4] stream A/B (tools/gpu_zc.sh), RSA-3072 layout A/B
# (class costs per library build), prep LDS slot A/B (ES256 line), then the
# integer / LDS counter passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_zc.sh || exit 1
echo "[rsa3k layouts] $(date +%T)"
for v in base r3k_u4 r3k_u14 r3k_u16 r3k_g2; do
  if [ $v = base ]; then lib=""; else lib="CAPJWT_LIB=$PWD/cap_amd/ab_$v.so"; fi
  env $lib timeout -k 10 300 python3 -u tools/class_costs.py gpurun_out/r3k_$v.json rsa3072,rsa4096 > gpurun_out/r3k_$v.txt 2>&1 || { echo "R3K_FAIL $v"; tail -20 gpurun_out/r3k_$v.txt; exit 1; }
  echo "$v: $(tr '\n' ' ' < gpurun_out/r3k_$v.txt)"
done
echo "[prep slot] $(date +%T)"
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_prep_slot_ab.json 'base:' 'slot33:CAPJWT_LIB=cap_amd/ab_slot33.so' 'slot34:CAPJWT_LIB=cap_amd/ab_slot34.so' 'slot40:CAPJWT_LIB=cap_amd/ab_slot40.so' 'base2:' || exit 1
bash tools/gpu_pmc_int.sh int || exit 1
