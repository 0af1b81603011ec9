# Round-4 session G: RSA modulus-in-LDS and Ed25519 point occupancy A/Bs by
# class cost (tools/class_costs.py; each class alone filling the chip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base nlds nlds_g4 ed4w base2; do
  lib=""; case $v in base|base2) ;; *) lib="CAPJWT_LIB=$PWD/cap_amd/ab_$v.so" ;; esac
  env $lib timeout -k 10 300 python3 -u tools/class_costs.py gpurun_out/cc_$v.json rsa2048,rsa2048_pss,rsa3072,rsa4096,rsa4096_pss,ed25519 > gpurun_out/cc_$v.txt 2>&1 || { echo "CC_FAIL $v"; tail -20 gpurun_out/cc_$v.txt; exit 1; }
  echo "$v: $(tr '\n' ' ' < gpurun_out/cc_$v.txt)"
done
echo "[point prefetch A/B] $(date +%T)"
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_point_pf_ab.json 'base:' 'ppf:CAPJWT_LIB=cap_amd/ab_ppf.so' 'base_b:' 'ppf_b:CAPJWT_LIB=cap_amd/ab_ppf.so' || exit 1
