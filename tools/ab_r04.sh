# Round-4 A/Bs on one box (run via gpurun from the repo root):
#   prep LDS slot stride (ES256 line), Ed25519 radix-2^25.5 vs round-3 Montgomery point loop (config lines)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "[ES256: prep slot, scalar block inversion] $(date +%T)"
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_prep_slot_ab.json 'base:' 'slot34:CAPJWT_LIB=cap_amd/ab_slot34.so' 'slot33:CAPJWT_LIB=cap_amd/ab_slot33.so' 'scalar_wpb1:CAPJWT_LIB=cap_amd/ab_scalar1.so' 'base2:' || exit 1
echo "[ed radix] $(date +%T)"
timeout -k 10 600 python3 tools/ab_run.py gpurun_out/r04_ed_radix_ab.json 'radix255:' 'mont_r03:CAPJWT_LIB=cap_amd/ab_edr03.so' -- --configs-only --steps 6 --warmup 2 --no-ab --no-refresh || exit 1
