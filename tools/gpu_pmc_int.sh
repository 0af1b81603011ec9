# Integer-instruction and LDS counters: SQ_INSTS_VALU_INT32 /
# _INT64, SQ_LDS_BANK_CONFLICT and SQ_LDS_IDX_ACTIVE per kernel, one rocprofv3
# --pmc pass over the headline bench (ES256 + RS256 lines: k_prep, k_ec_point,
# k_rsa_modexp) and one over the config lines (k_ed_point, P-384/521, RSA-4K).
# Run via gpurun from the repo root:  bash tools/gpu_pmc_int.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-int}
O=gpurun_out/$TAG
mkdir -p "$O"
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
echo "[1/2] headline $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc $CNT -d "$O/head" -o h --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --no-configs --no-ab > "$O/head.json" 2> "$O/head.err" || { echo HEAD_FAIL; tail -20 "$O/head.err"; exit 1; }
echo "[2/2] configs $(date +%T)"
timeout -s KILL 300 rocprofv3 --pmc $CNT -d "$O/cfg" -o c --output-format csv -- python3 bench.py --configs-only --steps 2 --warmup 1 --no-ab --no-refresh > "$O/cfg.json" 2> "$O/cfg.err" || { echo CFG_FAIL; tail -20 "$O/cfg.err"; exit 1; }
find "$O" -name "*counter_collection.csv"
echo "done $(date +%T)"
