# Round-4 rocprofv3 evidence (run via gpurun from the repo root): the
# headline passes of tools/gpu_profile_r03.sh (kernel trace, FETCH_SIZE,
# WRITE_SIZE, gather calibration, SQ) and the config passes of
# tools/gpu_profile_cfg.sh.   usage: bash tools/gpu_profile_r04.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
bash tools/gpu_profile_r03.sh "${TAG}h" || exit 1
bash tools/gpu_profile_cfg.sh "${TAG}c" || exit 1
