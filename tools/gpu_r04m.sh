# Round-4 session M: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's
# default 4) for the config lines and the ES256 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python3 tools/ab_run.py gpurun_out/r04_hwq_cfg_ab.json 'q4:' 'q8:GPU_MAX_HW_QUEUES=8' 'q16:GPU_MAX_HW_QUEUES=16' 'q4_b:' 'q8_b:GPU_MAX_HW_QUEUES=8' -- --configs-only --steps 8 --warmup 2 --no-ab --no-refresh || exit 1
timeout -k 10 400 python3 tools/ab_run.py gpurun_out/r04_hwq_es_ab.json 'q4:' 'q8:GPU_MAX_HW_QUEUES=8' 'q4_b:' 'q8_b:GPU_MAX_HW_QUEUES=8' || exit 1
