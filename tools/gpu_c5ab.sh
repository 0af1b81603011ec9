# configs[2..4] under HIP hardware-queue counts (the per-class fan-out streams of
# a mixed batch share GPU_MAX_HW_QUEUES queues round-robin): via gpurun
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/ab_run.py gpurun_out/r03_c5_hwq_ab.json base: hwq8:GPU_MAX_HW_QUEUES=8 hwq16:GPU_MAX_HW_QUEUES=16 -- --configs-only --no-ab --steps 6 --warmup 2
