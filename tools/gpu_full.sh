bash tools/gpu_check.sh && bash tools/gpu_profile.sh
