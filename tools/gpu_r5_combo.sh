bash tools/gpu_r5_dist.sh && bash tools/gpu_r5_groups.sh
