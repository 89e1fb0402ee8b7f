FP_TASKS="" bash tools/gpu_r5_t25.sh
