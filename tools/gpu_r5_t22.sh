# Round 5 experiment: part B with one LDS-path instantiation (B4_ONE_LDS: robot parts read for every
# contact row) against the shipped build -- does a smaller hot-code footprint help the four
# concurrent env groups?  Output: gpurun_out/ab/, gpurun_out/r5t22/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t22
VARIANTS="default onelds" ROUNDS=3 bash tools/gpu_ab_variants.sh > gpurun_out/r5t22/ab.log 2>&1 || exit 22
