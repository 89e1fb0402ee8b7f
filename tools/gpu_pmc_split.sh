# PMC passes (one block group per pass) over the split part-A kernels, then the approximate
# division build against the default in interleaved benches.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ps
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/ps/p1 -o p1 -- python3 $B > gpurun_out/ps/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum -d gpurun_out/ps/p2 -o p2 -- python3 $B > gpurun_out/ps/p2.log 2>&1 && \
python3 tools/pmc_query.py gpurun_out/ps substep_pairs narrowphase substep_a substep_b4 && \
VARIANTS="default fdiv" bash tools/gpu_variants.sh
echo rc=$?
