# PMC detail for the sub-step kernels: scalar-cache / L2 hit rates and wait/issue split
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/pmcb
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM -d gpurun_out/pmcb/p1 -o p1 -- python3 $B > gpurun_out/pmcb/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmcb/p2 -o p2 -- python3 $B > gpurun_out/pmcb/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES -d gpurun_out/pmcb/p3 -o p3 -- python3 $B > gpurun_out/pmcb/p3.log 2>&1
echo rc=$?
