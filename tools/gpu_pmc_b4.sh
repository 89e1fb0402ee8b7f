# PMC passes for the four-env part B: issue/wait mix, instruction fetch, vector-memory latency, L2 hits.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/pb4
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM -d gpurun_out/pb4/p1 -o p1 -- python3 $B > gpurun_out/pb4/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pb4/p2 -o p2 -- python3 $B > gpurun_out/pb4/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pb4/p3 -o p3 -- python3 $B > gpurun_out/pb4/p3.log 2>&1
rc=$?
python3 tools/pmc_query.py gpurun_out/pb4 substep_ 2>&1 | tail -30
echo rc=$rc
