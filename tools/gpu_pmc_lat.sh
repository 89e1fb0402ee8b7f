# Latency / occupancy PMC for the sub-step kernels (separate --pmc passes), plus the phase profile
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/lat
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/lat/p1 -o p1 -- python3 $B > gpurun_out/lat/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM -d gpurun_out/lat/p2 -o p2 -- python3 $B > gpurun_out/lat/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INST_LEVEL_LDS -d gpurun_out/lat/p3 -o p3 -- python3 $B > gpurun_out/lat/p3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_TC_STALL SQC_DCACHE_BUSY_CYCLES -d gpurun_out/lat/p4 -o p4 -- python3 $B > gpurun_out/lat/p4.log 2>&1 && \
PROF_STEPS=2 timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/lat/phases.txt 2>&1
echo rc=$?
