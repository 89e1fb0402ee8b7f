# quick parity + phase profile + kernel-trace split of a short bench
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/it2
timeout -k 10 300 python3 tools/gpu_quick.py 8 20 > gpurun_out/it2/gq.log 2>&1 && \
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/it2/prof_phases.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/it2/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/it2/kt_bench.log 2>&1
rc=$?
grep -E "worst|settle:" gpurun_out/it2/gq.log
grep -v amdgpu.ids gpurun_out/it2/prof_phases.txt | head -19
grep '"value"' gpurun_out/it2/kt_bench.log | cut -c1-190
echo rc=$rc
