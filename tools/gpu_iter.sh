set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gpu_quick.py 8 20 > gpurun_out/gq.log 2>&1 && \
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/prof_phases.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/gq.log | tail -12
grep -v amdgpu.ids gpurun_out/prof_phases.txt | head -16
tail -2 gpurun_out/bench.log
echo "rc=$rc"
