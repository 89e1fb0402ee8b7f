# phase profile (AVR_PROF build) at 4096 envs + quick parity
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ph
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/ph/prof_phases.txt 2>&1 && \
timeout -k 10 300 python3 tools/gpu_quick.py 8 10 > gpurun_out/ph/gq.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ph/prof_phases.txt | tail -30
grep -E "worst|settle:" gpurun_out/ph/gq.log
echo rc=$rc
