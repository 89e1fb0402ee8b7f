set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/prof_phases.txt 2>&1
echo "rc=$?"
cat gpurun_out/prof_phases.txt | grep -v amdgpu.ids
