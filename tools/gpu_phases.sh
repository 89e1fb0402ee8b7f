# Per-phase cycle breakdown of part A (AVR_PROF build) at the bench workload.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ph
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/ph/prof_phases.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ph/prof_phases.txt | tail -28
echo rc=$rc
