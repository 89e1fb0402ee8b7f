# Round 5: per-phase cycles of the step kernels (AVR_PROF build, tools/prof_phases.py): FeedingJaco
# at 1024 envs, ScratchItch and BedBathing at 512.  Output: gpurun_out/r5ph/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ph
timeout -k 10 300 python3 tools/prof_phases.py 1024 > gpurun_out/r5ph/feeding.txt 2>&1 || exit 11
TASK=1 timeout -k 10 300 python3 tools/prof_phases.py 512 > gpurun_out/r5ph/scratch.txt 2>&1 || exit 12
TASK=2 timeout -k 10 300 python3 tools/prof_phases.py 512 > gpurun_out/r5ph/bedbath.txt 2>&1 || exit 13
echo ok
