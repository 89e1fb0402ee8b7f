# Round 5: ScratchItch per-phase cycles with the slowest contact-row envs (AVR_PROF build).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ph
TASK=1 timeout -k 10 300 python3 tools/prof_phases.py 512 > gpurun_out/r5ph/scratch2.txt 2>&1
echo rc=$?
tail -8 gpurun_out/r5ph/scratch2.txt
