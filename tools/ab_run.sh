set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for t in 0 1 2; do
  TASK=$t AVR_FP_ROOT=/root/repo/_old timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/old$t.npz > gpurun_out/ab/old$t.log 2>&1 || exit 11
  TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/new$t.npz gpurun_out/ab/old$t.npz > gpurun_out/ab/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/ab/new$t.log
done
TASK=1 timeout -k 10 200 python3 tools/prof_phases.py 4096 > gpurun_out/ab/ph1.log 2>&1 || exit 12
timeout -k 10 300 python3 bench.py --task ScratchItchPR2-v0 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/b1.json 2> gpurun_out/ab/b1.err || exit 13
timeout -k 10 300 python3 bench.py --task BedBathingPR2-v0 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/b2.json 2> gpurun_out/ab/b2.err || exit 14
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/b0.json 2> gpurun_out/ab/b0.err || exit 15
