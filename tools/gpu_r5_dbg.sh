# Round 5 diagnostics: sub-step divergence of the ScratchItch contact pool state 31 and of the
# FeedingJaco arm-in-wheelchair state (EPA budget off), then a short FeedingJaco bench.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5
TASK=1 K=31 STEPS=3 timeout -k 10 240 python3 -u tools/dbg_substeps.py > gpurun_out/r5/sub_s31.log 2>&1 || exit 11
TASK=0 STEPS=4 timeout -k 10 240 python3 -u tools/dbg_substeps.py > gpurun_out/r5/sub_wheel.log 2>&1 || exit 12
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_feeding.json 2> gpurun_out/r5/bench.err || exit 13
