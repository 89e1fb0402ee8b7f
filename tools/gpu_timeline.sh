# Kernel-trace timeline of the default bench (4 env groups) and of one group: per-queue gaps between
# dependent launches.  Output: gpurun_out/tl/*.txt
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/tl
TASK=${TASK:-FeedingJaco-v0}
B="bench.py --task $TASK --steps 20 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl4 -o tl4 -- python3 $B > gpurun_out/tl/b4.log 2>&1 && \
AVR_ENV_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl1 -o tl1 -- python3 $B > gpurun_out/tl/b1.log 2>&1 && \
python3 tools/timeline.py /tmp/tl4 0.5 > gpurun_out/tl/tl4.txt 2>&1 && \
python3 tools/timeline.py /tmp/tl1 0.5 > gpurun_out/tl/tl1.txt 2>&1
