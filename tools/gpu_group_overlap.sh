# Env-group overlap of the FeedingJaco bench under three launch modes (graph replay, direct
# launches, graph replay with 8 hardware queues): kernel traces summarised by
# tools/group_overlap.py, then plain bench lines of the same modes.  Output: gpurun_out/go/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/go
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-steps 0"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/go/g -o g -- python3 $B > gpurun_out/go/g.log 2>&1 || exit 11
python3 tools/group_overlap.py gpurun_out/go/g > gpurun_out/go/g.txt 2>&1; rm -rf gpurun_out/go/g
AVR_GRAPH=0 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/go/d -o d -- python3 $B > gpurun_out/go/d.log 2>&1 || exit 12
python3 tools/group_overlap.py gpurun_out/go/d > gpurun_out/go/d.txt 2>&1; rm -rf gpurun_out/go/d
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/go/q -o q -- python3 $B > gpurun_out/go/q.log 2>&1 || exit 13
python3 tools/group_overlap.py gpurun_out/go/q > gpurun_out/go/q.txt 2>&1; rm -rf gpurun_out/go/q
for i in 1 2; do
  timeout -k 10 200 python3 $B > gpurun_out/go/b_graph_$i.json 2>/dev/null || exit 14
  AVR_GRAPH=0 timeout -k 10 200 python3 $B > gpurun_out/go/b_direct_$i.json 2>/dev/null || exit 15
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 $B > gpurun_out/go/b_q8_$i.json 2>/dev/null || exit 16
done
for f in gpurun_out/go/b_*.json; do echo "$f $(python3 -c "import json,sys; print(round(json.loads(open('$f').read().strip().splitlines()[-1])['value']))")"; done
