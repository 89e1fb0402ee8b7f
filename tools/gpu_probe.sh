set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g2
timeout -k 10 200 python3 tools/pool_probe.py ScratchItchPR2-v0 gpurun_out/g2/pool1.npy > gpurun_out/g2/pool1.log 2>&1 || exit 11
timeout -k 10 200 python3 tools/pool_probe.py BedBathingPR2-v0 gpurun_out/g2/pool2.npy > gpurun_out/g2/pool2.log 2>&1 || exit 12
for g in 1 2 4; do
AVR_ENV_GROUPS=$g timeout -k 10 200 python3 bench.py --task ScratchItchPR2-v0 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/g2/s_g$g.json 2>/dev/null || exit 13
done
for gr in 0 1; do
AVR_GRAPH=$gr timeout -k 10 200 python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/g2/f_graph$gr.json 2>/dev/null || exit 14
done
AVR_GRAPH=1 timeout -k 10 200 python3 bench.py --task ScratchItchPR2-v0 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/g2/s_graph1.json 2>/dev/null || exit 15
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k graph -x -v --timeout 200 --timeout-method thread > gpurun_out/g2/pytest_graph.log 2>&1 || exit 16
