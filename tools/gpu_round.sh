set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1 || exit 11
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/g1/b0.json 2> gpurun_out/g1/b0.err || exit 12
timeout -k 10 300 python3 bench.py --task ScratchItchPR2-v0 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/g1/b1.json 2> gpurun_out/g1/b1.err || exit 13
timeout -k 10 300 python3 bench.py --task BedBathingPR2-v0 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/g1/b2.json 2> gpurun_out/g1/b2.err || exit 14
bash tools/gpu_timeline.sh || exit 15
