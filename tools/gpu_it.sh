# iteration check: parity vs oracle (few envs), wave timeline, short bench
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/it
timeout -k 10 200 python3 tools/gpu_quick.py 8 20 > gpurun_out/it/gq.log 2>&1 && \
timeout -k 10 200 python3 tools/wavetime.py 4096 > gpurun_out/it/wt.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/it/bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/it/gq.log | tail -8
grep -v amdgpu.ids gpurun_out/it/wt.log | tail -4
grep '"value"' gpurun_out/it/bench.log | cut -c1-220
echo rc=$rc
