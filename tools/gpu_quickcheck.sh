# GPU parity suite, then bench (no CPU baseline) and the wave timeline at 4096 envs, one group.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/q
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q/bench.json 2>/dev/null && \
AVR_ENV_GROUPS=1 timeout -k 10 200 python3 tools/wavetime.py 4096 > gpurun_out/q/wt.log 2>&1
rc=$?
tail -3 gpurun_out/q/pytest_gpu.log
python3 -c "import json;d=json.loads(open('gpurun_out/q/bench.json').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value']),round(d['ms_per_step'],3),{k:round(v['avg_ms'],4) for k,v in r['kernels'].items()})"
grep -v amdgpu.ids gpurun_out/q/wt.log | tail -9
echo rc=$rc
