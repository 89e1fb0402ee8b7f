# Latency-chain check: step time at 1024 envs (one group) vs 4096 envs with 1 and 4 groups,
# and the AVR_PROF phase breakdown (coop pairs, cycles per phase).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/lat
timeout -k 10 200 python3 bench.py --envs 1024 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lat/b1024.json 2>/dev/null && \
AVR_ENV_GROUPS=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lat/b4096g1.json 2>/dev/null && \
AVR_ENV_GROUPS=2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lat/b4096g2.json 2>/dev/null && \
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/lat/prof_phases.txt 2>&1
rc=$?
for f in gpurun_out/lat/b*.json; do python3 -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',round(d['value']),round(d['ms_per_step'],3),{k:round(v['avg_ms'],4) for k,v in r['kernels'].items()})"; done
grep -v amdgpu.ids gpurun_out/lat/prof_phases.txt | tail -50
echo rc=$rc
