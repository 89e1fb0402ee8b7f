# One GPU call: parity suite, a short bench line, the phase profile (each step time-limited, chained with &&).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/c
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/c/bench.json 2> gpurun_out/c/bench.err && \
PROF_STEPS=1 timeout -k 10 240 python3 tools/prof_phases.py 4096 > gpurun_out/c/phases.txt 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|assert" gpurun_out/c/pytest_gpu.log | grep -v PASSED | tail -30
python3 -c "import json;d=json.loads(open('gpurun_out/c/bench.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})" 2>/dev/null
grep -v amdgpu.ids gpurun_out/c/phases.txt | grep -v "#" | tail -20
echo rc=$rc
