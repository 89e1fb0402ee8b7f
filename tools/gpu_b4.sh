# Parity suite, bench lines for both part-B variants, then the repeated-run flake probe.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/b4
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/b4/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/b4/pytest_gpu.log | tail -12
if [ $rc -ne 0 ]; then echo rc=$rc; exit $rc; fi
for v in 4 1; do
  timeout -k 10 300 env AVR_KERNEL_B=$v python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b4/bench$v.json 2> gpurun_out/b4/bench$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/b4/bench$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('B$v', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
timeout -k 10 300 python3 tools/flake.py 4096 12 > gpurun_out/b4/flake.log 2>&1 || { rc=$?; echo flake rc=$rc; exit $rc; }
grep -v amdgpu gpurun_out/b4/flake.log | tail -7 | cut -c1-200
echo rc=0
