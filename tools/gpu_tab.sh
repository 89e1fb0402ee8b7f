# Parity suite, then bench lines for support-table thresholds (AVR_TAB_MIN_NV: hulls with more vertices use a table).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/tab
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/tab/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/tab/pytest_gpu.log | tail -12
if [ $rc -ne 0 ]; then echo rc=$rc; exit $rc; fi
for v in 64 24 12 8 64; do
  timeout -k 10 300 env AVR_TAB_MIN_NV=$v python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tab/t$v.json 2> gpurun_out/tab/t$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/tab/t$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('tabmin $v', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
