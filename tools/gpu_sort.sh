# Row-count grouping of the four-env part B: parity subset, then bench with and without it.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/so
L=assistive-vr-gym_amd/avr
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "part_b or one_substep or golden or free_space or poison" -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/so/pytest.log 2>&1 || { rc=$?; tail -5 gpurun_out/so/pytest.log; exit $rc; }
tail -1 gpurun_out/so/pytest.log
for v in avr avr_nohc avr_hc28; do
  timeout -k 10 300 env AVR_LIB=$L/lib$v.so python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/so/$v.json 2> gpurun_out/so/$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/so/$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('$v', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
