# Part-B staging capacity vs occupancy: bench lines for the default build and two smaller-LDS builds.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/cap
L=assistive-vr-gym_amd/avr
for v in avr avr_c128 avr_c104 avr; do
  timeout -k 10 300 env AVR_LIB=$L/lib$v.so python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cap/$v.json 2> gpurun_out/cap/$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cap/$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('$v', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
