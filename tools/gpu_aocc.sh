# Part A occupancy: child AABBs on demand (LDS 17.8 -> 12.6 KB), and with a 3-waves/SIMD register budget.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ao
L=assistive-vr-gym_amd/avr
for v in avr avr_od avr_od3; do
  timeout -k 10 300 env AVR_LIB=$L/lib$v.so python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ao/$v.json 2> gpurun_out/ao/$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ao/$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('$v', round(d['value']), d['nan_or_overflow_envs'], d['reset_pool_sha1'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
