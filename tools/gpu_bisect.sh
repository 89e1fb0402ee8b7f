# Bench runs back to back: new, base (AVR_LIB=libavr_base.so), new, new -- variance / flake probe.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/bis
L=assistive-vr-gym_amd/avr
rc=0
for f in new1 base new2 new3; do
  if [ $f = base ]; then lib=$L/libavr_base.so; else lib=$L/libavr.so; fi
  timeout -k 10 300 env AVR_LIB=$lib python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bis/$f.json 2> gpurun_out/bis/$f.err || { rc=$?; break; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bis/$f.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('$f', round(d['value']), 'nan', d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})" || true
done
echo rc=$rc
