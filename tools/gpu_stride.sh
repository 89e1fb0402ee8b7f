# Row-buffer stride per env (floats): 20480 (80 KB), 16704 (66.8 KB), 16896 (66 KB + 1 KB), 17024.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/rs
for v in 20480 16704 16896 17024 20480; do
  timeout -k 10 300 env AVR_ROW_STRIDE=$v python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rs/$v.json 2> gpurun_out/rs/$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rs/$v.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('stride $v', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
