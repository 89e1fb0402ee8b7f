# Env groups on concurrent streams (AVR_ENV_GROUPS): bench lines, then the flake probe with 2 groups.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/gr
for v in 1 2 4 2; do
  timeout -k 10 300 env AVR_ENV_GROUPS=$v python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gr/g$v.json 2> gpurun_out/gr/g$v.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/gr/g$v.json').read().strip().splitlines()[-1])
print('groups $v', round(d['value']), d['nan_or_overflow_envs'], round(d['ms_per_step'],3))"
done
timeout -k 10 300 env AVR_ENV_GROUPS=2 python3 tools/flake.py 4096 12 > gpurun_out/gr/flake.log 2>&1 || { rc=$?; echo flake rc=$rc; exit $rc; }
grep -v amdgpu gpurun_out/gr/flake.log | tail -7 | cut -c1-200
echo rc=0
