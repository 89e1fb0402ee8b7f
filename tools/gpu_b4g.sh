# Four-env part B from global memory with pipeline depth D (libavr_b4g<D>.so) vs the default part B.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/b4g
L=assistive-vr-gym_amd/avr
timeout -k 10 300 env AVR_LIB=$L/libavr_b4g3.so python3 -u -m pytest tests/test_gpu_parity.py -k "part_b" -x -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/b4g/pytest.log 2>&1 || { rc=$?; tail -5 gpurun_out/b4g/pytest.log; exit $rc; }
tail -1 gpurun_out/b4g/pytest.log
for v in avr:1 avr_b4g2:4 avr_b4g3:4 avr_b4g5:4; do
  lib=${v%%:*}; kb=${v##*:}
  timeout -k 10 300 env AVR_LIB=$L/lib$lib.so AVR_KERNEL_B=$kb python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b4g/$lib$kb.json 2> gpurun_out/b4g/$lib$kb.err || { rc=$?; echo bench rc=$rc; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/b4g/$lib$kb.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']
print('$lib B$kb', round(d['value']), d['nan_or_overflow_envs'], {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
echo rc=0
