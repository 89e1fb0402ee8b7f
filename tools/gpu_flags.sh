# Compiler-flag experiment: default build vs flush-denormals (and + approximate transcendentals),
# quick oracle parity and interleaved short benches for each (AVR_LIB selects the build).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/fl
VS=${VARIANTS:-ftz ftzapx}
for v in $VS; do
  AVR_LIB=/root/repo/exp/libavr_$v.so timeout -k 10 200 python3 tools/gpu_quick.py 8 20 > gpurun_out/fl/gq_$v.log 2>&1 || exit $?
done
for r in 1 2; do
  for v in default $VS; do
    if [ $v = default ]; then L=""; else L=/root/repo/exp/libavr_$v.so; fi
    AVR_LIB=$L timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/fl/b_${v}_$r.json 2> gpurun_out/fl/b_${v}_$r.err || exit $?
    echo $v $r $(python3 -c "import json;d=json.loads(open('gpurun_out/fl/b_${v}_$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})")
  done
done
grep -h -E "worst|settle:" gpurun_out/fl/gq_*.log
