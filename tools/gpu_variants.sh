# Interleaved short benches of experiment builds (exp/libavr_<v>.so, built beforehand on the CPU
# by tools/build_variants.py <v> ...; "default" = the shipped build).  VARIANTS selects them, TASK
# the bench task (default FeedingJaco-v0).  Timing only: a variant's parity is checked separately
# (tools/fingerprint.py against the shipped build, or the GPU tests).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/var
VS=${VARIANTS:-default}
T=${TASK:-FeedingJaco-v0}
for r in 1 2; do
  for v in $VS; do
    L=""
    if [ $v != default ]; then L=/root/repo/exp/libavr_$v.so; fi
    AVR_LIB=$L timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/var/b_${v}_$r.json 2> gpurun_out/var/b_${v}_$r.err || exit $?
    echo $T $v $r $(python3 -c "import json;d=json.loads(open('gpurun_out/var/b_${v}_$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})")
  done
done
