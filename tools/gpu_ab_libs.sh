# Interleaved short benches of the default libavr.so and experiment libraries (LIBS: space-separated
# paths, used through AVR_LIB), ROUNDS times each, task TASK.  Timing only.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/abl
T=${TASK:-FeedingJaco-v0}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in base $LIBS; do
    if [ $lib = base ]; then unset AVR_LIB; tag=base; else export AVR_LIB=$lib; tag=$(basename $lib .so); fi
    timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0 > gpurun_out/abl/b_${tag}_$r.json 2> gpurun_out/abl/b_${tag}_$r.err || exit $?
    echo $T $tag $r $(python3 -c "import json;d=json.loads(open('gpurun_out/abl/b_${tag}_$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})")
  done
done
unset AVR_LIB
