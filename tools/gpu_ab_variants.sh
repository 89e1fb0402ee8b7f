# Interleaved benches of experiment builds (_ab/libavr_<v>.so from tools/build_variants.py; "default"
# = the shipped build), ROUNDS rounds, task TASK.  Prints value and per-kernel averages (bench detail).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
T=${TASK:-FeedingJaco-v0}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-default}; do
    L=""; [ $v != default ] && L=/root/repo/_ab/libavr_$v.so
    AVR_LIB=$L AVR_BENCH_DETAIL=gpurun_out/ab/d_${T}_${v}_$r.json timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0 > gpurun_out/ab/b_${T}_${v}_$r.json 2> gpurun_out/ab/b_${T}_${v}_$r.err || exit $?
    python3 - gpurun_out/ab/d_${T}_${v}_$r.json $T $v $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d = d[0] if isinstance(d, list) else d
k = d.get('kernels', {})
print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value']), {n.split('_kernel')[0][-12:]: round(x['avg_ms'], 4) for n, x in k.items()})
PY
  done
done
