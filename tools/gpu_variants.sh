# Interleaved short benches of experiment builds (exp/libavr_<v>.so, built beforehand on the CPU
# by tools/build_variants.py <v> ...; "default" = the shipped build, "glb" = the shipped build with
# AVR_B4_GLOBAL=1).  VARIANTS selects them; each build first passes the quick oracle parity check
# (tools/gpu_quick.py exits non-zero past the contact-rich chaos envelope).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/var
VS=${VARIANTS:-default}
for v in $VS; do
  L=""; G=0
  if [ $v = glb ]; then G=1; elif [ $v != default ]; then L=/root/repo/exp/libavr_$v.so; fi
  AVR_LIB=$L AVR_B4_GLOBAL=$G timeout -k 10 200 python3 tools/gpu_quick.py 8 20 > gpurun_out/var/q_$v.log 2>&1 || { echo "$v: quick parity failed"; tail -3 gpurun_out/var/q_$v.log; exit 1; }
done
for r in 1 2; do
  for v in $VS; do
    L=""; G=0
    if [ $v = glb ]; then G=1; elif [ $v != default ]; then L=/root/repo/exp/libavr_$v.so; fi
    AVR_LIB=$L AVR_B4_GLOBAL=$G timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/var/b_${v}_$r.json 2> gpurun_out/var/b_${v}_$r.err || exit $?
    echo $v $r $(python3 -c "import json;d=json.loads(open('gpurun_out/var/b_${v}_$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})")
  done
done
