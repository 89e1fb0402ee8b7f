# Interleaved short benches: a previous tree (AB, default _ab2/: a git worktree with its libavr.so built) and the
# working tree, ROUNDS times each, task TASK (default FeedingJaco-v0).  Timing only.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/abb
T=${TASK:-FeedingJaco-v0}
for r in $(seq 1 ${ROUNDS:-2}); do
  for tree in ${AB:-_ab2} .; do
    tag=$([ $tree = . ] && echo new || echo old)
    extra="--other-steps 0"
    (cd /root/repo/$tree && timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline $extra) > gpurun_out/abb/b_${tag}_$r.json 2> gpurun_out/abb/b_${tag}_$r.err || exit $?
    echo $T $tag $r $(python3 -c "import json;d=json.loads(open('gpurun_out/abb/b_${tag}_$r.json').read().strip().splitlines()[-1]);k=d['roofline']['kernels'];print(round(d['value']), d['nan_or_overflow_envs'], {n[4:16]:round(x['avg_ms'],4) for n,x in k.items()})")
  done
done
