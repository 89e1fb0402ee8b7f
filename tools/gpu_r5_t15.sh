# Round 5 experiment: device-random steps with free-running env groups (no per-step fork / join;
# AVR_FREE_GROUPS=1, direct launches) against direct launches with the join and the default graph
# replay, interleaved.  Output: gpurun_out/r5t15/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t15
for r in 1 2; do
  for v in graph direct free; do
    case $v in graph) E="";; direct) E="AVR_GRAPH=0";; free) E="AVR_GRAPH=0 AVR_FREE_GROUPS=1";; esac
    for T in FeedingJaco-v0 ScratchItchPR2-v0; do
      env $E timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0 > gpurun_out/r5t15/b_${T}_${v}_$r.json 2> gpurun_out/r5t15/b_${T}_${v}_$r.err || exit 11
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value']))" gpurun_out/r5t15/b_${T}_${v}_$r.json $T $v $r
    done
  done
done
