# Round 5 experiment: more env groups now that rollouts join them once per rollout -- 4 / 6 / 8
# groups with 4 / 8 hardware queues (GPU_MAX_HW_QUEUES, read at HIP start-up), FeedingJaco and
# BedBathing, interleaved.  Output: gpurun_out/r5grp/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5grp
for r in 1 2; do
  for cfg in "4 4" "6 8" "8 8" "4 8"; do
    set -- $cfg; G=$1; Q=$2
    for T in FeedingJaco-v0 BedBathingPR2-v0; do
      GPU_MAX_HW_QUEUES=$Q AVR_ENV_GROUPS=$G timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0 > gpurun_out/r5grp/b_${T}_${G}_${Q}_$r.json 2> gpurun_out/r5grp/b_${T}_${G}_${Q}_$r.err || exit 11
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], 'groups', sys.argv[3], 'queues', sys.argv[4], round(d['value']))" gpurun_out/r5grp/b_${T}_${G}_${Q}_$r.json $T $G $Q
    done
  done
done
