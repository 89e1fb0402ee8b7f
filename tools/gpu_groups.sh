# env-group sweep under the default graph replay (one bench per setting)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/grp
T=${TASK:-FeedingJaco-v0}
for g in 1 2 3 4 6 8; do
  AVR_ENV_GROUPS=$g timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/grp/$T.g$g.json 2>/dev/null || exit 11
  echo $T g$g $(python3 -c "import json;d=json.loads(open('gpurun_out/grp/$T.g$g.json').read().strip().splitlines()[-1]);print(round(d['value']))")
done
for g in 6 8; do
  GPU_MAX_HW_QUEUES=8 AVR_ENV_GROUPS=$g timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/grp/$T.q8g$g.json 2>/dev/null || exit 12
  echo $T q8 g$g $(python3 -c "import json;d=json.loads(open('gpurun_out/grp/$T.q8g$g.json').read().strip().splitlines()[-1]);print(round(d['value']))")
done
