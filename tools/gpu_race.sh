set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
for i in 1 2 3; do timeout -k 10 200 python3 tools/race_check.py libavr.so 4096 10 >> gpurun_out/race.log 2>&1 || exit $?; done
timeout -k 10 200 python3 tools/race_check.py libavr_nopf.so 4096 10 >> gpurun_out/race.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?
grep sha gpurun_out/race.log
tail -1 gpurun_out/bench.log
echo rc=$rc
