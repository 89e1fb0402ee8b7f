# Round 5: rollouts (per-group graphs for FeedingJaco, per-group branches for the PR2 tasks) -- the
# bit-identity test against the step loop, the device-random tests, interleaved benches of the
# rollout stepping and the per-step joins (--step-sync) on the three tasks, and the two-rank gloo
# rehearsal of the stacked-rollout gather.  Output: gpurun_out/r5t20/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t20
timeout -k 10 600 python3 -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rollout or random_device or graph" > gpurun_out/r5t20/tests.log 2>&1
rc=$?; echo tests rc=$rc; case $rc in 124|134|137|139) exit $rc ;; esac
for r in 1 2; do
  for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0; do
    for v in rollout sync; do
      F=""; [ $v = sync ] && F="--step-sync"
      timeout -k 10 200 python3 bench.py --task $T --steps 30 --warmup 3 --no-cpu-baseline --other-steps 0 $F > gpurun_out/r5t20/b_${T}_${v}_$r.json 2> gpurun_out/r5t20/b_${T}_${v}_$r.err || exit 11
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value']), d['config'].get('stepping'))" gpurun_out/r5t20/b_${T}_${v}_$r.json $T $v $r
    done
  done
done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --dist-backend gloo --steps 32 --warmup 2 --envs 1024 --no-cpu-baseline > gpurun_out/r5t20/rehearsal.json 2> gpurun_out/r5t20/rehearsal.err
echo rehearsal rc=$?
tail -1 gpurun_out/r5t20/rehearsal.json | cut -c1-400
