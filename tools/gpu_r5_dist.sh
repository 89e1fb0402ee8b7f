# Round 5: two-rank rehearsal of the multi-GPU bench path on the one-GPU box (gloo; the driver's
# runs use nccl = RCCL) at the full 4096 envs per rank, so each rank runs four env groups and the
# stacked per-group rollouts feed the all-gather.  Output: gpurun_out/r5dist/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5dist
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --dist-backend gloo --steps 32 --warmup 2 --no-cpu-baseline --other-steps 0 > gpurun_out/r5dist/rehearsal.json 2> gpurun_out/r5dist/rehearsal.err
echo rehearsal rc=$?
tail -1 gpurun_out/r5dist/rehearsal.json | cut -c1-900
