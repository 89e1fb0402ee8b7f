# Multi-rank rehearsal on a one-GPU box: two ranks share cuda:0 through the gloo backend (the
# driver's multi-GPU runs use nccl = RCCL); exercises sharding, barrier, max-over-ranks timing and
# the rollout all-gather.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/dist
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --dist-backend gloo --steps 32 --warmup 2 --envs 1024 --no-cpu-baseline > gpurun_out/dist/rehearsal.json 2> gpurun_out/dist/rehearsal.err
