"""One rank of the two-rank HIP-path rollout test (tests/test_gpu_dist.py), started by
torch.distributed.run before any process touches the GPU.

Each rank steps its shard of global env ids (env_offset = rank x E) through libavr on the one GPU
the ranks share, in stacked rollouts of G steps (avr_rollout_random_device, as bench.py's multi-GPU
path does), packs every chunk and all-gathers it over gloo (rollouts through host memory; the
driver's multi-GPU runs use nccl = RCCL over xGMI, one rank per GPU).  Rank 0 writes the gathered
rollout to --out.  Not a test module: it only runs under torch.distributed.run.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

import numpy as np                      # noqa: E402
import torch                            # noqa: E402
import torch.distributed as dist        # noqa: E402


def initial_states(task, n_global, pool=32):
    """Reset states of global envs 0..n_global-1: a pool of `pool` distinct host resets (keyed by
    global id) tiled over the ids -- the same rows whatever the rank layout."""
    from avr import _abi as ABI, reset as RS
    A = ABI.load_scene(task)
    md = ABI.ModelDesc(A)
    S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(pool)), impairment='random')
    return md, np.tile(S, ((n_global + pool - 1) // pool, 1))[:n_global].astype(np.float32)


def run_shard(md, S, offset, E, chunks, G, settle, device, on_chunk):
    """Settle, then `chunks` stacked rollouts of G steps of envs [offset, offset + E); on_chunk(c,
    obs, rew, done, info) receives each chunk's stacked device outputs."""
    from avr import _lib
    dev = torch.device('cuda', device)
    L = md.layout
    sim = _lib.Sim(md, E, device=device, seed=1001, env_offset=offset)
    try:
        sim.set_state(S[offset:offset + E])
        sim.settle(settle)
        so, sr = torch.zeros(G, E, L.OBS_DIM, device=dev), torch.zeros(G, E, device=dev)
        sd, si = torch.zeros(G, E, dtype=torch.uint8, device=dev), torch.zeros(G, E, L.INFO_DIM, device=dev)
        for c in range(chunks):
            sim.rollout_random_device(c * G, G, so.data_ptr(), sr.data_ptr(), sd.data_ptr(), si.data_ptr(), stacked=True)
            sim.sync()
            on_chunk(c, so, sr, sd, si)
        groups = sim.env_groups()
    finally:
        sim.close()
    return groups


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--task', type=int, default=0)
    ap.add_argument('--envs', type=int, default=2048, help='envs per rank')
    ap.add_argument('--chunks', type=int, default=2)
    ap.add_argument('--G', type=int, default=16)
    ap.add_argument('--settle', type=int, default=20)
    args = ap.parse_args()
    from avr import dist as D
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    md, S = initial_states(args.task, world * args.envs)
    off, E = D.shard(args.envs, rank)
    W = D.roll_width(md.layout.OBS_DIM)
    roll = torch.zeros(args.G, E, W, device=torch.device('cuda', 0))
    got = []

    def on_chunk(c, so, sr, sd, si):
        D.pack_rollout_stacked(roll, so, sr, si, sd, args.G)
        got.append(D.gather_rollouts(roll.cpu()).numpy().copy())

    groups = run_shard(md, S, off, E, args.chunks, args.G, args.settle, 0, on_chunk)
    if rank == 0:
        np.savez(args.out, rollout=np.concatenate(got, 0), env_groups=np.int32(groups), world=np.int32(world))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
