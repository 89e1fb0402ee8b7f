"""Env sharding + rollout all-gather (the multi-GPU data path of bench.py) on CPU with gloo,
world_size 2: the gathered rollout equals the single-process rollout of all global envs."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_step(env_ids, t):
    """Deterministic per-global-env outputs standing in for a sim step (host Philox actions)."""
    from avr import _lib
    a = _lib.random_actions(1001, env_ids, t).astype(np.float32)
    obs = np.concatenate([a, a, a, a[:, :4]], 1)            # 25
    rew = a.sum(1)
    info = a[:, :2] * 3
    done = (a[:, 0] > 0.5).astype(np.uint8)
    return obs, rew, info, done


def _worker(rank, world, port, E, G, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'assistive-vr-gym_amd'))
    from avr import dist as D
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    off, n = D.shard(E, rank)
    ids = np.arange(off, off + n)
    roll = torch.zeros(G, E, D.ROLL_WIDTH)
    for j in range(G):
        obs, rew, info, done = _fake_step(ids, j)
        D.pack_rollout(roll, j, torch.from_numpy(obs), torch.from_numpy(rew), torch.from_numpy(info), torch.from_numpy(done))
    out = D.gather_rollouts(roll)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_rollout_gather_world2_matches_single_process():
    import sys
    from avr import dist as D
    world, E, G = 2, 6, 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, E, G, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ids = np.arange(world * E)
    for j in range(G):
        obs, rew, info, done = _fake_step(ids, j)
        assert np.array_equal(got[j, :, :25], obs)
        assert np.array_equal(got[j, :, 25], rew)
        assert np.array_equal(got[j, :, 26:28], info)
        assert np.array_equal(got[j, :, 28], done.astype(np.float32))


def test_shard_blocks_cover_global_ids():
    from avr import dist as D
    seen = []
    for r in range(8):
        off, n = D.shard(4096, r)
        seen.extend(range(off, off + n))
    assert seen == list(range(8 * 4096))
