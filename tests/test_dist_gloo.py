"""Env sharding + rollout all-gather (the multi-GPU data path of bench.py) on CPU with gloo,
world_size 2: each rank simulates its shard of global env ids on the CPU oracle (reset states
and actions keyed by global id, as on the GPUs) and the gathered rollout equals the
single-process rollout of all global envs, bit for bit."""
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


SETTLE, G = 20, 3


def _rollout(ids, steps):
    """FeedingJaco rollout of the global envs `ids` on the CPU oracle: reset states from the host
    reset path keyed by global id, a settle, then `steps` gym steps of the Philox action stream --
    what one rank of bench.py runs on its shard (the oracle stands in for the GPU)."""
    from avr import _abi as ABI, _lib, reset as RS
    from oracle.oracle import Oracle
    A = ABI.load_scene()
    md = ABI.ModelDesc(A)
    S, _ = RS.batch_reset_states_fast(A, md, 1001, list(ids), impairment='random')
    o = Oracle(md, len(ids))
    o.set_state(S)
    o.settle(SETTLE)
    out = []
    for t in range(steps):
        obs, rew, done, info = o.step(_lib.random_actions(1001, np.asarray(ids), t))
        out.append((obs, rew, info, done.astype(np.uint8)))
    return out


def _worker(rank, world, port, E, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, 'assistive-vr-gym_amd'))
    sys.path.insert(0, root)
    from avr import dist as D
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    off, n = D.shard(E, rank)
    roll = torch.zeros(G, E, D.ROLL_WIDTH)
    for j, (obs, rew, info, done) in enumerate(_rollout(np.arange(off, off + n), G)):
        D.pack_rollout(roll, j, torch.from_numpy(obs), torch.from_numpy(rew), torch.from_numpy(info), torch.from_numpy(done))
    out = D.gather_rollouts(roll)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_rollout_gather_world2_matches_single_process():
    """Two gloo ranks, each simulating its shard (env_offset = rank x E) and packing its rollout as
    bench.py does; the all-gathered rollout equals one process simulating all global envs."""
    world, E = 2, 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, E, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref = _rollout(np.arange(world * E), G)
    for j, (obs, rew, info, done) in enumerate(ref):
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
