"""The multi-rank data path on the HIP backend: two ranks (torch.distributed.run, gloo) share the
one GPU, each steps its shard of global env ids through libavr in stacked rollouts and all-gathers
them (tests/gpu_dist_worker.py, bench.py's multi-GPU flow).  The gathered rollout must equal one
process stepping all 2E envs, bit for bit: env ids, reset states and Philox actions are keyed by
the global id, and the kernels' results do not depend on the env-group layout (2 groups per rank
vs 4 in the single process)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_two_rank_hip_rollouts_gather_equal_single_process(tmp_path):
    import torch
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import gpu_dist_worker as W
    from avr import dist as D
    E, chunks, G = 2048, 2, 16
    out = str(tmp_path / 'gathered.npz')
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.join(ROOT, 'tests', 'gpu_dist_worker.py'), '--out', out,
           '--envs', str(E), '--chunks', str(chunks), '--G', str(G)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-4000:]
    z = np.load(out)
    got = z['rollout']
    assert int(z['world']) == 2 and got.shape == (chunks * G, 2 * E, D.roll_width(25))

    md, S = W.initial_states(0, 2 * E)
    Wd = D.roll_width(md.layout.OBS_DIM)
    roll = torch.zeros(G, 2 * E, Wd, device=torch.device('cuda', 0))
    ref = []

    def on_chunk(c, so, sr, sd, si):
        D.pack_rollout_stacked(roll, so, sr, si, sd, G)
        ref.append(roll.cpu().numpy().copy())

    groups = W.run_shard(md, S, 0, 2 * E, chunks, G, 20, 0, on_chunk)
    ref = np.concatenate(ref, 0)
    assert groups > int(z['env_groups'])           # the layouts differ: 4 groups here, 2 per rank there
    assert np.isfinite(ref).all() and ref[..., md.layout.OBS_DIM].std() > 0      # live rewards, not zeros
    bad = np.argwhere(got != ref)
    assert bad.size == 0, 'first mismatches (step, env, column): %s' % bad[:5].tolist()
