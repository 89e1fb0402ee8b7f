"""Bit-identity fingerprint of the shipped kernels: reset states (FeedingJaco: impairment 'random'
and 100 settle frames; TASK=1/2: the PR2 tasks' bench reset pool), then K gym steps of Philox
random actions.  Writes every step's obs / reward /
info and the final state to an .npz, so that a refactor of the kernels can be checked bit for bit
against a run of the previous build (python tools/fingerprint.py OUT.npz [REF.npz]).
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.environ.get("AVR_FP_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)


def run(n=512, k=20, lib=None):
    from avr import _abi as ABI, reset as RS, _lib
    task = int(os.environ.get('TASK', '0'))
    A = ABI.load_scene(task)
    md = ABI.ModelDesc(A)
    states = os.environ.get('FP_STATES')      # initial states shared by an A/B pair of runs
    if states and os.path.exists(states):
        S = np.load(states)['S']
    elif task == 0:
        S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(n)), impairment='random')
    else:
        import bench
        S, _ = bench.reset_pool(task, A, md, list(range(32)), 'random')
        S = np.tile(S, ((n + len(S) - 1) // len(S), 1))[:n]
    if states and not os.path.exists(states):
        np.savez_compressed(states, S=S)
    sim = _lib.Sim(md, n, seed=1001)
    sim.set_state(S.astype(np.float32))
    sim.settle(100 if task == 0 else 0)
    out = dict(settle=sim.get_state())
    obs, rew, info = [], [], []
    for t in range(k):
        o, r, d, i = sim.step(_lib.random_actions(1001, np.arange(n), t))
        obs.append(o); rew.append(r); info.append(i)
    out.update(obs=np.stack(obs), rew=np.stack(rew), info=np.stack(info), state=sim.get_state())
    sim.close()
    return out


if __name__ == '__main__':
    out = run()
    np.savez_compressed(sys.argv[1], **out)
    for key, v in out.items():
        print(key, hashlib.sha1(np.ascontiguousarray(v).tobytes()).hexdigest()[:12])
    if len(sys.argv) > 2:
        ref = np.load(sys.argv[2])
        bad = [key for key in out if not np.array_equal(out[key], ref[key], equal_nan=True)]
        print('bit-identical to', sys.argv[2] if not bad else 'DIFFERS in %s' % bad)
        sys.exit(1 if bad else 0)
