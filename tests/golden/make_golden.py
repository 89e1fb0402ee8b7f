"""Generate tests/golden/feeding_golden.npz from the fp64 CPU oracle (TEST INFRASTRUCTURE).

Inputs: 6 FeedingJaco-v0 reset states (host reset path, seed 1001): global env ids 0..3 with
impairment 'none' (static human) and 4..5 with impairment 'tremor' (motor-driven head/neck
chain), and Philox actions (seed 1001).  Expected outputs: the oracle's state after the 100-frame settle and
after each of 10 gym steps, with obs / reward / done / info per step.  These pin GPU == CPU
restatement; parity against PyBullet itself is unpinned (PyBullet is absent).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

from avr import _abi as ABI, reset as RS, _lib  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

N_STATIC, N_TREMOR, K, SEED = 4, 2, 10, 1001
N = N_STATIC + N_TREMOR


def main(out=os.path.join(HERE, 'feeding_golden.npz')):
    A = ABI.load_scene()
    md = ABI.ModelDesc(A)
    S_a, _ = RS.batch_reset_states_fast(A, md, SEED, list(range(N_STATIC)))
    S_b, _ = RS.batch_reset_states_fast(A, md, SEED, list(range(N_STATIC, N)), impairment='tremor')
    S0 = np.concatenate([S_a, S_b])
    S0 = S0.astype(np.float32).astype(np.float64)     # the GPU consumes float32 inputs
    o = Oracle(md, N)
    o.set_state(S0)
    obs0 = o.settle(100)
    S_settled = o.get_state()
    acts, obs, rew, done, info, states = [], [], [], [], [], []
    for t in range(K):
        a = _lib.random_actions(SEED, np.arange(N), t)
        ob, r, d, i = o.step(a)
        acts.append(a); obs.append(ob); rew.append(r); done.append(d); info.append(i); states.append(o.get_state())
    # expected states stored as float32 (the comparisons below are looser than fp32 rounding)
    np.savez_compressed(out, S0=S0, obs0=obs0, S_settled=S_settled.astype(np.float32), actions=np.array(acts), obs=np.array(obs),
                        rew=np.array(rew), done=np.array(done), info=np.array(info), states=np.array(states, np.float32),
                        seed=SEED, env_ids=np.arange(N), tremor=np.arange(N) >= N_STATIC)
    print(out, os.path.getsize(out))


if __name__ == '__main__':
    main()
