"""Diagnostic: the state after each of K single sub-steps from one initial state (the fingerprint's
reset states), for locating where two builds' results part (tools/fingerprint.py says only that
they do).

    AVR_LIB=<lib> TASK=<t> python tools/substep_dump.py OUT.npz [K]
    python tools/substep_dump.py --cmp A.npz B.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)


def dump(out, K):
    from avr import _abi as ABI, reset as RS, _lib
    task = int(os.environ.get('TASK', '0'))
    A = ABI.load_scene(task)
    md = ABI.ModelDesc(A)
    n = 512
    if task == 0:
        S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(n)), impairment='random')
    else:
        import bench
        S, _ = bench.reset_pool(task, A, md, list(range(32)), 'random')
        S = np.tile(S, ((n + len(S) - 1) // len(S), 1))[:n]
    sim = _lib.Sim(md, n, seed=1001)
    sim.set_state(S.astype(np.float32))
    dt = 0.02
    states = []
    for k in range(K):
        sim.substep(dt)
        states.append(sim.get_state())
    sim.close()
    np.savez_compressed(out, S=np.stack(states))


def cmp(a, b):
    from avr import _abi as ABI
    A = np.load(a)['S']
    B = np.load(b)['S']
    L = ABI.ModelDesc(ABI.load_scene(int(os.environ.get('TASK', '0')))).layout
    names = {v: k for k, v in vars(L).items() if k.startswith('S_') and isinstance(v, int)}
    starts = sorted(names)
    for k in range(len(A)):
        d = np.argwhere(~((A[k] == B[k]) | (np.isnan(A[k]) & np.isnan(B[k]))))
        if len(d):
            envs = np.unique(d[:, 0])
            cols = np.unique(d[:, 1])
            lab = [names[max(s for s in starts if s <= c)] + '+%d' % (c - max(s for s in starts if s <= c)) for c in cols[:12]]
            e = envs[0]
            c0 = d[d[:, 0] == e][:, 1]
            print('substep %d: %d envs differ (first %s), columns %s' % (k, len(envs), envs[:8].tolist(), lab))
            print('  env %d: %s' % (e, [(int(c), float(A[k, e, c]), float(B[k, e, c])) for c in c0[:8]]))
            return
    print('identical over %d sub-steps' % len(A))


if __name__ == '__main__':
    if sys.argv[1] == '--cmp':
        cmp(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
