"""Launch-shape debugging (tests/test_pr2_launch_shape.py): a pool of states tiled over 4096 envs;
after 1..5 steps, do the GPU copies of one pool state agree with each other (position
independence), and which picked envs differ from the fp32 oracle, by how much, in which DoF."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'assistive-vr-gym_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
from avr import _abi as ABI, _lib
import test_pr2_launch_shape as T

task = int(os.environ.get('TASK', 1))
A, md, L, P, isc = T._pool(task, 16)
E = int(os.environ.get('E', 4096))
S = np.tile(P, (E // len(P) + 1, 1))[:E]
src = np.tile(np.arange(len(P)), E // len(P) + 1)[:E]
PICK = T.PICK[T.PICK < E]
sim = _lib.Sim(md, E)
o = T._oracle(md, len(PICK), 'f32')
sim.set_state(S)
o.set_state(S[PICK].astype(np.float64))
nd = md.n_dof + (int(A['hc_n']) if task == ABI.TASK_SCRATCH else 0)
print('pool', len(P), 'contact states', int(isc.sum()), 'groups', sim.env_groups(), flush=True)
for t in range(5):
    a = (_lib.random_actions(1001, np.arange(E), t) * 0.2).astype(np.float32)
    # the same action for every copy of a pool state, so copies must stay bit-identical
    a = a[src]
    sim.step(a)
    o.step(a[PICK])
    G = sim.get_state()
    C = o.get_state()
    bad = []
    for k in range(len(P)):
        idx = np.nonzero(src == k)[0]
        d = np.abs(G[idx] - G[idx[0]]).max()
        if d > 0:
            bad.append((k, float(d), idx[np.abs(G[idx] - G[idx[0]]).max(1) > 0][:4].tolist()))
    dq = np.abs(G[PICK, :nd] - C[:, :nd])
    worst = np.argsort(-dq.max(1))[:4]
    print('step', t, 'copies differ:', bad[:6], flush=True)
    print('   oracle worst picks', [(int(PICK[w]), int(src[PICK[w]]), bool(isc[src[PICK[w]]]), float(dq[w].max()), int(dq[w].argmax())) for w in worst], flush=True)
sim.close()
