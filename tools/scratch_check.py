"""ScratchItchPR2 GPU-vs-oracle check (development): one sub-step, then K gym steps of Philox
actions on N envs; prints the worst joint / free-body / reward / obs differences per phase."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

from avr import _abi as ABI, _lib, reset_scratch as RSS   # noqa: E402
from oracle.oracle import Oracle                          # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
SI = ABI.SI
A = ABI.load_scene(ABI.TASK_SCRATCH)
md = ABI.ModelDesc(A)
nd = md.n_dof + int(A['hc_n'])
t0 = time.time()
S, meta = RSS.batch_reset_states(A, md, 1001, range(N), attempts=20, iters=100)
print('reset %.1fs' % (time.time() - t0), [m['impairment'] for m in meta], flush=True)
S32 = S.astype(np.float32)
sim = _lib.Sim(md, N)
print('kernel info', sim.kernel_info(), flush=True)
o = Oracle(md, N)
o.set_threads(8)
sim.set_state(S32)
o.set_state(S32.astype(np.float64))
sim.substep(0.02)
o.substep(0.02)
G, C = sim.get_state(), o.get_state()
print('substep: dq %.3g  free %.3g' % (np.abs(G[:, :nd] - C[:, :nd]).max(),
                                       np.abs(G[:, SI.S_FREE:SI.S_FREE + 13] - C[:, SI.S_FREE:SI.S_FREE + 13]).max()), flush=True)
sim.set_state(S32)
o.set_state(S32.astype(np.float64))
ob0, oc0 = sim.settle(0), o.settle(0)
print('reset obs diff %.3g' % np.abs(ob0 - oc0).max(), flush=True)
worst = 0.0
for t in range(K):
    a = _lib.random_actions(1001, np.arange(N), t)
    g = sim.step(a)
    c = o.step(a)
    G, C = sim.get_state(), o.get_state()
    dq = np.abs(G[:, :nd] - C[:, :nd]).max()
    worst = max(worst, dq)
    if t % 10 == 9 or t == K - 1:
        print('step %d dq %.3g worst %.3g obs %.3g rew %.3g info %.3g ncp gpu %s cpu %s flags %s' % (
            t, dq, worst, np.abs(g[0] - c[0]).max(), np.abs(g[1] - c[1]).max(), np.abs(g[3] - c[3]).max(),
            G[:, SI.S_TASK + SI.T_NCP].astype(int).tolist()[:8], C[:, SI.S_TASK + SI.T_NCP].astype(int).tolist()[:8],
            G[:, SI.S_TASK + SI.T_FLAGS].astype(int).tolist()[:8]), flush=True)
sim.close()
