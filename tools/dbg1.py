"""Dev: one sub-step GPU vs oracle, per state section."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
from oracle.oracle import Oracle
N = 4
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, meta = RS.batch_reset_states(A, md, 1001, list(range(N)))
print('initial ncp', S[:, ABI.S_TASK + ABI.T_NCP])
sim = _lib.Sim(md, N); o = Oracle(md, N)
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    if k == 0:
        o.set_state(S); sim.set_state(S.astype(np.float32))
    sim.substep(0.01); o.substep(0.01)
    G, C = sim.get_state(), o.get_state()
    secs = [('q', ABI.S_Q, ABI.S_Q + 14), ('qd', ABI.S_QD, ABI.S_QD + 14), ('free', ABI.S_FREE, ABI.S_FREE + 130), ('task', ABI.S_TASK, ABI.S_TASK + 16)]
    line = []
    for nm, a, b in secs[:3]:
        d = np.abs(G[:, a:b] - C[:, a:b])
        line.append('%s %.2e@%s' % (nm, d.max(), np.unravel_index(d.argmax(), d.shape)))
    print(k, ' '.join(line), 'ncp', G[:, ABI.S_TASK + ABI.T_NCP], C[:, ABI.S_TASK + ABI.T_NCP])
    for e in range(0):
        print(' qd gpu', np.round(G[e, ABI.S_QD:ABI.S_QD + 10], 4))
        print(' qd ora', np.round(C[e, ABI.S_QD:ABI.S_QD + 10], 4))
        fb = (G[e, ABI.S_FREE:ABI.S_FREE + 130] - C[e, ABI.S_FREE:ABI.S_FREE + 130]).reshape(10, 13)
        print(' free diff per body (pos, quat, v, w)', np.round(np.abs(fb).max(1), 4))
