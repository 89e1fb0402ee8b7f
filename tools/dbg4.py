"""Dev: determinism + per-env parity of one sub-step from the reset states."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
from oracle.oracle import Oracle
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, meta = RS.batch_reset_states(A, md, 1001, list(range(N)))
sim = _lib.Sim(md, N); o = Oracle(md, N)
print('kernel', sim.kernel_info(), flush=True)
o.set_state(S); o.substep(0.01); C = o.get_state()
res = []
for rep in range(3):
    sim.set_state(S.astype(np.float32)); sim.substep(0.01); G = sim.get_state(); res.append(G)
    dq = np.abs(G[:, :10] - C[:, :10]).max(1)
    df = np.abs(G[:, ABI.S_FREE:ABI.S_FREE + 130] - C[:, ABI.S_FREE:ABI.S_FREE + 130]).max(1)
    print(rep, 'dq', np.array2string(dq, precision=1), 'dfree', np.array2string(df, precision=1), 'ncp', G[:, ABI.S_TASK + ABI.T_NCP].astype(int), flush=True)
print('rep-to-rep max diff', np.abs(res[0] - res[1]).max(), np.abs(res[0] - res[2]).max())
