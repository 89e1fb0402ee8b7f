"""Dev: settle frame by frame, GPU vs oracle (max |dq|, max |dfree|, ncp)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
from oracle.oracle import Oracle
N = 8
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, meta = RS.batch_reset_states(A, md, 1001, list(range(N)))
sim = _lib.Sim(md, N); o = Oracle(md, N)
o.set_state(S); sim.set_state(S.astype(np.float32))
for k in range(int(sys.argv[1])):
    sim.settle(1); o.settle(1)
    G, C = sim.get_state(), o.get_state()
    dq = np.abs(G[:, :10] - C[:, :10]).max(1)
    df = np.abs(G[:, ABI.S_FREE:ABI.S_FREE + 130] - C[:, ABI.S_FREE:ABI.S_FREE + 130]).max(1)
    print(k, 'dq', np.array2string(dq, precision=1), 'dfree', np.array2string(df, precision=1), 'ncp', G[:, ABI.S_TASK + ABI.T_NCP].astype(int), C[:, ABI.S_TASK + ABI.T_NCP].astype(int), flush=True)
