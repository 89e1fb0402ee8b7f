"""Dev check: GPU step vs CPU oracle on a few envs (prints max deviations)."""
import sys, time, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
from oracle.oracle import Oracle
if len(sys.argv) > 3:
    _lib.LIB_PATH = os.path.join(ROOT, 'assistive-vr-gym_amd', 'avr', sys.argv[3]); _lib.load(_lib.LIB_PATH)

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, meta = RS.batch_reset_states(A, md, 1001, list(range(N)))
sim = _lib.Sim(md, N)
print('kernel', sim.kernel_info(), flush=True)
o = Oracle(md, N)
o.set_state(S); sim.set_state(S.astype(np.float32))
# one substep
sim.substep(0.01); o.substep(0.01)
G, C = sim.get_state(), o.get_state()
print('1 substep: max|dq|', np.abs(G[:, :10] - C[:, :10]).max(), 'max|dfree|', np.abs(G[:, ABI.S_FREE:ABI.S_FREE+130] - C[:, ABI.S_FREE:ABI.S_FREE+130]).max(),
      'ncp', G[:, ABI.S_TASK+ABI.T_NCP], C[:, ABI.S_TASK+ABI.T_NCP], 'flags', G[:, ABI.S_TASK+ABI.T_FLAGS], flush=True)
o.set_state(S); sim.set_state(S.astype(np.float32))
t = time.time(); og = sim.settle(100); print('gpu settle', time.time() - t, flush=True)
oc = o.settle(100)
G, C = sim.get_state(), o.get_state()
print('settle: obs max diff', np.abs(og - oc).max(), 'q diff', np.abs(G[:, :10] - C[:, :10]).max(),
      'ncp', G[:, ABI.S_TASK+ABI.T_NCP], C[:, ABI.S_TASK+ABI.T_NCP], 'flags', G[:, ABI.S_TASK+ABI.T_FLAGS], flush=True)
# steps with identical actions
worst = 0
for k in range(K):
    a = _lib.random_actions(1001, np.arange(N), k)
    og, rg, dg, ig = sim.step(a)
    oc, rc, dc, ic = o.step(a)
    G, C = sim.get_state(), o.get_state()
    dq = np.abs(G[:, :7] - C[:, :7]).max()
    worst = max(worst, dq)
    if k % 5 == 0 or k == K - 1:
        print('step', k, 'max|dq_arm|', dq, 'obs', np.abs(og - oc).max(), 'rew', np.abs(rg - rc).max(), 'info', np.abs(ig - ic).max(), flush=True)
print('worst arm dq', worst)
# contact-rich chaos envelope of tests/test_gpu_parity.py (settle + steps): a build past it fails
TOL = 3e-3
if not worst < TOL:
    print('FAIL: worst arm dq %.3g >= %.3g' % (worst, TOL))
    sys.exit(1)
print('flags', G[:, ABI.S_TASK+ABI.T_FLAGS], C[:, ABI.S_TASK+ABI.T_FLAGS])
