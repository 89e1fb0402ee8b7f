"""Dev check: avr_settle(100) (back-to-back launches) vs 200 x avr_substep (host sync between)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states(A, md, 1001, list(range(N)))
S = S.astype(np.float32)
a = _lib.Sim(md, N); a.set_state(S); a.settle(100); Sa = a.get_state()
b = _lib.Sim(md, N); b.set_state(S)
for k in range(200):
    b.substep(0.01)
Sb = b.get_state()
c = _lib.Sim(md, N); c.set_state(S); c.settle(100); Sc = c.get_state()
print('groups', os.environ.get('AVR_ENV_GROUPS', '2'), 'settle vs substeps max|dq|', np.abs(Sa[:, :10] - Sb[:, :10]).max(1),
      'settle vs settle', np.abs(Sa[:, :10] - Sc[:, :10]).max(), 'flags', Sa[:, ABI.S_TASK + ABI.T_FLAGS], flush=True)
