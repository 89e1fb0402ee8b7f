"""Dev check: (substep, set_state, settle) vs (set_state, settle) on the same handle, repeated."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.join(ROOT, 'assistive-vr-gym_amd', 'avr', sys.argv[1]); _lib.load(_lib.LIB_PATH)
N = 8
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states(A, md, 1001, list(range(N)))
S = S.astype(np.float32)
ref = _lib.Sim(md, N); ref.set_state(S); ref.settle(100); R = ref.get_state()
sim = _lib.Sim(md, N)
res = []
for rep in range(4):
    sim.set_state(S); sim.substep(0.01); sim.set_state(S); sim.settle(100)
    res.append(np.abs(sim.get_state()[:, :10] - R[:, :10]).max())
print(sys.argv[1:] or 'libavr.so', 'groups', os.environ.get('AVR_ENV_GROUPS', '2'), 'diff vs fresh settle per rep', res, flush=True)
