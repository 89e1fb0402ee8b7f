"""Dev probe: is the four-env part B wrong on the first launch, on repeated launches within one
handle, or on a handle whose buffers reuse a closed handle's memory?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
A = ABI.load_scene(); md = ABI.ModelDesc(A)
P, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(1024)), impairment='random')
N = 4096
S = np.tile(P.astype(np.float32), (4, 1))
ref = _lib.Sim(md, N, flags=1); ref.set_state(S); ref.settle(20); S0 = ref.get_state()
ref.set_state(S0); ref.substep(0.01); R1 = ref.get_state()
def bad(G):
    d = np.abs(G[:, :28] - R1[:, :28]).max(1)
    return int(np.count_nonzero(d > 1e-3))
h1 = _lib.Sim(md, N, flags=0)       # created while ref is alive: fresh memory
for rep in range(3):
    h1.set_state(S0); h1.substep(0.01); print('h1 (fresh memory) rep', rep, 'bad', bad(h1.get_state()), flush=True)
h2 = _lib.Sim(md, N, flags=0)       # second live handle
h2.set_state(S0); h2.substep(0.01); print('h2 (second live handle) bad', bad(h2.get_state()), flush=True)
h1.set_state(S0); h1.substep(0.01); print('h1 again after h2 ran, bad', bad(h1.get_state()), flush=True)
ref.set_state(S0); ref.substep(0.01); print('ref (one-env B) again, bad', bad(ref.get_state()), flush=True)
h1.close()
h3 = _lib.Sim(md, N, flags=0)       # likely reuses h1's memory
h3.set_state(S0); h3.substep(0.01); print('h3 (after h1 closed) bad', bad(h3.get_state()), flush=True)
