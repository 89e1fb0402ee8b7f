"""Diagnostic: run the step with one library build and dump the final state (A/B exactness checks).

    AVR_LIB=<lib.so> python tools/ab_state.py <out.npy> [n_envs] [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
from avr import _abi as ABI, reset as RS, _lib  # noqa: E402

out = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 512
K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
A = ABI.load_scene()
md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(min(N, 256))), impairment='random')
S = np.tile(S, ((N + len(S) - 1) // len(S), 1))[:N]
sim = _lib.Sim(md, N)
sim.set_state(S.astype(np.float32))
sim.settle(20)
for t in range(K):
    sim.step(_lib.random_actions(1001, np.arange(N), t))
np.save(out, sim.get_state())
print('saved', out)
