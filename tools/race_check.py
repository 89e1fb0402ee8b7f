"""Dev check: run-to-run determinism of the step kernel at scale (a data race shows up as
bitwise differences between two identical runs) and NaN/overflow flag counts."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
so = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
_lib.LIB_PATH = os.path.join(ROOT, 'assistive-vr-gym_amd', 'avr', so)
_lib.load(_lib.LIB_PATH)
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(min(N, 256))))
S = np.tile(S, ((N + len(S) - 1) // len(S), 1))[:N].astype(np.float32)
sim = _lib.Sim(md, N)
sim.set_state(S); sim.settle(100)
S0 = sim.get_state()
outs = []
for rep in range(2):
    sim.set_state(S0)
    for k in range(K):
        sim.step(_lib.random_actions(1001, np.arange(N), k))
    outs.append(sim.get_state())
d = np.abs(outs[0] - outs[1])
bad = np.nonzero(d.max(1) > 0)[0]
fl = outs[0][:, ABI.S_TASK + ABI.T_FLAGS]
# tiled envs share initial states: env e and e+256 must match bitwise too
tile = np.abs(outs[0][:256] - outs[0][256:512]).max(1) if N >= 512 else np.zeros(1)
import hashlib
print(so, 'sha', hashlib.sha1(outs[0].tobytes()).hexdigest()[:12], 'N', N, 'K', K, 'nondeterministic envs', len(bad), 'max diff', d.max(), 'flagged', int(np.count_nonzero(fl)),
      'tile-mismatch envs', int(np.count_nonzero(tile)), 'arm |q| max', np.abs(outs[0][:, :7]).max(), flush=True)
