"""Dev probe: 100-frame settle of tiled reset states at several batch sizes and part-B configs;
flagged-env counts and where they sit (env // 256), to localise a scale-dependent failure."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
A = ABI.load_scene(); md = ABI.ModelDesc(A)
P, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(1024)), impairment='random')
P = P.astype(np.float32)
CONFIGS = [(4096, 1, 100), (4096, 0, 100), (4096, 2, 100), (1024, 0, 100), (512, 0, 100), (256, 0, 100),
           (4096, 0, 10), (4096, 0, 1)]
if os.environ.get('PROBE_SHORT'):
    CONFIGS = [(4096, 0, 100), (1024, 0, 100)]
print('lib', _lib.LIB_PATH, flush=True)
for N, flags, frames in CONFIGS:
    S = np.tile(P, ((N + 1023) // 1024, 1))[:N]
    sim = _lib.Sim(md, N, flags=flags)
    sim.set_state(S)
    sim.settle(frames)
    G = sim.get_state()
    fl = G[:, ABI.S_TASK + ABI.T_FLAGS].astype(int)
    bad = np.nonzero(fl)[0]
    h = np.bincount(bad // 256, minlength=N // 256) if len(bad) else []
    print('N', N, 'flags', flags, 'frames', frames, 'flagged', len(bad), 'first', bad[:8].tolist(), 'per-256', list(h), flush=True)
    sim.close()
