"""Dev probe: NaN-filled row scratch (AVR_DEBUG_NANFILL=1): a few sub-steps per part-B config;
a NaN in the state means some kernel read a row word nobody wrote."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
A = ABI.load_scene(); md = ABI.ModelDesc(A)
P, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(256)), impairment='random')
for N in (64, 1024):
    S = np.tile(P.astype(np.float32), (N // 256 + 1, 1))[:N]
    for flags in (1, 0, 2):
        sim = _lib.Sim(md, N, flags=flags); sim.set_state(S)
        out = []
        for k in range(3):
            sim.substep(0.01)
            G = sim.get_state()
            nan = ~np.isfinite(G[:, :ABI.S_CP]).all(1)
            out.append(int(nan.sum()))
        print('N', N, 'flags', flags, 'nan envs after substeps 1..3', out, 'first', np.nonzero(nan)[0][:8].tolist(), flush=True)
        sim.close()
