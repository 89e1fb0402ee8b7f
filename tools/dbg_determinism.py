"""Run-to-run determinism of the BedBathing step on the wiping states (fresh handles, repeated
steps): every repetition must give the same bits."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'assistive-vr-gym_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
from avr import _abi as ABI, _lib, reset_bedbath as RBB
import bedbath_util as BU
import test_bedbath as TB

BB = ABI.BB
A = ABI.load_scene(ABI.TASK_BEDBATH)
md = ABI.ModelDesc(A)
settled = RBB.settled_arms(A, md, runner=TB._oracle_runner(md))
S, meta = RBB.batch_reset_states(A, md, 1001, list(range(8)), attempts=12, iters=80, settled=settled)
W, ks = BU.wipe_states(A, md, S)
W32 = W.astype(np.float32)
wb = slice(BB.S_TASK + BB.T_WIPE, BB.S_TASK + BB.T_WIPE + 6)
outs = []
for rep in range(int(os.environ.get('REPS', 6))):
    n = len(W32) * (1 + rep % 3)            # also inside bigger batches
    sim = _lib.Sim(md, n)
    sim.set_state(np.tile(W32, (n // len(W32), 1)))
    sim.step(np.zeros((n, 7), np.float32))
    G = sim.get_state()[:len(W32)]
    sim.close()
    outs.append(G)
    print(rep, n, G[:, wb][:, 0].astype(int).tolist(), 'same as rep 0:', bool(np.array_equal(G, outs[0])),
          'max diff', float(np.abs(G - outs[0]).max()), flush=True)
