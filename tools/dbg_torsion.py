"""GPU vs fp32 oracle after one sub-step / one step from BedBathing wiping states, with the
rolling / spinning coefficients as compiled and zeroed (debugging the torsional rows)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'assistive-vr-gym_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
from avr import _abi as ABI, _lib, reset_bedbath as RBB
from oracle.oracle import Oracle
import bedbath_util as BU

BB = ABI.BB
A0 = dict(np.load(os.path.join(os.path.dirname(ABI.__file__), 'data', 'bed_bathing_pr2.npz')))
md0 = ABI.ModelDesc(A0)
if os.environ.get('DBG_FIXTURE'):      # tests/test_bedbath.py's states: arms settled by the fp64 oracle
    import test_bedbath as TB
    settled = RBB.settled_arms(A0, md0, runner=TB._oracle_runner(md0))
    S, meta = RBB.batch_reset_states(A0, md0, 1001, list(range(8)), attempts=12, iters=80, settled=settled)
else:
    S, meta = RBB.batch_reset_states(A0, md0, 1001, list(range(8)))
W, ks = BU.wipe_states(A0, md0, S)
nd = int(A0['n_dof'])
for variant in ('compiled', 'zero'):
    A = dict(A0)
    if variant == 'zero':
        A['body_rolling'] = np.zeros_like(A0['body_rolling'])
        A['body_spinning'] = np.zeros_like(A0['body_spinning'])
    md = ABI.ModelDesc(A)
    for what in ('substep', 'step'):
        sim = _lib.Sim(md, len(W))
        o = Oracle(md, len(W), 'f32')
        W32 = W.astype(np.float32)
        sim.set_state(W32); o.set_state(W32.astype(np.float64))
        if what == 'substep':
            sim.substep(0.02); o.substep(0.02)
        else:
            z = np.zeros((len(W), 7), np.float32)
            sim.step(z); o.step(z)
        G, C = sim.get_state(), o.get_state()
        dq = np.abs(G[:, BB.S_Q:BB.S_Q + nd] - C[:, BB.S_Q:BB.S_Q + nd]).max(1)
        dqd = np.abs(G[:, BB.S_QD:BB.S_QD + nd] - C[:, BB.S_QD:BB.S_QD + nd]).max(1)
        df = np.abs(G[:, BB.S_FREE:BB.S_FREE + 13] - C[:, BB.S_FREE:BB.S_FREE + 13]).max(1)
        ncg, ncc = G[:, BB.S_TASK + BB.T_NCP], C[:, BB.S_TASK + BB.T_NCP]
        wb = slice(BB.S_TASK + BB.T_WIPE, BB.S_TASK + BB.T_WIPE + 6)
        print('wipe bits equal', [bool(np.array_equal(G[e, wb], C[e, wb].astype(np.float32))) for e in range(len(W))],
              G[:, wb][:, 0].astype(int).tolist(), C[:, wb][:, 0].astype(int).tolist())
        print(variant, what, 'dq', np.array2string(dq, precision=2), 'dqd', np.array2string(dqd, precision=2), 'dfree', np.array2string(df, precision=2),
              'ncp', ncg.astype(int).tolist(), ncc.astype(int).tolist(), flush=True)
        sim.close()

# contact pools of the worst envs, initial state and after one sub-step
np.set_printoptions(precision=5, suppress=True, linewidth=200)
sim = _lib.Sim(md0, len(W))
o = Oracle(md0, len(W), 'f32')
W32 = W.astype(np.float32)
sim.set_state(W32); o.set_state(W32.astype(np.float64))
print('initial ncp', W32[:, BB.S_TASK + BB.T_NCP])
sim.substep(0.02); o.substep(0.02)
G, C = sim.get_state(), o.get_state()
for e in (5, 7, 0):
    for name, X in (('gpu', G), ('orc', C)):
        n = int(X[e, BB.S_TASK + BB.T_NCP])
        P = X[e, BB.S_CP:BB.S_CP + 16 * n].reshape(n, 16)
        print(e, name)
        print(P[:, [0, 1, 8, 9, 10, 11, 12, 13, 14]])
    print(e, 'free gpu', G[e, BB.S_FREE:BB.S_FREE + 13])
    print(e, 'free orc', C[e, BB.S_FREE:BB.S_FREE + 13])
