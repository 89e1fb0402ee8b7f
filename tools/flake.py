"""Dev: bench-shaped run repeated in one process (set_state, settle, K random steps): per-rep
NaN/overflow flag count, state hash and wall time; a second Sim handle repeats it."""
import os, sys, time, hashlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
A = ABI.load_scene(); md = ABI.ModelDesc(A)
P, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(min(N, 1024))), impairment='random')
S = np.tile(P, ((N + len(P) - 1) // len(P), 1))[:N].astype(np.float32)
outs = []
for h in range(2):
    sim = _lib.Sim(md, N, seed=1001)
    for rep in range(2):
        sim.set_state(S)
        t0 = time.perf_counter(); sim.settle(100); sim.sync(); t1 = time.perf_counter()
        S1 = sim.get_state()
        fl1 = int(np.count_nonzero(S1[:, ABI.S_TASK + ABI.T_FLAGS]))
        t2 = time.perf_counter()
        for k in range(K):
            sim.step(_lib.random_actions(1001, np.arange(N), k))
        sim.sync(); t3 = time.perf_counter()
        G = sim.get_state()
        fl = G[:, ABI.S_TASK + ABI.T_FLAGS]
        outs.append(G)
        print('handle', h, 'rep', rep, 'settle sha', hashlib.sha1(S1.tobytes()).hexdigest()[:10], 'flag', fl1,
              'settle s %.2f' % (t1 - t0), '| step sha', hashlib.sha1(G.tobytes()).hexdigest()[:10], 'flag', int(np.count_nonzero(fl)),
              'steps s %.2f' % (t3 - t2), 'bad envs', np.nonzero(fl)[0][:12].tolist(), flush=True)
    sim.close()
for i in range(1, len(outs)):
    d = np.abs(outs[0] - outs[i]).max(1)
    print('rep0 vs', i, 'differing envs', int(np.count_nonzero(d)), 'first', np.nonzero(d)[0][:10].tolist())
