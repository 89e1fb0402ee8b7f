"""Measure FeedingJaco GPU-vs-oracle agreement in the contact regime (development probe for the
tolerances of tests/test_gpu_parity.py): golden per-step obs / info / reward differences,
GPU vs fp32 oracle over 200 steps, and episode statistics vs the fp64 oracle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

from avr import _abi as ABI, _lib, reset as RS   # noqa: E402
from oracle.oracle import Oracle                  # noqa: E402

A = ABI.load_scene()
md = ABI.ModelDesc(A)
g = np.load(os.path.join(ROOT, 'tests', 'golden', 'feeding_golden.npz'))
n = len(g['env_ids'])
sim = _lib.Sim(md, n)
sim.set_state(g['S0'].astype(np.float32))
obs0 = sim.settle(100)
print('golden obs0 %.3g' % np.abs(obs0 - g['obs0']).max())
for t in range(g['actions'].shape[0]):
    ob, r, d, i = sim.step(g['actions'][t])
    print('golden t%d obs %.3g (cols>%s) rew %.3g info0 %s' % (t, np.abs(ob - g['obs'][t]).max(), np.argmax(np.abs(ob - g['obs'][t]).max(0)),
          np.abs(r - g['rew'][t]).max(), np.round(np.abs(i[:, 0] - g['info'][t][:, 0]), 3).tolist()))
sim.close()

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
S, meta = RS.batch_reset_states_fast(A, md, 1001, list(range(N)), impairment='random')
S32 = S.astype(np.float32)
sim = _lib.Sim(md, N)
o32 = Oracle(md, N, 'f32'); o32.set_threads(16)
o64 = Oracle(md, N); o64.set_threads(16)
sim.set_state(S32); o32.set_state(S32.astype(np.float64)); o64.set_state(S32.astype(np.float64))
t0 = time.time()
sim.settle(100); o32.settle(100); o64.settle(100)
print('settle %.1fs' % (time.time() - t0), flush=True)
R = {k: np.zeros(N) for k in ('g', 'c32', 'c64')}
for t in range(K):
    a = _lib.random_actions(1001, np.arange(N), t)
    x = sim.step(a); y = o32.step(a); z = o64.step(a)
    R['g'] += x[1]; R['c32'] += y[1]; R['c64'] += z[1]
    if t % 20 == 19:
        G, C32, C64 = sim.get_state(), o32.get_state(), o64.get_state()
        d32 = np.abs(G[:, :7] - C32[:, :7]).max(1)
        d64 = np.abs(G[:, :7] - C64[:, :7]).max(1)
        print('t%d dq vs f32: median %.2g p90 %.2g max %.2g | vs f64: median %.2g p90 %.2g max %.2g' % (
            t, np.median(d32), np.percentile(d32, 90), d32.max(), np.median(d64), np.percentile(d64, 90), d64.max()), flush=True)
G, C64 = sim.get_state(), o64.get_state()
L = ABI
for name, St in (('gpu', G), ('f64', C64)):
    succ = St[:, L.S_TASK + L.T_SUCCESS]
    alive = St[:, L.S_TASK + L.T_ALIVE].astype(int)
    hit = St[:, L.S_TASK + L.T_HIT].astype(int)
    print(name, 'eaten mean %.3f  alive mean %.3f  hit mean %.3f  success-rate %.3f' % (
        succ.mean(), np.mean([bin(x).count('1') for x in alive]), np.mean([bin(x).count('1') for x in hit]), np.mean(succ >= 6)))
print('episode reward mean gpu %.3f f32 %.3f f64 %.3f, std %.3f' % (R['g'].mean(), R['c32'].mean(), R['c64'].mean(), R['g'].std()))
