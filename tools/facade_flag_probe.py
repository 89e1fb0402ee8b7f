"""Facade slow-phase probe (development): the facade bench's 605 steps with rollovers, then 100
steps timed in synchronised chunks; prints the flagged envs (bits), and per-kernel launch times
over 5 steps of that phase.   python tools/facade_flag_probe.py [task]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))

import torch  # noqa: E402
from avr import env as EV  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else 'FeedingJaco-v0'
E = 4096
dev = torch.device('cuda', 0)
v = EV.AVRTorchVecEnv(task, E, device=0)
v.reset()
act = torch.empty(E, v.L.ACT_DIM, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(1001)
for k in range(605):
    act.uniform_(-1, 1, generator=g)
    _, _, _, info = v.step(act)
    if 'terminal_observation' in info or k % 50 == 0:
        torch.cuda.synchronize(dev)
        f = v.flags()
        print('step', k, 'roll' if 'terminal_observation' in info else '', 'flagged', np.nonzero(f)[0][:10].tolist(), f[f != 0][:10].tolist(), flush=True)
if v._prefetch:
    v._prefetch.wait()
torch.cuda.synchronize(dev)
rates = []
for c in range(10):
    t0 = time.perf_counter()
    for k in range(10):
        act.uniform_(-1, 1, generator=g)
        v.step(act)
    torch.cuda.synchronize(dev)
    rates.append(round(E * 10 / (time.perf_counter() - t0)))
print('chunks', rates, flush=True)
f = v.flags()
bad = np.nonzero(f)[0]
print('flagged', bad.tolist()[:20], f[bad].tolist()[:20])
S = v.get_state()
L = v.L
os.makedirs(os.path.join(ROOT, 'gpurun_out', 'fp'), exist_ok=True)
np.save(os.path.join(ROOT, 'gpurun_out', 'fp', 'flagged_states.npy'), S[bad[:8]])
for e in bad[:4]:
    print('env', e, 'iter', S[e, L.S_TASK + L.T_ITER], 'ncp', S[e, L.S_TASK + L.T_NCP], 'finite', bool(np.all(np.isfinite(S[e]))), 'q', S[e, :7])
v.sim.profile_kernels(True)
for k in range(5):
    act.uniform_(-1, 1, generator=g)
    v.step(act)
kt = v.sim.kernel_times()
v.sim.profile_kernels(False)
print({k: round(a / max(n, 1), 4) for k, (a, n) in kt.items()})
v.close()
