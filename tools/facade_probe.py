"""Facade step-rate probe (development): AVRTorchVecEnv, chunks of 10 synchronised steps across an
episode boundary; prints env-steps/s per chunk.   python tools/facade_probe.py [task] [prefetch 0/1]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))

import torch  # noqa: E402
from avr import env as EV  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else 'FeedingJaco-v0'
pf = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
E = 4096
dev = torch.device('cuda', 0)
v = EV.AVRTorchVecEnv(task, E, device=0, prefetch=pf)
v.reset()
act = torch.empty(E, v.L.ACT_DIM, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(1001)
torch.cuda.synchronize(dev)
rates = []
for c in range(30):
    t0 = time.perf_counter()
    roll = False
    for k in range(10):
        act.uniform_(-1, 1, generator=g)
        _, _, _, info = v.step(act)
        roll = roll or 'terminal_observation' in info
    torch.cuda.synchronize(dev)
    rates.append((c * 10, round(E * 10 / (time.perf_counter() - t0)), roll))
print(task, 'prefetch', pf, rates, flush=True)
v.close()
