"""Diagnostic: per-step rates of the stepping forms a policy-in-the-loop caller can use (outputs of
every step synchronised back to the host stream), FeedingJaco at 4096 envs:
  step      avr_step_random_device (one graph of four group branches, forked and joined)
  roll1     avr_rollout_random_device(t, 1) (one graph per group on the group's stream, joined)
  roll16    avr_rollout_random_device(t, 16) per 16 steps (the bench headline's form)
python tools/step_modes.py [task] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

import numpy as np   # noqa: E402


def main():
    import bench
    from avr import _abi as ABI, _lib
    name = sys.argv[1] if len(sys.argv) > 1 else 'FeedingJaco-v0'
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    T = bench.TASKS[name]
    A = ABI.load_scene(T['task'])
    md = ABI.ModelDesc(A)
    E = 4096
    S, _ = bench.reset_pool(T['task'], A, md, list(range(T['pool'])), 'random')
    S = np.tile(S, (E // len(S) + 1, 1))[:E].astype(np.float32)
    sim = _lib.Sim(md, E, seed=1001)
    sim.set_state(S)
    sim.settle(T['settle'])
    t = 0
    res = {}
    for rnd in range(2):
        for mode in ('step', 'roll1', 'roll16'):
            for k in range(3):                  # warm: graph captures
                sim.step_random_device(t) if mode == 'step' else sim.rollout_random_device(t, 1)
                t += 1
            sim.sync()
            t0 = time.perf_counter()
            if mode == 'roll16':
                for k in range(0, K, 16):
                    sim.rollout_random_device(t, 16)
                    t += 16
            else:
                for k in range(K):
                    sim.step_random_device(t) if mode == 'step' else sim.rollout_random_device(t, 1)
                    t += 1
            sim.sync()
            el = time.perf_counter() - t0
            res.setdefault(mode, []).append(E * K / el)
            print('%s round %d: %.0f env-steps/s' % (mode, rnd, E * K / el), flush=True)
    sim.close()
    print({k: [round(v) for v in vs] for k, vs in res.items()})


if __name__ == '__main__':
    main()
