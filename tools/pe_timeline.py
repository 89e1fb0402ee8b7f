"""Policy-eval timeline (GPU box, under rocprofv3 --kernel-trace): 60 harness steps with the eager
policy, then 60 with the graph-replayed one; then (with ANALYZE=<db dir>) the gap between one env
step's last kernel and the next env step's first, and the policy kernels that run in it.

    rocprofv3 --kernel-trace -d gpurun_out/pt -o pt -- python3 tools/pe_timeline.py
    ANALYZE=gpurun_out/pt python3 tools/pe_timeline.py
"""
import glob
import os
import sqlite3
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))


def analyze(d):
    f = sorted(glob.glob(os.path.join(d, '**', '*.db'), recursive=True))[0]
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute('pragma table_info(kernels)')]
    rows = c.execute('select name, start, "end" from kernels order by start').fetchall()
    print('columns', cols[:12])
    if os.environ.get('DUMP'):
        t0 = rows[0][1]
        mid = len(rows) // 4
        for r in rows[mid:mid + 160]:
            print('%10.1f %8.1f %s' % ((r[1] - t0) / 1e3, (r[2] - r[1]) / 1e3, r[0][:70]))
    takes = [i for i, r in enumerate(rows) if 'avr_take_step_kernel' in r[0]]
    # one take_step per env group: a step starts at the first of a cluster
    steps = [i for k, i in enumerate(takes) if k == 0 or rows[i][1] - rows[takes[k - 1]][1] > 500e3]
    out = []
    for a, b in zip(steps[:-1], steps[1:]):
        seg = rows[a:b]
        sim = [r for r in seg if r[0].startswith('avr_')]
        pol = [r for r in seg if not r[0].startswith('avr_')]
        last_sim_end = max(r[2] for r in sim)
        nxt = rows[b][1]
        out.append((nxt - rows[a][1], nxt - last_sim_end, len(pol), sum(r[2] - r[1] for r in pol)))
    out = np.array(out, float) / np.array([1e3, 1e3, 1, 1e3])
    half = len(out) // 2
    for name, o in (('eager', out[5:half]), ('graph', out[half + 5:])):
        print(name, 'step us median %.0f, gap after the env step %.0f us, policy kernels %d, their busy time %.0f us'
              % tuple(np.median(o, 0)))


def run():
    import torch
    from avr import policy_eval as PE
    from avr.env import AVRTorchVecEnv
    E = int(os.environ.get('ENVS', 4096))
    env = AVRTorchVecEnv('FeedingJaco-v0', E, device=0, seed=1001, auto_reset=False)
    L = env.L
    torch.manual_seed(0)
    pol = PE.ActorCritic(L.OBS_DIM, L.ACT_DIM).to(env.dev).eval()
    rms = PE.DeviceRMS(PE.RunningMeanStd((L.OBS_DIM,)), env.dev)
    hxs = torch.zeros(E, 1, device=env.dev)
    masks = torch.zeros(E, 1, device=env.dev)
    obs = env.reset()[:, :env.obs_robot_len]
    for _ in range(60):
        with torch.no_grad():
            _, a, _, _ = pol.act(PE.normalize(obs, rms), hxs, masks, deterministic=False)
        obs = env.step(a)[0][:, :env.obs_robot_len]
    policy = PE._graphed_policy(pol, rms, obs, hxs, masks, False)
    for _ in range(60):
        obs = env.step(policy(obs, masks))[0][:, :env.obs_robot_len]
    torch.cuda.synchronize()
    env.close()


if __name__ == '__main__':
    if os.environ.get('ANALYZE'):
        analyze(os.environ['ANALYZE'])
    else:
        run()
