"""Where the policy-evaluation loop's time goes (GPU box): the stepping loop of
avr.policy_eval.evaluate at 4096 envs, timed as (a) env.step with a fresh torch.rand action tensor
only, (b) the policy forward only, (c) both (the harness), (d) the harness with the host clock
split between the policy call and env.step (no synchronisation, so it shows host issue time)."""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
import torch  # noqa: E402

from avr import policy_eval as PE, _abi as ABI  # noqa: E402
from avr.env import AVRTorchVecEnv  # noqa: E402

E, T = int(os.environ.get('ENVS', 4096)), int(os.environ.get('STEPS', 200))
name = os.environ.get('TASK', 'FeedingJaco-v0')
torch.manual_seed(0)
env = AVRTorchVecEnv(name, E, device=0, seed=1001, auto_reset=False)
L = env.L
pol = PE.ActorCritic(L.OBS_DIM, L.ACT_DIM).to(env.dev).eval()
rms = PE.RunningMeanStd((L.OBS_DIM,))
if not os.environ.get('HOST_RMS'):
    rms = PE.DeviceRMS(rms, env.dev)
hxs = torch.zeros(E, 1, device=env.dev)
masks = torch.zeros(E, 1, device=env.dev)
out = {}


def run(label, fn, steps):
    env.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = fn(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out[label] = dict(ms_per_step=dt / steps * 1e3, env_steps_per_s=E * steps / dt, host=host)


def step_only(steps):
    for _ in range(steps):
        env.step(torch.rand(E, L.ACT_DIM, device=env.dev) * 2 - 1)


def policy_only(steps):
    obs = env.t_obs[:, :env.obs_robot_len]
    for _ in range(steps):
        with torch.no_grad():
            pol.act(PE.normalize(obs, rms), hxs, masks, deterministic=False)


def harness(steps, split=False):
    obs = env.t_obs[:, :env.obs_robot_len].clone()
    tp = ts = 0.0
    for _ in range(steps):
        t0 = time.perf_counter()
        with torch.no_grad():
            _, action, _, _ = pol.act(PE.normalize(obs, rms), hxs, masks, deterministic=False)
        t1 = time.perf_counter()
        obs, rew, done, info = env.step(action)
        obs = obs[:, :env.obs_robot_len]
        t2 = time.perf_counter()
        tp += t1 - t0
        ts += t2 - t1
    return dict(policy_host_ms=tp / steps * 1e3, step_host_ms=ts / steps * 1e3) if split else None


def harness_graph(steps):
    obs = env.t_obs[:, :env.obs_robot_len].clone()
    policy = PE._graphed_policy(pol, rms, obs, hxs, masks, False)
    assert policy is not None
    torch.cuda.synchronize()
    for _ in range(steps):
        obs, rew, done, info = env.step(policy(obs, masks))
        obs = obs[:, :env.obs_robot_len]


run('warm', step_only, 5)
run('env_step_only', step_only, T)
run('policy_only', policy_only, T)
run('harness', harness, T)
run('harness_host_split', lambda s: harness(s, True), T)
run('harness_policy_graph', harness_graph, T)
env.close()
print(json.dumps(out))
