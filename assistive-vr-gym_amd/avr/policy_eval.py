"""Policy-evaluation harness: enjoy_vr.py's contract (enjoy_vr.py:61-120) on the batched backend.

What the reference does per trial: make the env with a setup() hook that fixes the participant's
gender / policy name (feeding.py:20-28), torch.load (actor_critic, ob_rms) from
trained_models/ppo/<Task><Robot>[New]-v0.pt, install ob_rms into the VecNormalize wrapper in eval
mode, reset, slice obs[:, :obs_robot_len], then 200 x {actor_critic.act(obs, hidden, masks,
deterministic) -> env.step(action)}.

Here: the trained policies are absent from the reference (trained_models/ppo/ holds only
__init__.py) and a2c_ppo_acktr is not importable, so the harness defines the same pieces itself
-- an actor-critic with that act() signature (Gaussian MLP policy), a RunningMeanStd ob_rms with
VecNormalize's eval-mode normalisation (clip((obs - mean) / sqrt(var + 1e-8), -10, 10)), and a
checkpoint format that loads with torch.load(weights_only=True) -- and evaluates on
AVRTorchVecEnv, n_envs episodes at once.  Policies are synthetic (random init) unless a
checkpoint saved by save_policy is given.
"""
import time

import numpy as np
import torch

CLIP_OBS, EPS = 10.0, 1e-8          # baselines VecNormalize defaults (clipob, epsilon)


class RunningMeanStd:
    """ob_rms: running mean / variance of observations (baselines RunningMeanStd semantics)."""

    def __init__(self, shape, mean=None, var=None, count=1e-4):
        self.mean = np.zeros(shape) if mean is None else np.asarray(mean, float)
        self.var = np.ones(shape) if var is None else np.asarray(var, float)
        self.count = float(count)

    def update(self, x):
        x = np.asarray(x, float)
        bm, bv, bc = x.mean(0), x.var(0), x.shape[0]
        d = bm - self.mean
        tot = self.count + bc
        self.mean = self.mean + d * bc / tot
        self.var = (self.var * self.count + bv * bc + d * d * self.count * bc / tot) / tot
        self.count = tot


class DeviceRMS:
    """ob_rms's mean / variance as device tensors, converted once: torch.as_tensor of a numpy
    array is a pageable host-to-device copy, which waits for the stream's queued work and would
    stop the stepping loop from running ahead of the GPU if it happened every step."""

    def __init__(self, ob_rms, device, dtype=torch.float32):
        self.mean = torch.as_tensor(ob_rms.mean, dtype=dtype, device=device)
        self.var = torch.as_tensor(ob_rms.var, dtype=dtype, device=device)


def normalize(obs, ob_rms):
    """VecNormalize in eval mode (enjoy_vr.py:85-88): obs are not used to update ob_rms."""
    m = torch.as_tensor(ob_rms.mean, dtype=obs.dtype, device=obs.device)
    v = torch.as_tensor(ob_rms.var, dtype=obs.dtype, device=obs.device)
    return torch.clamp((obs - m) / torch.sqrt(v + EPS), -CLIP_OBS, CLIP_OBS)


class ActorCritic(torch.nn.Module):
    """MLP actor-critic with a2c_ppo_acktr's act() signature (non-recurrent: hidden size 1)."""
    recurrent_hidden_state_size = 1

    def __init__(self, obs_dim, act_dim, hidden=64):
        super().__init__()
        self.obs_dim, self.act_dim, self.hidden = obs_dim, act_dim, hidden
        self.actor = torch.nn.Sequential(torch.nn.Linear(obs_dim, hidden), torch.nn.Tanh(), torch.nn.Linear(hidden, hidden), torch.nn.Tanh())
        self.critic = torch.nn.Sequential(torch.nn.Linear(obs_dim, hidden), torch.nn.Tanh(), torch.nn.Linear(hidden, hidden), torch.nn.Tanh(),
                                          torch.nn.Linear(hidden, 1))
        self.mu = torch.nn.Linear(hidden, act_dim)
        self.logstd = torch.nn.Parameter(torch.zeros(act_dim))

    def act(self, obs, rnn_hxs, masks, deterministic=False, generator=None):
        mean = self.mu(self.actor(obs))
        std = self.logstd.exp().expand_as(mean)
        if deterministic:
            action = mean
        else:
            action = mean + std * torch.randn(mean.shape, device=mean.device, generator=generator)
        logp = (-((action - mean) ** 2) / (2 * std * std) - std.log() - 0.5 * np.log(2 * np.pi)).sum(-1, keepdim=True)
        return self.critic(obs), action, logp, rnn_hxs


def save_policy(path, policy, ob_rms):
    torch.save({'state_dict': policy.state_dict(), 'obs_dim': policy.obs_dim, 'act_dim': policy.act_dim, 'hidden': policy.hidden,
                'ob_rms_mean': torch.as_tensor(ob_rms.mean), 'ob_rms_var': torch.as_tensor(ob_rms.var),
                'ob_rms_count': torch.tensor(ob_rms.count)}, path)


def load_policy(path, device='cpu'):
    """(actor_critic, ob_rms) -- the pair enjoy_vr.py:80 unpacks -- from a save_policy checkpoint
    (weights and arrays only: torch.load(weights_only=True) executes nothing from the file)."""
    ck = torch.load(path, map_location=device, weights_only=True)
    pol = ActorCritic(int(ck['obs_dim']), int(ck['act_dim']), int(ck['hidden'])).to(device)
    pol.load_state_dict(ck['state_dict'])
    rms = RunningMeanStd(ck['ob_rms_mean'].shape, ck['ob_rms_mean'].cpu().numpy(), ck['ob_rms_var'].cpu().numpy(), float(ck['ob_rms_count']))
    return pol, rms


def _graphed_policy(actor_critic, ob_rms, obs, hxs, masks, deterministic):
    """The policy forward captured once into a torch CUDA (HIP) graph with static obs / masks
    buffers; returns step(obs, masks) -> action (a fresh tensor per step), or None when capture is
    unavailable.  Sampling inside the graph draws from the default generator's Philox stream,
    whose offset the replays advance."""
    try:
        s_obs, s_masks = obs.clone(), masks.clone()
        side = torch.cuda.Stream(device=obs.device)
        side.wait_stream(torch.cuda.current_stream(obs.device))
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(3):                      # warm-up (library handles, workspaces) off the capture
                actor_critic.act(normalize(s_obs, ob_rms), hxs, s_masks, deterministic=deterministic)
        torch.cuda.current_stream(obs.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g), torch.no_grad():
            _, s_act, _, _ = actor_critic.act(normalize(s_obs, ob_rms), hxs, s_masks, deterministic=deterministic)
    except Exception:
        return None

    def step(o, m):
        s_obs.copy_(o)
        s_masks.copy_(m)
        g.replay()
        return s_act.clone()
    return step


def evaluate(env_id, actor_critic, ob_rms, n_envs=64, steps=200, deterministic=True, setup=None, device=0, seed=1001, graph=False):
    """Run one 200-step trial in each of n_envs envs (enjoy_vr.py:92-116 per env) and return
    per-env episode return, mean total_force_on_human and final task_success, plus the stepping
    loop's wall time (policy forward + env.step, synchronised at both ends) as loop_s.
    setup: dict(gender, participant, policy_name[, hipbone_to_mouth_height]) for env.setup.
    graph: replay the policy forward (normalisation + act) as one captured graph (eager if the
    capture fails).  Off by default: measured at 4096 envs it made the loop slower (7.09 vs 6.49
    ms per step, tools/pe_breakdown.py) -- the eager kernels are short, and the copies into the
    graph's static buffers add to the chain the env step waits on."""
    from .env import AVRTorchVecEnv
    env = AVRTorchVecEnv(env_id, n_envs, device=device, seed=seed, auto_reset=False)
    try:
        if setup:
            env.setup(**setup)
        dev = env.dev
        actor_critic = actor_critic.to(dev).eval()
        hxs = torch.zeros(n_envs, actor_critic.recurrent_hidden_state_size, device=dev)
        masks = torch.zeros(n_envs, 1, device=dev)
        obs = env.reset()[:, :env.obs_robot_len]
        ob_rms = DeviceRMS(ob_rms, dev, obs.dtype)
        ret = torch.zeros(n_envs, device=dev)
        force = torch.zeros(n_envs, device=dev)
        info = None
        policy = _graphed_policy(actor_critic, ob_rms, obs, hxs, masks, deterministic) if graph else None
        if policy is None:
            # one untimed forward (the mode: no draw from the torch RNG the loop samples from), so
            # that the BLAS handles and kernel code objects load outside the timed loop
            with torch.no_grad():
                actor_critic.act(normalize(obs, ob_rms), hxs, masks, deterministic=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            if policy is not None:
                action = policy(obs, masks)
            else:
                with torch.no_grad():
                    _, action, _, hxs = actor_critic.act(normalize(obs, ob_rms), hxs, masks, deterministic=deterministic)
            obs, rew, done, info = env.step(action)
            obs = obs[:, :env.obs_robot_len]
            masks = (~done).float()[:, None]
            ret += rew
            force += info['total_force_on_human']
        torch.cuda.synchronize(dev)
        loop_s = time.perf_counter() - t0
        return dict(returns=ret.cpu().numpy(), mean_force=(force / steps).cpu().numpy(),
                    task_success=info['task_success'].cpu().numpy() if info is not None else None, done=done.cpu().numpy(),
                    loop_s=loop_s, graph_captures=env.sim.graph_captures(), policy_graph=policy is not None)
    finally:
        env.close()
