"""State snapshots and episode record / replay on the batched backend -- the reference's
`.bullet` + setup.pkl + actions.pkl flow:

  * p.saveBullet / p.restoreState of the whole world (env.py:300-301 per frame while a VR
    participant acts; feeding.py:322-330 frame 0) -> save_state / load_state: the device state
    block of every env (include/avr_model.h layout) with its task, layout size and ABI version,
    in an .npz that loads with numpy's pickle-free loader;
  * setup.pkl [robot_type, gender, hipbone_to_mouth_height] and actions.pkl (feeding.py:50-54,
    153-157, 328-329) -> setup.json + actions.npy of a recording directory, plus states.npy: the
    state after the reset (the reference's frame_0.bullet) and after every env step (the
    reference saves each of the 5 frames of a step; the batched step fuses them, so the snapshot
    granularity here is the env step);
  * env.replay_setup(dir) + step() restoring the recorded frames (env.py:74-78, feeding.py:31-39)
    -> ReplayEnv: reset restores frame 0; every step re-simulates the recorded action from the
    recorded state and checks the result against the next recorded state (bit-identical on the
    same build, since the step is deterministic), so obs / reward / info come from the backend
    exactly as a live episode's;
  * replay_vr_savemeta.py (observations, rewards, actions, forces, task success of every
    recording) -> savemeta().
"""
import glob
import json
import os

import numpy as np

from . import _abi as ABI

FORMAT = 'avr-state-1'


def _sim(x):
    return x.sim if hasattr(x, 'sim') else x


def save_state(path, env):
    """Snapshot every env's state block (p.saveBullet counterpart)."""
    sim = _sim(env)
    S = sim.get_state()
    np.savez(path, format=np.array(FORMAT), task=np.int32(sim.md.task), state_words=np.int32(S.shape[1]),
             abi=np.int32(ABI.ABI_VERSION), state=S)


def load_state(path, env):
    """Restore a snapshot (p.restoreState counterpart); the task and layout must match."""
    sim = _sim(env)
    with np.load(path, allow_pickle=False) as z:
        if str(z['format']) != FORMAT:
            raise ValueError('%s: not an %s snapshot' % (path, FORMAT))
        if int(z['task']) != sim.md.task or int(z['state_words']) != sim.words or int(z['abi']) != ABI.ABI_VERSION:
            raise ValueError('%s: snapshot of task %d / %d words / ABI %d; this handle is task %d / %d words / ABI %d'
                             % (path, int(z['task']), int(z['state_words']), int(z['abi']), sim.md.task, sim.words, ABI.ABI_VERSION))
        S = z['state']
    if S.shape[0] != sim.n:
        raise ValueError('%s: %d envs in the snapshot, %d in the handle' % (path, S.shape[0], sim.n))
    if hasattr(env, 'set_state'):
        env.set_state(S)
    else:
        sim.set_state(S)


class Recorder:
    """Records one episode of an AVRVecEnv (auto_reset off) into a directory: reset(), then
    step(action) as usual; close() writes setup.json, actions.npy and states.npy."""

    def __init__(self, env, directory, robot_type=None):
        self.env, self.dir = env, directory
        os.makedirs(directory, exist_ok=True)
        self.robot_type = robot_type or ('pr2' if 'PR2' in env.env_id else 'jaco')
        self.actions, self.states = [], []

    def reset(self):
        obs = self.env.reset()
        self.states = [self.env.get_state()]
        self.actions = []
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action, np.float32).reshape(self.env.n, -1)
        out = self.env.step(a)
        self.actions.append(a.copy())
        self.states.append(self.env.get_state())
        return out

    def close(self):
        S = self.states[0]
        L = self.env.L
        genders = ['male' if g == 0 else 'female' for g in S[:, L.S_TASK + L.T_GENDER].astype(int)]
        setup = dict(env_id=self.env.env_id, robot_type=self.robot_type, gender=genders,
                     hipbone_to_mouth_height=[0.6 if g == 'male' else 0.54 for g in genders],
                     seed=self.env.seed, env_offset=self.env.env_offset, n_envs=self.env.n, task=int(self.env.task),
                     state_words=int(S.shape[1]), abi=int(ABI.ABI_VERSION), format=FORMAT, snapshot_every='env step')
        with open(os.path.join(self.dir, 'setup.json'), 'w') as f:
            json.dump(setup, f, indent=1)
        np.save(os.path.join(self.dir, 'actions.npy'), np.stack(self.actions) if self.actions else np.zeros((0, self.env.n, self.env.L.ACT_DIM), np.float32))
        np.save(os.path.join(self.dir, 'states.npy'), np.stack(self.states))


class ReplayEnv:
    """replay_setup(dir) + reset/step of a recording (see the module docstring).  The action passed
    to step() is ignored, as in the reference's replay (feeding.py:38: action = action_list[i])."""

    def __init__(self, directory, device=0, verify=True):
        from . import env as EV
        with open(os.path.join(directory, 'setup.json')) as f:
            self.setup_info = json.load(f)
        if self.setup_info.get('format') != FORMAT or self.setup_info.get('abi') != ABI.ABI_VERSION:
            raise ValueError('%s: recording format %s / ABI %s' % (directory, self.setup_info.get('format'), self.setup_info.get('abi')))
        self.action_list = np.load(os.path.join(directory, 'actions.npy'), allow_pickle=False)
        self.states = np.load(os.path.join(directory, 'states.npy'), mmap_mode='r', allow_pickle=False)
        self.env = EV.AVRVecEnv(self.setup_info['env_id'], int(self.setup_info['n_envs']), device=device, seed=int(self.setup_info['seed']),
                                env_offset=int(self.setup_info['env_offset']), auto_reset=False, prefetch=False)
        self.verify = verify
        self.iteration = 0
        self.mismatch = []

    def reset(self):
        self.iteration = 0
        self.env.set_state(np.asarray(self.states[0]))
        return self.env.observe()

    def step(self, action=None):
        t = self.iteration
        obs, rew, done, info = self.env.step(self.action_list[t])
        self.iteration += 1
        if self.verify:
            S = self.env.get_state()
            want = np.asarray(self.states[t + 1])
            if not np.array_equal(S, want):
                self.mismatch.append((t, float(np.abs(S - want).max())))
        done = np.full(self.env.n, self.iteration >= len(self.action_list))   # (feeding.py:73: replay ends at the last action)
        return obs, rew, done, info

    def close(self):
        self.env.close()


def savemeta(pattern, out=None, device=0):
    """replay_vr_savemeta.py over every recording matching `pattern`: observations, rewards,
    actions, total_force_on_human and final task_success per recording (arrays in an .npz when
    `out` is given)."""
    res = {}
    for d in sorted(glob.glob(pattern)):
        if not os.path.exists(os.path.join(d, 'setup.json')):
            continue
        r = ReplayEnv(d, device=device)
        obs = [r.reset()]
        rews, forces, succ = [], [], None
        done = np.zeros(r.env.n, bool)
        while not done.all():
            o, rw, done, info = r.step()
            obs.append(o); rews.append(rw); forces.append(info['total_force_on_human']); succ = info['task_success']
        res[d] = dict(observations=np.stack(obs), rewards=np.stack(rews), actions=r.action_list, forces=np.stack(forces),
                      task_success=succ, replay_mismatch=list(r.mismatch))
        r.close()
    if out:
        flat = {}
        for i, (d, v) in enumerate(res.items()):
            for k in ('observations', 'rewards', 'actions', 'forces', 'task_success'):
                flat['%d_%s' % (i, k)] = v[k]
        flat['dirs'] = np.array(list(res))
        np.savez(out, **flat)
    return res
