"""Gym-style facade over libavr: the reference's FeedingJaco-v0 reset/step contract, batched.

Reference contract being mirrored:
  * ids registered in assistive_gym/__init__.py (FeedingJaco-v0 -> FeedingJacoEnv, TimeLimit 200);
  * reset() -> obs (25,), feeding.py:144-331 (scene randomisation, IK, 100 food-drop frames);
  * step(a) -> (obs (25,), reward, done, info) with info keys total_force_on_human,
    task_success, action_robot_len, action_human_len, obs_robot_len, obs_human_len
    (feeding.py:76); done at iteration >= 200 (TimeLimit).
  * observation/action spaces: Box(-1e9, 1e9, (25,)) and Box(-1, 1, (7,)), float32
    (env.py:34-35 with action_robot_len 7, obs_robot_len 25 for FeedingJaco).

AVRVecEnv steps all envs of one GPU in one kernel launch; AVREnv is the single-env view
(n_envs=1) that reads like `gym.make('FeedingJaco-v0')`.  Physics runs only on the GPU (libavr);
there is no CPU fallback here.
"""
import numpy as np

from . import _abi as ABI
from . import _lib
from . import reset as RS

MAX_EPISODE_STEPS = 200          # assistive_gym/__init__.py TimeLimit
SETTLE_FRAMES = 100              # feeding.py:318-320


class Box:
    """Minimal stand-in for gym.spaces.Box (gym is not a dependency of this package)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.low = np.full(shape, low, dtype)
        self.high = np.full(shape, high, dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return 'Box(%s, %s, %s, %s)' % (self.low.min(), self.high.max(), self.shape, self.dtype)


# id -> (task, robot, implemented): every id the reference registers (assistive_gym/__init__.py);
# this build implements the FeedingJaco-v0 hot path, the rest raise NotImplementedError.
REGISTRY = {
    'HumanTesting-v0':           ('human_testing', '-', False),
    'ScratchItchPR2-v0':         ('scratch_itch', 'pr2', False),
    'ScratchItchJaco-v0':        ('scratch_itch', 'jaco', False),
    'ScratchItchPR2Human-v0':    ('scratch_itch', 'pr2', False),
    'ScratchItchJacoHuman-v0':   ('scratch_itch', 'jaco', False),
    'ScratchItchPR2New-v0':      ('scratch_itch', 'pr2', False),
    'ScratchItchJacoNew-v0':     ('scratch_itch', 'jaco', False),
    'ScratchItchVRPR2-v0':       ('scratch_itch', 'pr2', False),
    'ScratchItchVRJaco-v0':      ('scratch_itch', 'jaco', False),
    'ScratchItchVRPR2Human-v0':  ('scratch_itch', 'pr2', False),
    'ScratchItchVRJacoHuman-v0': ('scratch_itch', 'jaco', False),
    'ScratchItchVRPR2New-v0':    ('scratch_itch', 'pr2', False),
    'ScratchItchVRJacoNew-v0':   ('scratch_itch', 'jaco', False),
    'BedBathingPR2-v0':          ('bed_bathing', 'pr2', False),
    'BedBathingJaco-v0':         ('bed_bathing', 'jaco', False),
    'BedBathingPR2Human-v0':     ('bed_bathing', 'pr2', False),
    'BedBathingJacoHuman-v0':    ('bed_bathing', 'jaco', False),
    'BedBathingPR2New-v0':       ('bed_bathing', 'pr2', False),
    'BedBathingJacoNew-v0':      ('bed_bathing', 'jaco', False),
    'BedBathingVRPR2-v0':        ('bed_bathing', 'pr2', False),
    'BedBathingVRJaco-v0':       ('bed_bathing', 'jaco', False),
    'BedBathingVRPR2Human-v0':   ('bed_bathing', 'pr2', False),
    'BedBathingVRJacoHuman-v0':  ('bed_bathing', 'jaco', False),
    'BedBathingVRPR2New-v0':     ('bed_bathing', 'pr2', False),
    'BedBathingVRJacoNew-v0':    ('bed_bathing', 'jaco', False),
    'DrinkingPR2-v0':            ('drinking', 'pr2', False),
    'DrinkingJaco-v0':           ('drinking', 'jaco', False),
    'DrinkingPR2Human-v0':       ('drinking', 'pr2', False),
    'DrinkingJacoHuman-v0':      ('drinking', 'jaco', False),
    'DrinkingPR2New-v0':         ('drinking', 'pr2', False),
    'DrinkingJacoNew-v0':        ('drinking', 'jaco', False),
    'DrinkingVRPR2-v0':          ('drinking', 'pr2', False),
    'DrinkingVRJaco-v0':         ('drinking', 'jaco', False),
    'DrinkingVRPR2Human-v0':     ('drinking', 'pr2', False),
    'DrinkingVRJacoHuman-v0':    ('drinking', 'jaco', False),
    'DrinkingVRPR2New-v0':       ('drinking', 'pr2', False),
    'DrinkingVRJacoNew-v0':      ('drinking', 'jaco', False),
    'FeedingPR2-v0':             ('feeding', 'pr2', False),
    'FeedingJaco-v0':            ('feeding', 'jaco', True),
    'FeedingPR2Human-v0':        ('feeding', 'pr2', False),
    'FeedingJacoHuman-v0':       ('feeding', 'jaco', False),
    'FeedingPR2New-v0':          ('feeding', 'pr2', False),
    'FeedingJacoNew-v0':         ('feeding', 'jaco', False),
    'FeedingVRPR2-v0':           ('feeding', 'pr2', False),
    'FeedingVRJaco-v0':          ('feeding', 'jaco', False),
    'FeedingVRPR2Human-v0':      ('feeding', 'pr2', False),
    'FeedingVRJacoHuman-v0':     ('feeding', 'jaco', False),
    'FeedingVRPR2New-v0':        ('feeding', 'pr2', False),
    'FeedingVRJacoNew-v0':       ('feeding', 'jaco', False),
}

_SCENES = {}


def _scene(task):
    if task not in _SCENES:
        A = ABI.load_scene()
        _SCENES[task] = (A, ABI.ModelDesc(A))
    return _SCENES[task]


class AVRVecEnv:
    """n_envs FeedingJaco-v0 environments on one GPU.

    env_offset: global id of env 0 (multi-GPU sharding: rank * n_envs); reset randomness and the
    synthetic action stream are keyed by the global env id, so results do not depend on how
    envs are split over GPUs.

    impairment: 'random' (FeedingJaco-v0's own setting, feeding.py:175: none / limits /
    weakness / tremor, one draw per episode), a fixed one of those four, or 'no_tremor'.
    """

    def __init__(self, env_id='FeedingJaco-v0', n_envs=1, device=0, seed=1001, env_offset=0, auto_reset=True,
                 impairment='random'):
        if env_id not in REGISTRY:
            raise KeyError('unknown env id %r' % env_id)
        task, robot, ok = REGISTRY[env_id]
        if not ok:
            raise NotImplementedError('%s: only the FeedingJaco-v0 hot path is built (SURVEY 8)' % env_id)
        self.env_id = env_id
        self.n = int(n_envs)
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.auto_reset = auto_reset
        self.impairment = impairment
        self.A, self.md = _scene(task)
        self.sim = _lib.Sim(self.md, self.n, device=device, seed=self.seed, env_offset=self.env_offset)
        self.observation_space = Box(-1e9, 1e9, (ABI.OBS_DIM,))
        self.action_space = Box(-1.0, 1.0, (ABI.ACT_DIM,))
        self.episode = np.zeros(self.n, np.int64)
        self._obs = np.zeros((self.n, ABI.OBS_DIM), np.float32)

    # ------------------------------------------------------------------ reset
    def _reset_rows(self, mask):
        idx = np.nonzero(mask)[0]
        S = np.zeros((self.n, ABI.STATE_WORDS), np.float32)
        if len(idx):
            Si, _ = RS.batch_reset_states_fast(self.A, self.md, self.seed, [self.env_offset + int(i) for i in idx],
                                               impairment=self.impairment, episodes=self.episode[idx])
            S[idx] = Si
        self.sim.reset(mask.astype(np.uint8), S, SETTLE_FRAMES, self._obs)

    def reset(self, mask=None):
        """Reset all envs (mask None) or the masked ones; returns obs (n_envs, 25) float32."""
        mask = np.ones(self.n, bool) if mask is None else np.asarray(mask, bool)
        self._reset_rows(mask)
        return self._obs.copy()

    # ------------------------------------------------------------------ step
    def step(self, actions):
        """actions (n_envs, 7) -> obs, reward (n_envs,), done (n_envs,) bool, info dict of arrays.

        With auto_reset, finished envs are reset (next episode stream) and their final
        observation is returned in info['terminal_observation'] (vectorised-gym convention)."""
        a = np.ascontiguousarray(actions, np.float32).reshape(self.n, ABI.ACT_DIM)
        obs, rew, done, inf = self.sim.step(a)
        info = {
            'total_force_on_human': inf[:, 0].copy(),
            'task_success': inf[:, 1].astype(np.int64),
            'action_robot_len': ABI.ACT_DIM, 'action_human_len': 0,
            'obs_robot_len': ABI.OBS_DIM, 'obs_human_len': 0,
            'flags': self.flags(),
        }
        self._obs[:] = obs
        if self.auto_reset and done.any():
            info['terminal_observation'] = obs.copy()
            self.episode[done] += 1
            self._reset_rows(done)
            obs = self._obs.copy()
        return obs, rew, done, info

    def flags(self):
        """Per-env health flags (bit0 NaN/failed factorisation, bit1 contact-cache overflow, ...)."""
        St = self.sim.get_state()
        return St[:, ABI.S_TASK + ABI.T_FLAGS].astype(np.int64)

    def get_state(self):
        return self.sim.get_state()

    def set_state(self, S):
        self.sim.set_state(S)

    def close(self):
        self.sim.close()


class AVREnv:
    """Single-env view with the reference's gym.Env signatures."""

    def __init__(self, env_id='FeedingJaco-v0', device=0, seed=1001, impairment='random'):
        self.v = AVRVecEnv(env_id, 1, device=device, seed=seed, auto_reset=False, impairment=impairment)
        self.observation_space = self.v.observation_space
        self.action_space = self.v.action_space

    def seed(self, seed=1001):
        self.v.seed = int(seed)
        return [seed]

    def reset(self):
        return self.v.reset()[0].astype(np.float64)

    def step(self, action):
        obs, rew, done, info = self.v.step(np.asarray(action, np.float32)[None])
        i = {k: (v[0] if isinstance(v, np.ndarray) else v) for k, v in info.items()}
        i['task_success'] = int(i['task_success'])
        i['total_force_on_human'] = float(i['total_force_on_human'])
        return obs[0].astype(np.float64), float(rew[0]), bool(done[0]), i

    def close(self):
        self.v.close()


def make(env_id, **kw):
    """gym.make replacement: AVREnv for one env, AVRVecEnv when n_envs is given."""
    if 'n_envs' in kw:
        return AVRVecEnv(env_id, **kw)
    return AVREnv(env_id, **kw)
