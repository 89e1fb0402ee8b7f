"""Gym-style facade over libavr: the reference's reset/step contract, batched.

Reference contract being mirrored:
  * ids registered in assistive_gym/__init__.py (FeedingJaco-v0 -> FeedingJacoEnv,
    ScratchItchPR2-v0 -> ScratchItchPR2Env; TimeLimit 200);
  * reset() -> obs: FeedingJaco (25,), feeding.py:144-331 (scene randomisation, IK, 100 food-drop
    frames); ScratchItchPR2 (30,), scratch_itch.py:130-273 (base-pose search + IK, no settle);
  * step(a) -> (obs, reward, done, info) with info keys total_force_on_human, task_success,
    action_robot_len, action_human_len, obs_robot_len, obs_human_len (feeding.py:76,
    scratch_itch.py:78); done at iteration >= 200 (TimeLimit).
  * observation/action spaces: Box(-1e9, 1e9, (obs,)) and Box(-1, 1, (7,)), float32 (env.py:34-35).

AVRVecEnv steps all envs of one GPU in one launch sequence (host arrays in/out); AVRTorchVecEnv
is the same with device tensors (no host copies per step); AVREnv is the single-env view
(n_envs=1) that reads like `gym.make('FeedingJaco-v0')`.  Physics runs only on the GPU (libavr);
there is no CPU fallback here.

Episode rollover (auto_reset): FeedingJaco resets run the IK on the device (avr_reset_ik) from
the host's reset draws (reset.reset_inputs), which a background thread prepares for the next
episode while the current one steps; ScratchItch resets run the host base-pose search + IK
(reset_scratch.batch_reset_states), then avr_reset.
"""
import sys
import threading
import time

import numpy as np

from . import _abi as ABI
from . import _lib
from . import reset as RS

MAX_EPISODE_STEPS = 200          # assistive_gym/__init__.py TimeLimit
# settle frames after the reset state is in place: feeding.py:318-320; scratch_itch.py has none;
# bed_bathing.py's 100-frame arm settle (:288-289) comes before the robot is placed (reset_bedbath)
SETTLE_FRAMES = {ABI.TASK_FEEDING: 100, ABI.TASK_SCRATCH: 0, ABI.TASK_BEDBATH: 0, ABI.TASK_DRESSING: 0}


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
# this build implements FeedingJaco-v0, ScratchItchPR2-v0 and BedBathingPR2-v0, the
# rest raise NotImplementedError.
REGISTRY = {
    'HumanTesting-v0':           ('human_testing', '-', False),
    'ScratchItchPR2-v0':         ('scratch_itch', 'pr2', True),
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
    'BedBathingPR2-v0':          ('bed_bathing', 'pr2', True),
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
    # BASELINE.json configs[4]; not registered by the reference (it has no dressing task, SURVEY
    # 0.5): a build-defined task on the reference's dressing hooks (include/avr_dressing.h)
    'DressingJaco-v0':           ('dressing', 'jaco', True),
}

_SCENES = {}
_TASK_OF = {'feeding': ABI.TASK_FEEDING, 'scratch_itch': ABI.TASK_SCRATCH, 'bed_bathing': ABI.TASK_BEDBATH, 'dressing': ABI.TASK_DRESSING}


def _scene(task, heights=None):
    """(arrays, ModelDesc) of a task's scene with the human at per-gender hipbone_to_mouth_height
    `heights` (None: the defaults, the committed npz; otherwise rebuilt by the model compiler
    from its asset cache, human_creation.py:60-63,75)."""
    from . import model_compiler as MC
    H = MC.human_heights(heights)
    key = (task,) + tuple(H[g] for g in ('male', 'female'))
    if key not in _SCENES:
        if task == 'dressing':
            if not MC.default_heights(H):
                raise NotImplementedError('DressingJaco-v0: only the default human proportions are built')
            from . import reset_dressing as RD
            A = RD.dressing_scene()
        elif MC.default_heights(H):
            A = ABI.load_scene(_TASK_OF[task])
        else:
            A = MC.scene_arrays(ABI.SCENES[_TASK_OF[task]], H)
        _SCENES[key] = (A, ABI.ModelDesc(A))
    return _SCENES[key]


class _Prefetch:
    """Reset draws of the next episode of a set of envs, prepared on a background thread while
    the stepping thread keeps the GPU fed.  The stepping thread takes and drops the GIL around
    every ctypes / torch call; at the default 5 ms switch interval a GIL-bound worker would delay
    each re-acquisition by up to 5 ms and starve the launches, so the interval is lowered to
    0.1 ms while the worker runs."""

    def __init__(self, fn):
        self.fn = fn
        self.key = None
        self.result = None
        self.thread = None

    def start(self, key, *args):
        self.wait()
        self.key, self.result = key, None

        def run():
            old = sys.getswitchinterval()
            sys.setswitchinterval(1e-4)
            try:
                self.result = self.fn(*args)
            finally:
                sys.setswitchinterval(old)
        self.thread = threading.Thread(target=run, daemon=True)
        self.thread.start()

    def wait(self):
        if self.thread is not None:
            self.thread.join()
            self.thread = None

    def take(self, key):
        self.wait()
        if self.key == key and self.result is not None:
            r, self.key, self.result = self.result, None, None
            return r
        return None


class AVRVecEnv:
    """n_envs environments of one task on one GPU; host arrays in and out.

    env_offset: global id of env 0 (multi-GPU sharding: rank * n_envs); reset randomness and the
    synthetic action stream are keyed by the global env id, so results do not depend on how
    envs are split over GPUs.

    impairment: 'random' (the tasks' own setting, feeding.py:175 / scratch_itch.py:178: none /
    limits / weakness / tremor, one draw per episode), a fixed one of those four, or 'no_tremor'.
    reset_ik: 'device' (default: FeedingJaco's and DressingJaco's IK through avr_reset_ik, the PR2
    tasks' base-pose search through avr_base_search) or 'host' (the fp64 host restatements, then
    avr_reset).
    reset_stream: FeedingJaco's reset draws, 'philox' (counter-based, vectorised; default) or
    'numpy' (the per-env Generator stream of the bench's reset pools and the golden fixtures).
    human_heights: the human's proportions, {gender: hipbone_to_mouth_height} (create_human's
    hmhs = height / 0.6 male, / 0.54 female, human_creation.py:60-63: capsule lengths and joint
    offsets scale by it, BedBathing's wipe targets too, bed_bathing.py:359-370); a gender not
    named keeps its default.  One set per handle: the reference builds its human at the height
    the env holds (a replay's setup.pkl, feeding.py:153-156; setup(), feeding.py:20-28).
    """

    def __init__(self, env_id='FeedingJaco-v0', n_envs=1, device=0, seed=1001, env_offset=0, auto_reset=True,
                 impairment='random', reset_ik='device', prefetch=True, scratch_attempts=100, scratch_iters=200,
                 reset_stream='philox', human_heights=None):
        if env_id not in REGISTRY:
            raise KeyError('unknown env id %r' % env_id)
        task, robot, ok = REGISTRY[env_id]
        if not ok:
            raise NotImplementedError('%s: only FeedingJaco-v0, ScratchItchPR2-v0, BedBathingPR2-v0 and DressingJaco-v0 are built (SURVEY 8)' % env_id)
        self.env_id = env_id
        self.n = int(n_envs)
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self.auto_reset = auto_reset
        self.impairment = impairment
        self.A, self.md = _scene(task, human_heights)
        from . import model_compiler as MC
        self.human_heights = MC.human_heights(human_heights)
        self.task = self.md.task
        self.L = self.md.layout
        self.device_ik = self.task == ABI.TASK_FEEDING and reset_ik == 'device'
        self.device_dress_ik = self.task == ABI.TASK_DRESSING and reset_ik == 'device'
        self.device_search = self.task in (ABI.TASK_SCRATCH, ABI.TASK_BEDBATH) and reset_ik == 'device'
        self.scratch_attempts, self.scratch_iters = scratch_attempts, scratch_iters
        self.reset_stream = reset_stream
        self.device = device
        self.sim = _lib.Sim(self.md, self.n, device=device, seed=self.seed, env_offset=self.env_offset)
        self.observation_space = Box(-1e9, 1e9, (self.L.OBS_DIM,))
        self.action_space = Box(-1.0, 1.0, (self.L.ACT_DIM,))
        self.obs_robot_len, self.obs_human_len = self.L.OBS_DIM, 0
        self.action_robot_len, self.action_human_len = self.L.ACT_DIM, 0
        self.genders = None                # setup(): fixed gender for every reset
        self.participant, self.policy_name = -1, ''
        self.hipbone_to_mouth_height = None   # setup(): kept, not modelled (see setup)
        self.episode = np.zeros(self.n, np.int64)
        # host mirror of the per-env iteration counters: the kernels' done is exactly
        # T_ITER >= max_steps (TimeLimit), so rollovers are known without reading the device
        self.iteration = np.zeros(self.n, np.int64)
        self.max_steps = int(self.md.params['max_episode_steps'])
        self._obs = np.zeros((self.n, self.L.OBS_DIM), np.float32)
        self._keepout = RS.keepout_box(self.A) if self.task == ABI.TASK_FEEDING else None
        if self.task == ABI.TASK_BEDBATH:          # the reset's arm settle, once per gender (device)
            from . import reset_bedbath as RBB
            RBB.settled_arms(self.A, self.md, device)
        self._prefetch = _Prefetch(self._inputs) if (prefetch and (self.device_ik or self.device_search or self.task == ABI.TASK_DRESSING)) else None
        self.last_ik_ok = None
        self.reset_timing = None

    # ------------------------------------------------------------------ setup hook
    def setup(self, gender, participant, policy_name, hipbone_to_mouth_height=None):
        """FeedingEnv.setup / ScratchItchEnv.setup (feeding.py:20-28): the evaluation harness fixes
        the participant's gender (every later reset uses it) and names the policy.

        hipbone_to_mouth_height is accepted and kept (`self.hipbone_to_mouth_height`) but, as in
        the reference's non-VR envs, does not shape the human: their reset overwrites it with the
        gender's default before building the world (feeding.py:173-174, scratch_itch.py:161,
        bed_bathing.py:187), so enjoy_vr.py's `env.setup(gender, participant, policy, 0.54)`
        (enjoy_vr.py:50,63) runs unchanged for both genders."""
        if gender not in ('male', 'female'):
            raise ValueError('gender must be male or female')
        self.hipbone_to_mouth_height = None if hipbone_to_mouth_height is None else float(hipbone_to_mouth_height)
        self.genders = gender
        self.participant, self.policy_name = int(participant), str(policy_name)
        if self._prefetch:
            self._prefetch.wait()
            self._prefetch.key = None      # draws prepared before setup() are for the old genders

    def _genders(self, idx):
        return None if self.genders is None else [self.genders] * len(idx)

    # ------------------------------------------------------------------ reset
    def _inputs(self, idx, episodes):
        """The host part of the masked envs' resets (everything before the device's part)."""
        ids = [self.env_offset + int(i) for i in idx]
        if self.task == ABI.TASK_DRESSING:
            from . import reset_dressing as RD
            P = RD.prepare_reset(self.A, self.md, self.seed, ids, genders=self._genders(idx), episodes=list(episodes))
            return P if self.device_dress_ik else RD.finish_reset(self.A, self.md, P)
        if self.task == ABI.TASK_BEDBATH:
            from . import reset_bedbath as RBB
            return RBB.prepare_reset(self.A, self.md, self.seed, ids, genders=self._genders(idx), episodes=list(episodes),
                                     attempts=self.scratch_attempts, device=self.device)
        if self.task == ABI.TASK_SCRATCH:
            from . import reset_scratch as RSS
            return RSS.prepare_reset(self.A, self.md, self.seed, ids, genders=self._genders(idx), impairment=self.impairment,
                                     episodes=list(episodes), attempts=self.scratch_attempts)
        out = RS.reset_inputs(self.A, self.md, self.seed, ids, genders=self._genders(idx),
                              impairment=self.impairment, episodes=list(episodes), stream=self.reset_stream)
        # + the self-contact screening's re-drawn target orientations (ik_random_restarts' step_sim)
        return out + (RS.ik_alt_orients(self.seed, ids, list(episodes), out[2].shape[1], self.reset_stream),)

    def _reset_rows(self, mask):
        idx = np.nonzero(mask)[0]
        if not len(idx):
            return
        self.iteration[idx] = 0
        eps = self.episode[idx].copy()
        S = np.zeros((self.n, self.L.STATE_WORDS), np.float32)
        frames = SETTLE_FRAMES[self.task]
        if self.device_ik:
            t0 = time.perf_counter()
            key = (tuple(idx.tolist()), tuple(eps.tolist()))
            got = self._prefetch.take(key) if self._prefetch else None
            Si, t7, init, _, _, alt = got if got is not None else self._inputs(idx, eps)
            t1 = time.perf_counter()
            S[idx] = Si
            T = np.zeros((self.n, 7), np.float32)
            T[:, 6] = 1.0
            T[idx] = t7
            I = np.zeros((self.n,) + init.shape[1:], np.float32)
            I[idx] = init
            Al = np.zeros((self.n, init.shape[1], 4), np.float32)
            Al[..., 3] = 1.0
            Al[idx] = alt
            t2 = time.perf_counter()
            _, ok = self.sim.reset_ik(mask.astype(np.uint8), S, T, I, keepout8=self._keepout, frames=frames, obs=self._obs, alt=Al)
            self.last_ik_ok = ok
            self.reset_timing = dict(inputs_s=t1 - t0, prefetched=got is not None, pack_s=t2 - t1, device_s=time.perf_counter() - t2)
            if self._prefetch:           # speculate: the same envs end their next episode together
                self._prefetch.start((key[0], tuple((eps + 1).tolist())), idx, eps + 1)
            return
        ids = [self.env_offset + int(i) for i in idx]
        if self.task == ABI.TASK_DRESSING:
            # host draws (prefetched like the others' host parts), then the IK on the device
            # (avr_reset_ik) or, with reset_ik='host', the host IK and avr_reset
            t0 = time.perf_counter()
            key = (tuple(idx.tolist()), tuple(eps.tolist()))
            got = self._prefetch.take(key) if self._prefetch else None
            P = got if got is not None else self._inputs(idx, eps)
            t1 = time.perf_counter()
            if self._prefetch:
                self._prefetch.start((key[0], tuple((eps + 1).tolist())), idx, eps + 1)
            if self.device_dress_ik:
                Si, tpos, tquat, init, _ = P
                S[idx] = Si
                T = np.zeros((self.n, 7), np.float32)
                T[:, 6] = 1.0
                T[idx, :3], T[idx, 3:] = tpos, tquat
                I = np.zeros((self.n,) + init.shape[1:], np.float32)
                I[idx] = init
                _, ok = self.sim.reset_ik(mask.astype(np.uint8), S, T, I, iters=150, tol=0.01, frames=0, obs=self._obs)
                self.last_ik_ok = ok
            else:
                S[idx] = P[0]
                self.sim.reset(mask.astype(np.uint8), S, 0, self._obs)
            self.reset_timing = dict(host_s=t1 - t0, prefetched=got is not None, device_s=time.perf_counter() - t1)
            return
        if self.task in (ABI.TASK_SCRATCH, ABI.TASK_BEDBATH):
            # host part (prefetched on a background thread during the previous episode when the
            # same envs finish together), then the base-pose search on the device
            from . import reset_bedbath as RBB, reset_scratch as RSS
            t0 = time.perf_counter()
            key = (tuple(idx.tolist()), tuple(eps.tolist()))
            got = self._prefetch.take(key) if self._prefetch else None
            P = got if got is not None else self._inputs(idx, eps)
            t1 = time.perf_counter()
            fin = RBB.finish_reset if self.task == ABI.TASK_BEDBATH else RSS.finish_reset
            Si, _ = fin(self.A, self.md, P, self.scratch_iters, self.sim if self.device_search else None)
            t2 = time.perf_counter()
            if self._prefetch:
                self._prefetch.start((key[0], tuple((eps + 1).tolist())), idx, eps + 1)
            S[idx] = Si
            self.sim.reset(mask.astype(np.uint8), S, frames, self._obs)
            self.reset_timing = dict(inputs_s=t1 - t0, prefetched=got is not None, search_s=t2 - t1, device_s=time.perf_counter() - t2)
            return
        else:
            Si, _ = RS.batch_reset_states_fast(self.A, self.md, self.seed, ids, genders=self._genders(idx), impairment=self.impairment, episodes=eps,
                                               stream=self.reset_stream, self_contact=self.sim.robot_self_contact)
        S[idx] = Si
        self.sim.reset(mask.astype(np.uint8), S, frames, self._obs)

    def reset(self, mask=None):
        """Reset all envs (mask None) or the masked ones; returns obs (n_envs, obs_dim) float32."""
        mask = np.ones(self.n, bool) if mask is None else np.asarray(mask, bool)
        self._reset_rows(mask)
        return self._obs.copy()

    # ------------------------------------------------------------------ step
    def _info(self, inf):
        return {
            'total_force_on_human': inf[:, 0].copy(),
            'task_success': inf[:, 1].astype(np.int64),
            'action_robot_len': self.L.ACT_DIM, 'action_human_len': 0,
            'obs_robot_len': self.L.OBS_DIM, 'obs_human_len': 0,
        }

    def step(self, actions):
        """actions (n_envs, 7) -> obs, reward (n_envs,), done (n_envs,) bool, info dict of arrays.

        With auto_reset, finished envs are reset (next episode stream) and their final
        observation is returned in info['terminal_observation'] (vectorised-gym convention)."""
        a = np.ascontiguousarray(actions, np.float32).reshape(self.n, self.L.ACT_DIM)
        obs, rew, done, inf = self.sim.step(a)
        self.iteration += 1
        info = self._info(inf)
        self._obs[:] = obs
        if self.auto_reset and done.any():
            info['terminal_observation'] = obs.copy()
            self.episode[done] += 1
            self._reset_rows(done)
            obs = self._obs.copy()
        return obs, rew, done, info

    def observe(self):
        """Observation of the current state without stepping (what _get_obs returns right after
        p.restoreState, feeding.py:322-325)."""
        self._obs[:] = self.sim.settle(0)
        return self._obs.copy()

    def flags(self):
        """Per-env health flags (include/avr.h avr_get_flags), without copying the state.  Bits 0-4
        (_lib.FLAGS_FAULT_MASK) are faults, 0 there = healthy; bit 5 is informational (the env ran
        under the EPA budget, its state is finite)."""
        return self.sim.get_flags().astype(np.int64)

    def get_state(self):
        return self.sim.get_state()

    def set_state(self, S):
        self.sim.set_state(S)
        self.iteration[:] = np.asarray(S)[:, self.L.S_TASK + self.L.T_ITER].astype(np.int64)

    def close(self):
        if self._prefetch:
            self._prefetch.wait()
        self.sim.close()


class AVRTorchVecEnv(AVRVecEnv):
    """AVRVecEnv with torch device tensors: step(actions (n, 7) cuda float32) -> obs, reward, done,
    info as cuda tensors, written by the kernels directly (avr_step_device).  No per-step host
    traffic or synchronisation: whether a rollover is due follows from the host mirror of the
    iteration counters (done == T_ITER >= max_steps in the kernels), so launches of consecutive
    steps queue ahead of the GPU; a rollover step synchronises for the reset."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        import torch
        self.torch = torch
        self.dev = torch.device('cuda', int(self.device))
        self.ext = torch.cuda.ExternalStream(self.sim.stream(), device=self.dev)
        n, L = self.n, self.L
        self.t_obs = torch.zeros(n, L.OBS_DIM, device=self.dev)
        self.t_rew = torch.zeros(n, device=self.dev)
        self.t_done = torch.zeros(n, dtype=torch.uint8, device=self.dev)
        self.t_info = torch.zeros(n, ABI.INFO_DIM, device=self.dev)

    def reset(self, mask=None):
        obs = super().reset(mask)
        self.t_obs.copy_(self.torch.from_numpy(obs))
        return self.t_obs.clone()

    def step(self, actions):
        torch = self.torch
        a = actions.to(self.dev, torch.float32).contiguous()
        assert a.shape == (self.n, self.L.ACT_DIM)
        self.ext.wait_stream(torch.cuda.current_stream(self.dev))
        # (the kernels read `a` on the sim stream; torch's stream waits for that stream below, so the
        # caching allocator cannot hand `a`'s memory to later work before the step has read it)
        self.sim.step_device(a.data_ptr(), self.t_obs.data_ptr(), self.t_rew.data_ptr(), self.t_done.data_ptr(), self.t_info.data_ptr())
        torch.cuda.current_stream(self.dev).wait_stream(self.ext)
        self.iteration += 1
        obs, rew, done = self.t_obs.clone(), self.t_rew.clone(), self.t_done.bool()
        info = {'total_force_on_human': self.t_info[:, 0].clone(), 'task_success': self.t_info[:, 1].to(torch.int64),
                'action_robot_len': self.L.ACT_DIM, 'action_human_len': 0, 'obs_robot_len': self.L.OBS_DIM, 'obs_human_len': 0}
        if self.auto_reset:
            dh = self.iteration >= self.max_steps
            if dh.any():
                torch.cuda.current_stream(self.dev).synchronize()
                info['terminal_observation'] = obs
                self.episode[dh] += 1
                self._reset_rows(dh)
                m = torch.from_numpy(dh).to(self.dev)
                obs = torch.where(m[:, None], torch.from_numpy(self._obs).to(self.dev), obs)
        return obs, rew, done, info

    def close(self):
        self.torch.cuda.synchronize(self.dev)
        super().close()


class AVREnv:
    """Single-env view with the reference's gym.Env signatures."""

    def __init__(self, env_id='FeedingJaco-v0', device=0, seed=1001, impairment='random'):
        self.v = AVRVecEnv(env_id, 1, device=device, seed=seed, auto_reset=False, impairment=impairment, prefetch=False)
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
    """gym.make replacement: AVREnv for one env, AVRVecEnv when n_envs is given (AVRTorchVecEnv
    with torch=True)."""
    if kw.pop('torch', False):
        return AVRTorchVecEnv(env_id, **kw)
    if 'n_envs' in kw:
        return AVRVecEnv(env_id, **kw)
    return AVREnv(env_id, **kw)
