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

Reference-format recordings (a participant directory the reference wrote: setup.pkl,
actions.pkl, frame_%d.bullet; feeding.py:50-54,146-157,322-330, scratch_itch.py:136-144,268-272,
bed_bathing.py:163-170,352-356) are read by load_reference_pickle -- a restricted unpickler that
executes nothing from the file: it admits lists, tuples, dicts, strings, numbers and numpy arrays
/ scalars of numeric dtypes, rebuilt by this module's own constructors from the raw bytes; any
other global refuses the file -- and replayed by ReferenceReplayEnv (replay_setup + reset + step,
env.py:74-78, feeding.py:31-39): the recorded gender is set up, the episode starts from this
build's reset for it, and the recorded actions are re-simulated.  The frame_%d.bullet states are
Bullet serializer output and cannot be restored here, so the replayed trajectory is the
re-simulation of the participant's actions, not the participant's recorded frames.
savemeta_reference() is replay_vr_savemeta.py over such directories.
"""
import glob
import json
import math
import os
import pickle

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


# ---------------------------------------------------------------- reference-format recordings

_NUMERIC_KINDS = 'biufc'


class _DType:
    """numpy.dtype(name, align, copy) as pickled; only numeric dtypes are admitted."""

    def __init__(self, name, align=False, copy=True):
        if not isinstance(name, str):
            raise pickle.UnpicklingError('dtype spec %r' % (name,))
        dt = np.dtype(name)
        if dt.kind not in _NUMERIC_KINDS or dt.fields is not None or dt.subdtype is not None:
            raise pickle.UnpicklingError('dtype %r is not a plain numeric dtype' % (name,))
        self.dtype = dt

    def __setstate__(self, state):
        # (version, byteorder, subdescr, names, fields, elsize, alignment, flags)
        if not isinstance(state, tuple) or len(state) < 5 or state[1] not in ('<', '>', '=', '|'):
            raise pickle.UnpicklingError('dtype state %r' % (state,))
        if state[2] is not None or state[3] is not None or state[4] is not None:
            raise pickle.UnpicklingError('structured dtype')
        if state[1] in '<>':
            self.dtype = self.dtype.newbyteorder(state[1])


def _as_dtype(d):
    if isinstance(d, _DType):
        return d.dtype
    raise pickle.UnpicklingError('expected a dtype, got %r' % type(d))


def _shape(shape):
    """An array shape as pickled: a tuple of non-negative Python ints (the element count is then
    formed with Python ints, so a hostile shape cannot wrap around a fixed-width product)."""
    if not isinstance(shape, (tuple, list)) or len(shape) > 32:
        raise pickle.UnpicklingError('ndarray shape %r' % (shape,))
    if not all(isinstance(s, int) and not isinstance(s, bool) and s >= 0 for s in shape):
        raise pickle.UnpicklingError('ndarray shape %r' % (shape,))
    return tuple(shape)


class _ArrayBuilder:
    """numpy.core.multiarray._reconstruct(ndarray, (0,), b'b') + BUILD(state) as pickled
    (protocols 0-4): the state carries shape, dtype, order and the raw bytes."""

    def __init__(self, cls, shape, code):
        if cls is not _NDARRAY:
            raise pickle.UnpicklingError('only numpy.ndarray is reconstructed')
        self.array = None

    def __setstate__(self, state):
        if not isinstance(state, tuple) or len(state) != 5:
            raise pickle.UnpicklingError('ndarray state')
        _, shape, dt, fortran, raw = state
        dt = _as_dtype(dt)
        if isinstance(raw, str):               # protocol 0-2 pickles carry the bytes as latin-1 text
            raw = raw.encode('latin1')
        if not isinstance(raw, (bytes, bytearray)):
            raise pickle.UnpicklingError('ndarray data of type %r' % type(raw))
        shape = _shape(shape)
        n = math.prod(shape)
        if n * dt.itemsize != len(raw):
            raise pickle.UnpicklingError('ndarray of shape %s / %s with %d data bytes' % (shape, dt, len(raw)))
        a = np.frombuffer(bytes(raw), dt, count=n).reshape(shape, order='F' if fortran else 'C')
        self.array = a.astype(dt.newbyteorder('='), copy=True)


def _frombuffer(buf, dt, shape, order):
    """numpy.core.numeric._frombuffer as pickled by protocol 5 (in-band buffer)."""
    dt = _as_dtype(dt)
    raw = bytes(buf)
    shape = _shape(shape)
    n = math.prod(shape)
    if n * dt.itemsize != len(raw) or order not in ('C', 'F'):
        raise pickle.UnpicklingError('ndarray buffer')
    return np.frombuffer(raw, dt, count=n).reshape(shape, order=order).astype(dt.newbyteorder('='), copy=True)


def _scalar(dt, raw=None):
    """numpy.core.multiarray.scalar(dtype, bytes): a numpy scalar (e.g. a float64 height)."""
    dt = _as_dtype(dt)
    if isinstance(raw, str):
        raw = raw.encode('latin1')
    if not isinstance(raw, (bytes, bytearray)) or len(raw) != dt.itemsize:
        raise pickle.UnpicklingError('numpy scalar data')
    return np.frombuffer(bytes(raw), dt, count=1)[0].astype(dt.newbyteorder('=')).item()


def _codecs_encode(s, enc='utf-8'):
    if enc != 'latin1' or not isinstance(s, str):
        raise pickle.UnpicklingError('_codecs.encode(%r)' % enc)
    return s.encode('latin1')


_NDARRAY = object()
_MODS = ('numpy.core.multiarray', 'numpy._core.multiarray')
_SAFE = {('numpy', 'dtype'): _DType, ('numpy', 'ndarray'): _NDARRAY, ('_codecs', 'encode'): _codecs_encode}
for _m in _MODS:
    _SAFE[(_m, '_reconstruct')] = _ArrayBuilder
    _SAFE[(_m, 'scalar')] = _scalar
for _m in ('numpy.core.numeric', 'numpy._core.numeric'):
    _SAFE[(_m, '_frombuffer')] = _frombuffer


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        f = _SAFE.get((module, name))
        if f is None:
            raise pickle.UnpicklingError('%s.%s is not admitted by the recording reader' % (module, name))
        return f

    def persistent_load(self, pid):
        raise pickle.UnpicklingError('persistent ids are not admitted')


def _finish(x):
    if isinstance(x, _ArrayBuilder):
        if x.array is None:
            raise pickle.UnpicklingError('ndarray without state')
        return x.array
    if isinstance(x, (_DType,)) or x is _NDARRAY:
        raise pickle.UnpicklingError('stray numpy object')
    if isinstance(x, list):
        return [_finish(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_finish(v) for v in x)
    if isinstance(x, dict):
        return {_finish(k): _finish(v) for k, v in x.items()}
    if x is None or isinstance(x, (bool, int, float, complex, str, bytes, np.ndarray)):
        return x
    raise pickle.UnpicklingError('object of type %r' % type(x))


def load_reference_pickle(path):
    """Read a reference recording's pickle (setup.pkl / actions.pkl) without executing anything
    from the file (see the module docstring); raises pickle.UnpicklingError on anything else."""
    with open(path, 'rb') as f:
        try:
            return _finish(_RestrictedUnpickler(f).load())
        except pickle.UnpicklingError:
            raise
        except (EOFError, ValueError, TypeError, IndexError, KeyError, AttributeError, OverflowError, MemoryError,
                RecursionError, UnicodeError) as e:      # malformed input, whatever opcode it broke
            raise pickle.UnpicklingError('%s: malformed pickle (%s: %s)' % (path, type(e).__name__, e)) from e


def write_reference_recording(directory, robot_type, gender, hipbone_to_mouth_height, actions):
    """Write setup.pkl and actions.pkl as the reference's VR episodes do (feeding.py:50-54,
    328-329): [robot_type, gender, hipbone_to_mouth_height] and the list of 200 actions."""
    os.makedirs(directory, exist_ok=True)
    with open(os.path.join(directory, 'setup.pkl'), 'wb') as f:
        pickle.dump([robot_type, gender, hipbone_to_mouth_height], f)
    with open(os.path.join(directory, 'actions.pkl'), 'wb') as f:
        pickle.dump([np.asarray(a, np.float32) for a in actions], f)


_TASK_KEYS = (('scratch_itch', 'ScratchItch'), ('feeding', 'Feeding'), ('drinking', 'Drinking'), ('bed_bathing', 'BedBathing'))


def reference_env_id(directory):
    """The env id replay_vr_savemeta.py derives from a recording directory's name
    (replay_vr_savemeta.py:20): task from 'scratch_itch' / 'feeding' / 'drinking' /
    'bed_bathing', robot 'Jaco' if 'jaco' is in the name, else 'PR2'.  None: skipped."""
    d = os.path.basename(os.path.normpath(directory))
    for k, name in _TASK_KEYS:
        if k in d:
            return '%s%s-v0' % (name, 'Jaco' if 'jaco' in d else 'PR2')
    return None


class ReferenceReplayEnv:
    """replay_setup(dir) + reset/step over a reference participant directory (setup.pkl,
    actions.pkl).  reset() sets up the recorded gender and starts from this build's reset for it;
    each step() re-simulates the next recorded action (the action passed in is ignored, as in
    feeding.py:38); done after the last recorded action (feeding.py:79-80: 200).

    The human is built at the recording's hipbone_to_mouth_height (feeding.py:153-156 reads it
    from setup.pkl before create_new_world; AVRVecEnv's human_heights), on this build's non-VR
    human model -- the reference builds its VR human for replays (world_creation.py:19-20), a
    model this build does not compile.  default_proportions=True replays on the default human
    instead (noted in `self.proportions`).  The recording's frame_%d.bullet states are not read."""

    def __init__(self, directory, env_id=None, device=0, seed=1001, default_proportions=False):
        from . import env as EV
        self.directory = directory
        self.env_id = env_id or reference_env_id(directory)
        if self.env_id is None:
            raise ValueError('%s: no task name in the directory name (replay_vr_savemeta.py:20)' % directory)
        setup = load_reference_pickle(os.path.join(directory, 'setup.pkl'))
        if not isinstance(setup, (list, tuple)) or len(setup) != 3:
            raise ValueError('%s/setup.pkl: expected [robot_type, gender, hipbone_to_mouth_height]' % directory)
        self.robot_type, self.gender, hip = setup
        self.hipbone_to_mouth_height = None if hip is None else float(hip)
        if self.gender not in ('male', 'female'):
            raise ValueError('%s/setup.pkl: gender %r' % (directory, self.gender))
        acts = load_reference_pickle(os.path.join(directory, 'actions.pkl'))
        self.action_list = np.asarray([np.asarray(a, np.float32).reshape(-1) for a in acts], np.float32)
        hip = self.hipbone_to_mouth_height
        self.proportions = 'recorded' if hip is not None else 'default'
        if hip is not None and default_proportions:
            hip, self.proportions = None, 'default (recorded %.4f)' % self.hipbone_to_mouth_height
        self.env = EV.AVRVecEnv(self.env_id, 1, device=device, seed=seed, auto_reset=False, prefetch=False,
                                human_heights={self.gender: hip})
        if self.action_list.ndim != 2 or self.action_list.shape[1] != self.env.L.ACT_DIM:
            self.env.close()
            raise ValueError('%s/actions.pkl: actions of shape %s, the task takes %d' % (directory, self.action_list.shape, self.env.L.ACT_DIM))
        self.env.setup(self.gender, -1, '', hip)
        self.iteration = 0

    def reset(self):
        self.iteration = 0
        return self.env.reset()

    def step(self, action=None):
        obs, rew, _, info = self.env.step(self.action_list[self.iteration][None])
        self.iteration += 1
        done = np.full(1, self.iteration >= len(self.action_list))
        return obs, rew, done, info

    def close(self):
        self.env.close()


def savemeta_reference(replay_dir, out=None, device=0, default_proportions=False):
    """replay_vr_savemeta.py: every participant_*/* recording under replay_dir replayed; per
    directory the observations, rewards, actions, total_force_on_human per step and the final
    task_success (an .npz at `out`, not a pickle)."""
    res = {}
    for d in sorted(glob.glob(os.path.join(replay_dir, 'participant_*', '*'))):
        if reference_env_id(d) is None or not os.path.exists(os.path.join(d, 'setup.pkl')):
            continue
        r = ReferenceReplayEnv(d, device=device, default_proportions=default_proportions)
        r.reset()
        obs, rews, forces, succ = [], [], [], 0.0
        done = np.zeros(1, bool)
        while not done.all():
            o, rw, done, info = r.step()
            obs.append(o[0]); rews.append(float(rw[0])); forces.append(float(info['total_force_on_human'][0]))
            succ = float(info['task_success'][0])
        res[d] = dict(env_id=r.env_id, observations=np.stack(obs), rewards=np.array(rews), actions=r.action_list,
                      forces=np.array(forces), task_success=succ, proportions=r.proportions)
        r.close()
    if out:
        flat = {'dirs': np.array(list(res))}
        for i, v in enumerate(res.values()):
            for k in ('observations', 'rewards', 'actions', 'forces', 'task_success'):
                flat['%d_%s' % (i, k)] = np.asarray(v[k])
        np.savez(out, **flat)
    return res
