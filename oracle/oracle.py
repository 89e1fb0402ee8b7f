"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU oracle (oracle/avr_oracle.c).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker / baseline, never as the measured or shipped path.  Parity vs PyBullet is
UNPINNED (PyBullet is absent from this image); the oracle is pinned by analytic
known-answer tests and by self-generated golden vectors (tests/golden/).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def _load(precision, task=0):
    name = 'libavr_oracle%s%s.so' % ({1: '_scratch', 2: '_bedbath', 3: '_dressing'}.get(task, ''), '' if precision == 'f64' else '_f32')
    path = os.path.join(HERE, name)
    if not os.path.exists(path):
        build()
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.avr_oracle_create.argtypes = [vp, C.c_int, C.POINTER(vp)]
    lib.avr_oracle_destroy.argtypes = [vp]
    lib.avr_oracle_set_state.argtypes = [vp, vp]
    lib.avr_oracle_get_state.argtypes = [vp, vp]
    lib.avr_oracle_settle.argtypes = [vp, C.c_int, vp]
    lib.avr_oracle_step.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.avr_oracle_set_threads.argtypes = [vp, C.c_int]
    lib.avr_oracle_last_error.argtypes = [vp]
    lib.avr_oracle_last_error.restype = C.c_char_p
    lib.avr_oracle_state_words.restype = C.c_int
    if task == 3:           # DressingJaco (oracle/avr_oracle_dressing.c): the step API only
        return lib
    lib.avr_oracle_substep.argtypes = [vp, C.c_double]
    lib.avr_oracle_stats.argtypes = [vp, vp]
    lib.avr_oracle_set_island_exit.argtypes = [vp, C.c_int]
    lib.avr_oracle_narrowphase.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_double, vp]
    lib.avr_oracle_robot_fk.argtypes = [vp, C.c_int, vp]
    lib.avr_oracle_robot_self_contact.argtypes = [vp, C.c_int, vp, vp]
    lib.avr_oracle_set_threads.argtypes = [vp, C.c_int]
    lib.avr_oracle_last_error.argtypes = [vp]
    lib.avr_oracle_last_error.restype = C.c_char_p
    lib.avr_oracle_state_words.restype = C.c_int
    if task == 2:
        lib.avr_oracle_bb_closest.argtypes = [vp, C.c_int, vp]
    return lib


_LIBS = {}


def lib(precision='f64', task=0):
    """The oracle build for `task` (0 FeedingJaco, 1 ScratchItchPR2, 2 BedBathingPR2; avr_model.h AVR_TASK_*)."""
    key = (precision, task)
    if key not in _LIBS:
        _LIBS[key] = _load(precision, task)
    return _LIBS[key]


class Oracle:
    def __init__(self, md, n_envs, precision='f64'):
        self.task = getattr(md, 'task', 0)
        self.lib = lib(precision, self.task)
        self.md = md
        self.n = n_envs
        h = C.c_void_p()
        rc = self.lib.avr_oracle_create(C.cast(md.ptr(), C.c_void_p), n_envs, C.byref(h))
        if rc:
            raise RuntimeError('avr_oracle_create failed: %d' % rc)
        self.h = h
        self.words = self.lib.avr_oracle_state_words()
        self.obs_dim = {1: 30, 2: 24, 3: 24}.get(self.task, 25)

    def set_threads(self, n):
        self.lib.avr_oracle_set_threads(self.h, int(n))

    def close(self):
        if self.h:
            self.lib.avr_oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_state(self, S):
        S = np.ascontiguousarray(S, np.float64).reshape(self.n, self.words)
        self.lib.avr_oracle_set_state(self.h, S.ctypes.data)

    def get_state(self):
        S = np.zeros((self.n, self.words))
        self.lib.avr_oracle_get_state(self.h, S.ctypes.data)
        return S

    def settle(self, frames=100):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        if self.lib.avr_oracle_settle(self.h, frames, obs.ctypes.data):
            raise RuntimeError(self.lib.avr_oracle_last_error(self.h).decode())
        return obs

    def step(self, act):
        act = np.ascontiguousarray(act, np.float32).reshape(self.n, 7)
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        rew = np.zeros(self.n, np.float32)
        done = np.zeros(self.n, np.uint8)
        info = np.zeros((self.n, 2), np.float32)
        if self.lib.avr_oracle_step(self.h, act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data, info.ctypes.data):
            raise RuntimeError(self.lib.avr_oracle_last_error(self.h).decode())
        return obs, rew, done.astype(bool), info

    def substep(self, dt):
        if self.lib.avr_oracle_substep(self.h, float(dt)):
            raise RuntimeError('substep failed')

    def set_island_exit(self, on=True):
        """Test-only: the PGS residual exit per island instead of per env (solve_islands)."""
        self.lib.avr_oracle_set_island_exit(self.h, int(bool(on)))

    def stats(self):
        s = np.zeros(6, np.int64)      # GJK runs, EPA runs, rows built, PGS iterations, PGS solves, stall reruns
        self.lib.avr_oracle_stats(self.h, s.ctypes.data)
        return s

    def narrowphase(self, sa, pa, sb, pb, thr):
        out = np.zeros(7)
        pa = np.ascontiguousarray(pa, np.float64)
        pb = np.ascontiguousarray(pb, np.float64)
        r = self.lib.avr_oracle_narrowphase(self.h, sa, pa.ctypes.data, sb, pb.ctypes.data, thr, out.ctypes.data)
        return bool(r), out

    def bb_closest(self, env=0):
        """BedBathing: min getClosestPoints(tool, human, 4.0) distance of env's current state."""
        out = np.zeros(1)
        self.lib.avr_oracle_bb_closest(self.h, int(env), out.ctypes.data)
        return float(out[0])

    def robot_self_contact(self, Q):
        """Touching robot shape pairs at each row of Q (n, robot DoFs [+ head chain]), env 0's
        state otherwise (avr_oracle_robot_self_contact; the device's avr_robot_self_contact)."""
        Q = np.asarray(Q, np.float64)
        nq = self.md.desc.n_dof + self.md.desc.hc_n
        q = np.zeros((len(Q), nq))
        q[:, :Q.shape[1]] = Q
        out = np.zeros(len(Q), np.int32)
        r = self.lib.avr_oracle_robot_self_contact(self.h, len(q), q.ctypes.data, out.ctypes.data)
        assert r == 0
        return out

    def robot_fk(self, env=0):
        out = np.zeros((self.md.desc.n_links, 7))
        self.lib.avr_oracle_robot_fk(self.h, env, out.ctypes.data)
        return out
