"""ctypes binding of libavr.so (include/avr.h) -- the product path.

The library is built in-tree (`python -m avr.build` or `__graft_entry__.build()`) for gfx950.
There is no fallback: if the shared object or a GPU is missing, the calls raise.
"""
import ctypes as C
import os

import numpy as np

from . import _abi as ABI

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('AVR_LIB') or os.path.join(HERE, 'libavr.so')   # AVR_LIB: experiment builds

EXPORTS = [
    'avr_create', 'avr_destroy', 'avr_set_state', 'avr_get_state', 'avr_set_state_masked', 'avr_settle',
    'avr_step', 'avr_step_device', 'avr_step_random_device', 'avr_rollout_random_device', 'avr_random_actions_device', 'avr_sync',
    'avr_stream', 'avr_state_device_ptr', 'avr_n_envs', 'avr_env_groups', 'avr_state_words', 'avr_abi_version',
    'avr_kernel_info', 'avr_last_error', 'avr_substep', 'avr_reset', 'avr_profile_kernels', 'avr_kernel_times',
    'avr_hull_support_table', 'avr_task', 'avr_task_state_words', 'avr_task_obs_dim', 'avr_task_act_dim', 'avr_n_dof',
    'avr_get_q', 'avr_get_link_pose', 'avr_get_contact_summary', 'avr_get_flags', 'avr_reset_ik', 'avr_base_search',
    'avr_graph_captures', 'avr_robot_self_contact', 'avr_narrowphase_query',
]
FLAGS_FAULT_MASK = 0x1f      # include/avr.h AVR_FLAGS_FAULT_MASK: bits 0-4; bit 5 (EPA budget) is informational


# avr_config.flags: no bit is defined (include/avr.h); avr_create rejects any set bit


class avr_config(C.Structure):
    _fields_ = [('n_envs', C.c_int32), ('device', C.c_int32), ('env_offset', C.c_int32), ('flags', C.c_int32),
                ('seed', C.c_uint64)]


_LIB = None


def load(path=LIB_PATH):
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError('libavr.so not built (%s); run __graft_entry__.build()' % path)
    # One HIP runtime per process: if torch is importable, let it load its libamdhip64 first so
    # libavr binds to the same runtime (device pointers from torch tensors stay valid here).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.avr_create.argtypes = [C.POINTER(avr_config), vp, C.POINTER(vp)]
    if hasattr(lib, 'avr_hull_support_table'):      # (absent in experiment builds of older trees)
        lib.avr_hull_support_table.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, C.c_int32]
        lib.avr_hull_support_table.restype = C.c_int32
    lib.avr_destroy.argtypes = [vp]
    lib.avr_set_state.argtypes = [vp, vp]
    lib.avr_get_state.argtypes = [vp, vp]
    lib.avr_set_state_masked.argtypes = [vp, vp, vp]
    lib.avr_settle.argtypes = [vp, C.c_int32, vp]
    lib.avr_step.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.avr_step_device.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.avr_step_random_device.argtypes = [vp, C.c_int64, vp, vp, vp, vp]
    lib.avr_rollout_random_device.argtypes = [vp, C.c_int64, C.c_int32, vp, vp, vp, vp, C.c_int32]
    lib.avr_random_actions_device.argtypes = [vp, C.c_int64, vp]
    lib.avr_sync.argtypes = [vp]
    lib.avr_stream.argtypes = [vp]
    lib.avr_stream.restype = vp
    lib.avr_state_device_ptr.argtypes = [vp]
    lib.avr_state_device_ptr.restype = vp
    lib.avr_n_envs.argtypes = [vp]
    lib.avr_env_groups.argtypes = [vp]
    lib.avr_env_groups.restype = C.c_int32
    lib.avr_graph_captures.argtypes = [vp]
    lib.avr_graph_captures.restype = C.c_int64
    lib.avr_state_words.restype = C.c_int32
    lib.avr_abi_version.restype = C.c_int32
    lib.avr_kernel_info.argtypes = [vp, vp]
    lib.avr_last_error.argtypes = [vp]
    lib.avr_last_error.restype = C.c_char_p
    lib.avr_substep.argtypes = [vp, C.c_float]
    lib.avr_reset.argtypes = [vp, vp, vp, C.c_int32, vp]
    lib.avr_profile_kernels.argtypes = [vp, C.c_int32]
    lib.avr_kernel_times.argtypes = [vp, vp, vp]
    lib.avr_task.argtypes = [vp]
    lib.avr_n_dof.argtypes = [vp]
    for f in ('avr_task_state_words', 'avr_task_obs_dim', 'avr_task_act_dim'):
        getattr(lib, f).argtypes = [C.c_int32]
        getattr(lib, f).restype = C.c_int32
    lib.avr_get_q.argtypes = [vp, vp, vp]
    lib.avr_get_link_pose.argtypes = [vp, C.c_int32, vp]
    lib.avr_get_contact_summary.argtypes = [vp, vp]
    lib.avr_get_flags.argtypes = [vp, vp]
    lib.avr_reset_ik.argtypes = [vp, vp, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_float, vp, C.c_int32, vp, vp]
    lib.avr_robot_self_contact.argtypes = [vp, C.c_int32, vp, vp]
    lib.avr_narrowphase_query.argtypes = [vp, C.c_int32, vp, vp, C.c_float, vp]
    lib.avr_base_search.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp, C.c_int32, C.c_float, vp, vp, vp, vp]
    if lib.avr_abi_version() != ABI.ABI_VERSION or any(
            lib.avr_task_state_words(t) != L.STATE_WORDS or lib.avr_task_obs_dim(t) != L.OBS_DIM or lib.avr_task_act_dim(t) != L.ACT_DIM
            for t, L in ABI.LAYOUTS.items()):
        raise RuntimeError('%s: ABI %d / state layouts differ from this package (ABI %d); rebuild'
                           % (path, lib.avr_abi_version(), ABI.ABI_VERSION))
    _LIB = lib
    return lib


class Sim:
    """One libavr handle = one GPU, n_envs environments."""

    def __init__(self, md, n_envs, device=0, seed=1001, env_offset=0, flags=0):
        """flags: avr_config.flags, must be 0 (include/avr.h)."""
        self.lib = load()
        self.md = md
        self.n = int(n_envs)
        self.kernel_kinds = ('avr_take_step_kernel', 'avr_substep_a_kernel', 'avr_substep_b4_kernel', 'avr_task_kernel',
                             'avr_substep_pairs_kernel', 'avr_narrowphase_kernel', 'avr_coop_kernel')
        cfg = avr_config(n_envs=self.n, device=device, env_offset=env_offset, flags=int(flags), seed=seed)
        h = C.c_void_p()
        rc = self.lib.avr_create(C.byref(cfg), C.cast(md.ptr(), C.c_void_p), C.byref(h))
        self.h = h
        if rc:
            msg = self.lib.avr_last_error(h).decode() if h.value else 'avr_create failed'
            if h.value:
                self.lib.avr_destroy(h)
                self.h = None
            raise RuntimeError('avr_create failed (%d): %s' % (rc, msg))
        self.task = int(self.lib.avr_task(h))
        self.L = ABI.LAYOUTS[self.task]
        if self.task == ABI.TASK_DRESSING:      # one kernel per step, timed in kind slot 2 (avr_dressing.hip)
            self.kernel_kinds = ('-', '-', 'avr_dress_step_kernel', '-', '-', '-', '-')
        self.words = self.lib.avr_task_state_words(self.task)
        self.obs_dim, self.act_dim = self.L.OBS_DIM, self.L.ACT_DIM

    def _chk(self, rc):
        if rc:
            raise RuntimeError(self.lib.avr_last_error(self.h).decode())

    def close(self):
        if getattr(self, 'h', None):
            self.lib.avr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_state(self, S):
        S = np.ascontiguousarray(S, np.float32).reshape(self.n, self.words)
        self._chk(self.lib.avr_set_state(self.h, S.ctypes.data))

    def set_state_masked(self, mask, S):
        S = np.ascontiguousarray(S, np.float32).reshape(self.n, self.words)
        mask = np.ascontiguousarray(mask, np.uint8)
        self._chk(self.lib.avr_set_state_masked(self.h, mask.ctypes.data, S.ctypes.data))

    def get_state(self):
        S = np.zeros((self.n, self.words), np.float32)
        self._chk(self.lib.avr_get_state(self.h, S.ctypes.data))
        return S

    def settle(self, frames=100):
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        self._chk(self.lib.avr_settle(self.h, frames, obs.ctypes.data))
        return obs

    def reset(self, mask, S, frames=100, obs=None):
        """Masked episode reset (include/avr.h avr_reset): rows of S for mask!=0, settle, obs."""
        S = np.ascontiguousarray(S, np.float32).reshape(self.n, self.words)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8).reshape(self.n)
        if obs is None:
            obs = np.zeros((self.n, self.obs_dim), np.float32)
        assert obs.dtype == np.float32 and obs.flags.c_contiguous and obs.shape == (self.n, self.obs_dim)
        self._chk(self.lib.avr_reset(self.h, None if m is None else m.ctypes.data, S.ctypes.data, int(frames), obs.ctypes.data))
        return obs

    def reset_ik(self, mask, S, target7, init, iters=80, tol=0.01, keepout8=None, frames=100, obs=None, alt=None):
        """Masked reset with the IK on the device (include/avr.h avr_reset_ik): S rows without the
        arm joints, target7 (n_envs, 7), init (n_envs, restarts, n_arm) restart draws, alt
        (n_envs, restarts, 4) the self-contact screening's re-drawn orientations (None: no
        screening).  Returns (obs, ok)."""
        S = np.ascontiguousarray(S, np.float32).reshape(self.n, self.words)
        t = np.ascontiguousarray(target7, np.float32).reshape(self.n, 7)
        init = np.ascontiguousarray(init, np.float32)
        assert init.ndim == 3 and init.shape[0] == self.n
        if alt is not None:
            alt = np.ascontiguousarray(alt, np.float32)
            assert alt.shape == (self.n, init.shape[1], 4)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8).reshape(self.n)
        box = None if keepout8 is None else np.ascontiguousarray(keepout8, np.float32).reshape(8)
        if obs is None:
            obs = np.zeros((self.n, self.obs_dim), np.float32)
        assert obs.dtype == np.float32 and obs.flags.c_contiguous and obs.shape == (self.n, self.obs_dim)
        ok = np.zeros(self.n, np.uint8)
        self._chk(self.lib.avr_reset_ik(self.h, None if m is None else m.ctypes.data, S.ctypes.data, t.ctypes.data, init.ctypes.data,
                                        None if alt is None else alt.ctypes.data, int(init.shape[1]), int(iters), float(tol), None if box is None else box.ctypes.data, int(frames),
                                        obs.ctypes.data, ok.ctypes.data))
        return obs, ok.astype(bool)

    def robot_self_contact(self, Q):
        """Touching robot shape pairs at each row of Q (n, n_dof()) -- avr_get_q's layout, or just
        the robot DoFs (the human chain's then 0) -- (include/avr.h avr_robot_self_contact:
        p.getContactPoints(robot, robot) after a reset restart)."""
        Q = np.asarray(Q, np.float32)
        nd = self.n_dof()
        assert Q.ndim == 2 and Q.shape[1] <= nd
        q = np.zeros((len(Q), nd), np.float32)
        q[:, :Q.shape[1]] = Q
        out = np.zeros(len(q), np.int32)
        self._chk(self.lib.avr_robot_self_contact(self.h, int(len(q)), q.ctypes.data, out.ctypes.data))
        return out

    def narrowphase(self, pairs, poses14, thr=0.02):
        """The step's narrowphase per (sa, sb) row of pairs at body poses poses14 (n, 14)
        (include/avr.h avr_narrowphase_query): (n, 8) {rc, normal on B, point on B, distance}."""
        p = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        x = np.ascontiguousarray(poses14, np.float32).reshape(len(p), 14)
        out = np.zeros((len(p), 8), np.float32)
        self._chk(self.lib.avr_narrowphase_query(self.h, int(len(p)), p.ctypes.data, x.ctypes.data, float(thr), out.ctypes.data))
        return out

    def base_search(self, base7, rest, tstart, goals, iters=200, tol=0.03, per_attempt=False):
        """PR2 base-pose search on the device (include/avr.h avr_base_search): base7 (n, attempts, 7),
        rest (n, attempts, n_arm), tstart (n, 3), goals (n, 3, 3).  Returns (best (n,) attempt index,
        ok (n,) bool, q_arm (n, n_arm)[, res (n, attempts, 4) when per_attempt])."""
        b = np.ascontiguousarray(base7, np.float32)
        assert b.ndim == 3 and b.shape[2] == 7
        n, att = b.shape[:2]
        r = np.ascontiguousarray(rest, np.float32)
        na = r.shape[2]
        assert r.shape[:2] == (n, att)
        t = np.ascontiguousarray(tstart, np.float32).reshape(n, 3)
        g = np.ascontiguousarray(goals, np.float32).reshape(n, 9)
        best = np.zeros(n, np.int32)
        ok = np.zeros(n, np.uint8)
        q = np.zeros((n, na), np.float32)
        res = np.zeros((n, att, 4), np.float32) if per_attempt else None
        self._chk(self.lib.avr_base_search(self.h, int(n), int(att), b.ctypes.data, r.ctypes.data, t.ctypes.data, g.ctypes.data, int(iters),
                                           float(tol), best.ctypes.data, ok.ctypes.data, q.ctypes.data, None if res is None else res.ctypes.data))
        return (best, ok.astype(bool), q) + ((res,) if per_attempt else ())

    def substep(self, dt):
        self._chk(self.lib.avr_substep(self.h, dt))

    def step(self, act):
        act = np.ascontiguousarray(act, np.float32).reshape(self.n, self.act_dim)
        obs = np.zeros((self.n, self.obs_dim), np.float32)
        rew = np.zeros(self.n, np.float32)
        done = np.zeros(self.n, np.uint8)
        info = np.zeros((self.n, ABI.INFO_DIM), np.float32)
        self._chk(self.lib.avr_step(self.h, act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data, info.ctypes.data))
        return obs, rew, done.astype(bool), info

    # device-pointer variants (torch tensors' data_ptr()); asynchronous on the handle's stream
    def step_device(self, d_act, d_obs, d_rew, d_done, d_info):
        self._chk(self.lib.avr_step_device(self.h, d_act, d_obs, d_rew, d_done, d_info))

    def step_random_device(self, t, d_obs=None, d_rew=None, d_done=None, d_info=None):
        self._chk(self.lib.avr_step_random_device(self.h, int(t), d_obs, d_rew, d_done, d_info))

    def rollout_random_device(self, t0, n, d_obs=None, d_rew=None, d_done=None, d_info=None, stacked=False):
        """n device-random steps from step index t0 (= n step_random_device calls, bit for bit); the
        env groups are joined at the end only.  stacked: step k's outputs to slot k of [n, E, ...]
        device arrays (all four required)."""
        self._chk(self.lib.avr_rollout_random_device(self.h, int(t0), int(n), d_obs, d_rew, d_done, d_info, int(bool(stacked))))

    def random_actions_device(self, t, d_act):
        self._chk(self.lib.avr_random_actions_device(self.h, int(t), d_act))

    def sync(self):
        self._chk(self.lib.avr_sync(self.h))

    def stream(self):
        return self.lib.avr_stream(self.h)

    def env_groups(self):
        return int(self.lib.avr_env_groups(self.h))

    def graph_captures(self):
        """HIP-graph captures this handle has made (one per distinct output-buffer key)."""
        return int(self.lib.avr_graph_captures(self.h))

    def profile_kernels(self, enable=True):
        self._chk(self.lib.avr_profile_kernels(self.h, int(bool(enable))))

    def kernel_times(self):
        """{kernel: (total_ms, launches)} accumulated since profile_kernels(True)."""
        ms = np.zeros(8, np.float64)
        n = np.zeros(8, np.int64)
        self._chk(self.lib.avr_kernel_times(self.h, ms.ctypes.data, n.ctypes.data))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(self.kernel_kinds) if n[i]}

    # ---- state queries (include/avr.h avr_get_*)
    def n_dof(self):
        return int(self.lib.avr_n_dof(self.h))

    def get_q(self):
        """(q, qd), each (n_envs, n_dof): robot DoFs, then the articulated human chain's."""
        nd = self.n_dof()
        q = np.zeros((self.n, nd), np.float32)
        qd = np.zeros((self.n, nd), np.float32)
        self._chk(self.lib.avr_get_q(self.h, q.ctypes.data, qd.ctypes.data))
        return q, qd

    def get_link_pose(self, link):
        """(n_envs, 7) world COM frame of articulated link `link` (-1: robot base)."""
        out = np.zeros((self.n, 7), np.float32)
        self._chk(self.lib.avr_get_link_pose(self.h, int(link), out.ctypes.data))
        return out

    def get_contact_summary(self):
        """(n_envs, 4): contact points, sum of normal force, robot-human, tool-human."""
        out = np.zeros((self.n, 4), np.float32)
        self._chk(self.lib.avr_get_contact_summary(self.h, out.ctypes.data))
        return out

    def get_flags(self):
        """(n_envs,) int32 health flags (0 = healthy; bits in include/avr.h avr_get_flags)."""
        out = np.zeros(self.n, np.int32)
        self._chk(self.lib.avr_get_flags(self.h, out.ctypes.data))
        return out

    def kernel_info(self):
        """{kernel: dict(vgprs, lds_bytes, scratch_bytes)} of the step's kernels (include/avr.h)."""
        out = np.zeros(20, np.int32)
        self._chk(self.lib.avr_kernel_info(self.h, out.ctypes.data))
        names = ('pairs', 'narrowphase', 'a', 'b', 'task')
        return {n: dict(vgprs=int(out[4 * i]), lds_bytes=int(out[4 * i + 2]), scratch_bytes=int(out[4 * i + 3])) for i, n in enumerate(names)}


# ---------------------------------------------------------------- Philox4x32-10 (host mirror)
M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85


def philox4x32_10(c, k0, k1):
    """Vectorised Philox4x32-10 on uint64 arrays holding 32-bit values; c: (4, N)."""
    c = [np.asarray(x, np.uint64) & 0xFFFFFFFF for x in c]
    k0 = np.uint64(k0 & 0xFFFFFFFF)
    k1 = np.uint64(k1 & 0xFFFFFFFF)
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c[0]
        p1 = np.uint64(M1) * c[2]
        h0, l0 = p0 >> np.uint64(32), p0 & mask
        h1, l1 = p1 >> np.uint64(32), p1 & mask
        c = [h1 ^ c[1] ^ k0, l1, h0 ^ c[3] ^ k1, l0]
        k0 = (k0 + np.uint64(W0)) & mask
        k1 = (k1 + np.uint64(W1)) & mask
    return c


def random_actions(seed, env_ids, t, act_dim=ABI.ACT_DIM):
    """a[e, j] ~ U(-1,1) float32 from Philox4x32-10 keyed by (seed, env, t) -- identical to the
    device generator (examples/random_actions.py semantics with a counter-based stream)."""
    env_ids = np.asarray(env_ids, np.uint64)
    out = np.zeros((len(env_ids), act_dim), np.float32)
    for blk in range((act_dim + 3) // 4):
        c = [env_ids, np.full_like(env_ids, t & 0xFFFFFFFF), np.full_like(env_ids, blk), np.full_like(env_ids, (t >> 32) & 0xFFFFFFFF)]
        r = philox4x32_10(c, seed, seed >> 32)
        for k in range(4):
            j = 4 * blk + k
            if j < act_dim:
                x = (r[k] >> np.uint64(8)).astype(np.float32)
                out[:, j] = x * np.float32(1.0 / 16777216.0) * np.float32(2.0) - np.float32(1.0)
    return out


def hull_support_table(verts, G=16):
    """Host support table of one hull (avr_hull_support_table): (cell[6G^2, 2], idx[total])."""
    lib = load()
    v = np.ascontiguousarray(verts, dtype=np.float32).reshape(-1, 3)
    cell = np.zeros((6 * G * G, 2), dtype=np.int32)
    tot = lib.avr_hull_support_table(v.ctypes.data, len(v), G, cell.ctypes.data, None, 0)
    if tot < 0:
        raise RuntimeError('avr_hull_support_table failed')
    idx = np.zeros(max(tot, 1), dtype=np.int32)
    lib.avr_hull_support_table(v.ctypes.data, len(v), G, cell.ctypes.data, idx.ctypes.data, tot)
    return cell, idx[:tot]
