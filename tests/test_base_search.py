"""PR2 base-pose search on the device (include/avr.h avr_base_search, csrc/avr_base_search.hip)
against its fp64 host restatement (avr/reset_scratch.position_robot_toc / base_search_host,
env.py:489-585).

CPU: the host search's rules -- per-row early exit makes every attempt independent of the batch
it runs in; the draws follow the documented ranges.
GPU: on the same draws the device reaches the same goals on the same attempts, its manipulability
agrees, the chosen bases are the host's for nearly every env, and every base the device accepts is
valid when re-checked in fp64; a PR2 env's rollover through AVRVecEnv uses it."""
import numpy as np
import pytest

from avr import _abi as ABI
from avr import reset as RS
from avr import reset_scratch as RSS

TOL = 0.03


def _scene(task):
    A = ABI.load_scene(task)
    return A, ABI.ModelDesc(A)


def _inputs(A, md, n, attempts, task):
    """Draws and human goals of n envs (ScratchItch: the reset's own human pose per env)."""
    rngs = [RS._rng(1001, e, 0) for e in range(n)]
    lo, hi = RS.arm_limits(md)
    As = A if task == ABI.TASK_SCRATCH else ABI.load_scene(ABI.TASK_SCRATCH)
    goals = np.zeros((n, 3, 3))
    for k in range(n):                 # the seated human's shoulder, elbow, wrist (scratch_itch.py:187-190)
        g = 'male' if k % 2 == 0 else 'female'
        qh, _, _ = RSS.human_joint_angles(As, g)
        _, _, P, _ = RS.human_link_poses(As, g, qh)
        goals[k] = P[[9, 11, 13]]
    tstart = None if task == ABI.TASK_SCRATCH else np.repeat(np.array([[-0.5, -0.1, 1.0]]), n, 0)
    off = (0.1, 0, 0) if task == ABI.TASK_SCRATCH else (0, 0, 0)
    ts, base, rest = RSS.base_search_draws(rngs, attempts, lo, hi, off, tstart)
    return ts, base, rest, goals


def _check_fp64(A, md, base, q_arm, tstart):
    """fp64 FK of the tool link at the device's joints: within TOL of the start goal."""
    nd = int(A['n_dof'])
    Q = np.zeros((len(base), nd))
    Q[:, md.arm_dofs] = q_arm
    CP, CQ, _, _ = RSS.arm_fk(A, Q, base[:, :3], base[:, 3:])
    link = int(A['task_tool_link'])
    pe = np.linalg.norm(CP[:, link] - tstart, axis=1)
    qe = np.linalg.norm(CQ[:, link] - np.array([0, 0, 0, 1.0]), axis=1)
    return pe, qe


def test_draw_ranges():
    A, md = _scene(ABI.TASK_SCRATCH)
    ts, base, rest, _ = _inputs(A, md, 4, 50, ABI.TASK_SCRATCH)
    lo, hi = RS.arm_limits(md)
    assert base.shape == (4, 50, 7) and rest.shape == (4, 50, len(md.arm_dofs))
    x = base[..., 0] - (-0.85 + 0.1)
    y = base[..., 1] - (-0.4)
    assert np.all((x >= -0.5) & (x <= 0)) and np.all((y >= -0.5) & (y <= 0.5))
    yaw = 2 * np.arctan2(base[..., 5], base[..., 6])
    assert np.all(np.abs(yaw) <= np.deg2rad(30) + 1e-12)
    np.testing.assert_allclose(np.linalg.norm(base[..., 3:], axis=-1), 1.0, atol=1e-12)
    assert np.all((rest >= lo) & (rest <= hi))
    assert np.all(np.abs(ts - np.array([-0.55, 0, 0.8])) <= 0.05)


def test_host_search_is_batch_independent():
    """ik_dls stops each row on its own: an attempt's result does not depend on its batch."""
    A, md = _scene(ABI.TASK_SCRATCH)
    ts, base, rest, goals = _inputs(A, md, 3, 6, ABI.TASK_SCRATCH)
    g_all, m_all, pe_all, q_all = RSS.base_search_host(A, md, base, rest, ts, goals, 120)
    for e in range(3):
        g1, m1, pe1, q1 = RSS.base_search_host(A, md, base[e:e + 1, 2:4], rest[e:e + 1, 2:4], ts[e:e + 1], goals[e:e + 1], 120)
        np.testing.assert_array_equal(g1[0], g_all[e, 2:4])
        np.testing.assert_array_equal(q1[0], q_all[e, 2:4])
        np.testing.assert_array_equal(m1[0], m_all[e, 2:4])


def test_host_search_reaches_start_goal():
    A, md = _scene(ABI.TASK_SCRATCH)
    ts, base, rest, goals = _inputs(A, md, 4, 10, ABI.TASK_SCRATCH)
    g, m, pe, Q = RSS.base_search_host(A, md, base, rest, ts, goals, 200)
    assert (g >= 1).mean() > 0.3, g
    assert np.all(pe[g >= 1] < TOL)
    assert np.all(m[g >= 1] > 0)


@pytest.mark.gpu
@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH])
def test_device_search_matches_host(task):
    from avr import _lib
    A, md = _scene(task)
    n, att, iters = 24, 16, 200
    ts, base, rest, goals = _inputs(A, md, n, att, task)
    sim = _lib.Sim(md, 1)
    try:
        best, ok, q, res = sim.base_search(base, rest, ts, goals, iters=iters, tol=TOL, per_attempt=True)
    finally:
        sim.close()
    g_h, m_h, pe_h, Q_h = RSS.base_search_host(A, md, base, rest, ts, goals, iters)
    g_d = res[..., 0].astype(int)
    # the same goals on the same attempts (fp32 vs fp64 DLS: a start IK that converges near the
    # 0.03 threshold, or into another local solution, may differ)
    same = g_d == g_h
    assert same.mean() >= 0.9, (same.mean(), g_d, g_h)
    # start-goal error where both reached it; manipulability where both agree on the goals
    both = same & (g_h >= 1)
    assert both.sum() > 0.2 * n * att
    assert np.all(res[..., 2][both] < TOL)
    # (the position-only solves leave a 4-dimensional self-motion manifold: fp32 and fp64 DLS can
    # settle at different points of it, with a different JLWKI -- typically the same to 1e-6, for
    # some attempts a few 1e-2 apart; near a singular pose JLWKI ~ 0 carries no relative accuracy)
    dm = np.abs(res[..., 1][both] - m_h[both])
    rel = dm / np.maximum(m_h[both], 1e-9)
    assert np.median(rel) < 1e-3, np.median(rel)
    assert np.mean((rel < 1e-2) | (dm < 5e-3)) >= 0.8, np.sort(dm)[-10:]
    assert dm.max() < 0.25 and abs(res[..., 1][both].mean() - m_h[both].mean()) < 0.02 * m_h[both].mean()
    # the picked bases: the host's rule applied to the device's per-attempt results, and the
    # host's own pick for nearly every env
    for e in range(n):
        cand = [a for a in range(att) if g_d[e, a] > 0]
        if cand:
            key = max((g_d[e, a], res[e, a, 1], -a) for a in cand)
            assert best[e] == -key[2] and ok[e]
        else:
            assert not ok[e] and best[e] == int(np.argmin(res[e, :, 2]))
    hb = np.full(n, -1)
    for e in range(n):
        cand = [a for a in range(att) if g_h[e, a] > 0]
        if cand:
            hb[e] = -max((g_h[e, a], m_h[e, a], -a) for a in cand)[2]
    agree = (hb == best) | ((hb == -1) & ~ok)
    assert agree.mean() >= 0.75, (hb, best)
    # every accepted base is valid in fp64
    b = base[np.arange(n), best]
    pe, qe = _check_fp64(A, md, b, q, ts)
    assert np.all(pe[ok] < TOL + 1e-4), pe[ok]
    assert np.all((qe[ok] < TOL + 1e-4) | (np.abs(qe[ok] - 2) < TOL + 1e-4))


@pytest.mark.gpu
def test_feeding_has_no_base_search():
    from avr import _lib
    A, md = _scene(ABI.TASK_FEEDING)
    sim = _lib.Sim(md, 1)
    try:
        with pytest.raises(RuntimeError, match='base'):
            sim.base_search(np.zeros((1, 2, 7)), np.zeros((1, 2, 7)), np.zeros((1, 3)), np.zeros((1, 3, 3)))
    finally:
        sim.close()


@pytest.mark.gpu
def test_scratch_env_rollover_uses_device_search():
    """AVRVecEnv for ScratchItchPR2 at the reference's 100 attempts x 200 IK iterations: the reset
    runs through avr_base_search (seconds for 64 envs), bases land within the search box, and the
    episode steps."""
    import time
    from avr import env as E
    env = E.AVRVecEnv('ScratchItchPR2-v0', n_envs=64)
    try:
        assert env.device_search
        t0 = time.perf_counter()
        obs = env.reset()
        dt = time.perf_counter() - t0
        assert dt < 60, dt
        S = env.get_state()
        L = env.L
        bp = S[:, L.S_RBASE:L.S_RBASE + 3]
        assert np.all((bp[:, 0] >= -1.25 - 1e-5) & (bp[:, 0] <= -0.75 + 1e-5)), bp[:, 0]
        assert np.all(np.abs(bp[:, 1] + 0.4) <= 0.5 + 1e-5)
        assert np.all(np.isfinite(obs))
        o, r, d, i = env.step(np.zeros((64, L.ACT_DIM), np.float32))
        assert np.all(np.isfinite(o)) and np.all(np.isfinite(r))
    finally:
        env.close()


def test_retry_until_a_start_goal_is_reached():
    """position_robot_toc keeps drawing bases until one reaches the start goal (`while iteration <
    attempts or best_position is None`, env.py:509): with 2 attempts per env, the envs whose two
    bases both miss draw further blocks and take the first base that reaches it; envs that
    succeeded in the first block are untouched."""
    from avr import reset_scratch as RSS
    A = ABI.load_scene(ABI.TASK_SCRATCH)
    md = ABI.ModelDesc(A)
    P = RSS.prepare_reset(A, md, 1001, list(range(8)), attempts=2)
    P0 = dict(P)
    P0.pop('retry')
    S0, m0 = RSS.finish_reset(A, md, P0, iters=60)
    S1, m1 = RSS.finish_reset(A, md, P, iters=60)
    ok0 = np.array([m['base_ok'] for m in m0])
    ok1 = np.array([m['base_ok'] for m in m1])
    assert (~ok0).any(), 'the 2-attempt search should miss for some env'
    assert ok1.all() and np.all(ok1 >= ok0)
    np.testing.assert_array_equal(S1[ok0], S0[ok0])
    L = ABI.SI
    link = int(A['task_tool_link'])
    nd = int(A['n_dof'])
    for e in np.nonzero(~ok0)[0]:
        st = S1[e]
        CP, _, _, _ = RSS.arm_fk(A, st[L.S_Q:L.S_Q + nd][None], st[L.S_RBASE:L.S_RBASE + 3][None], st[L.S_RBASE + 3:L.S_RBASE + 7][None])
        assert np.linalg.norm(CP[0, link] - P['tstart'][e]) < 0.03


@pytest.mark.gpu
def test_device_search_retries_until_a_start_goal_is_reached():
    from avr import _lib, reset_scratch as RSS
    A = ABI.load_scene(ABI.TASK_SCRATCH)
    md = ABI.ModelDesc(A)
    P = RSS.prepare_reset(A, md, 1001, list(range(16)), attempts=2)
    P0 = dict(P)
    P0.pop('retry')
    sim = _lib.Sim(md, 16)
    try:
        S0, m0 = RSS.finish_reset(A, md, P0, iters=60, sim=sim)
        S1, m1 = RSS.finish_reset(A, md, P, iters=60, sim=sim)
    finally:
        sim.close()
    ok0 = np.array([m['base_ok'] for m in m0])
    ok1 = np.array([m['base_ok'] for m in m1])
    assert (~ok0).any() and ok1.all()
    np.testing.assert_array_equal(S1[ok0], S0[ok0])
    L = ABI.SI
    link, nd = int(A['task_tool_link']), int(A['n_dof'])
    for e in np.nonzero(~ok0)[0]:
        st = S1[e]
        CP, _, _, _ = RSS.arm_fk(A, st[L.S_Q:L.S_Q + nd][None], st[L.S_RBASE:L.S_RBASE + 3][None], st[L.S_RBASE + 3:L.S_RBASE + 7][None])
        assert np.linalg.norm(CP[0, link] - P['tstart'][e]) < 0.031
