"""ScratchItchPR2-v0 (BASELINE configs[2]): compiled scene facts, host reset path and oracle task
glue on the CPU; the gfx950 kernels through the C-ABI against the oracle on the GPU.

Tolerances (fp32 kernel vs fp64 oracle):
  * one sub-step: |dq| <= 1e-5 rad, tool body <= 1e-4;
  * 200 gym steps of random actions (tool and arm rarely touch): |dq| <= 1e-3 rad (north star);
  * contact regime (the scratcher pressed onto the arm, tests/scratch_util.contact_states): held
    against the fp32 build of the oracle, which shares the kernel's rounding class, at 1e-3 rad
    over 10 steps, and against fp64 at 5e-3 rad (contact makes the trajectories sensitive).
"""
import os

import numpy as np
import pytest

from avr import _abi as ABI

SI = ABI.SI
REF = '/root/reference/assistive_gym/envs/assets'


@pytest.fixture(scope='module')
def sc():
    import scratch_util as U
    return U.scene()


@pytest.fixture(scope='module')
def states(sc):
    import scratch_util as U
    A, md = sc
    return U.reset_states(A, md, range(8))


def oracle(md, n, precision='f64'):
    from oracle.oracle import Oracle
    o = Oracle(md, n, precision)
    o.set_threads(4)
    return o


# ----------------------------------------------------------------------------- CPU: scene
def test_pr2_subtree_topology(sc):
    A, md = sc
    assert int(A['n_links']) == 22 and int(A['n_dof']) == 14        # PR2 links 64..85, 14 DoF
    assert list(A['rl_urdf']) == list(range(64, 86))
    assert list(A['task_arm_dofs']) == list(range(7))                # joints 64,65,66,68,69,71,72 (world_creation.py:189)
    assert list(A['task_finger_dofs']) == [9, 10, 11, 12]            # 79..82 (world_creation.py:311)
    assert int(A['task_tool_link']) == 76 - 64                       # l_gripper_tool_frame (world_creation.py:332)
    lim = A['rl_has_limit'][A['rl_dof'] >= 0][:7]
    assert list(lim) == [1, 1, 1, 1, 0, 1, 0]                         # forearm / wrist roll continuous
    lo = A['rl_lower'][np.nonzero(A['rl_has_limit'])[0]][:3]
    assert np.allclose(lo, [-0.714601836603, -0.5236, -0.8])         # pr2_no_torso_lift_tall.urdf l_shoulder_*
    assert A['rl_mass'][0] == pytest.approx(25.799322)               # inertia from file (world_creation.py:187)
    assert int(A['n_rstatic']) == 3


def test_scratcher_composite(sc):
    A, md = sc
    assert A['fb_mass'][0] == pytest.approx(0.11)                    # 0.05 + 0.05 + 0.01 (tool_scratch.urdf)
    c = 0.01 * 0.075 / 0.11                                          # composite COM along the handle x axis
    assert np.allclose(A['task_tool_pivot'], [-c, 0, 0])
    assert np.allclose(A['task_tool_tip'], [0.075 - c, 0, 0])
    tb = int(A['task_tool_body'])
    assert A['body_shape_count'][tb] == 3 and int(A['task_tool_handle_shapes']) == 1
    assert np.all(A['fb_gravity'] == 0)                              # world gravity 0 (scratch_itch.py:259)


def test_scratch_pairs_and_chain(sc):
    A, md = sc
    kinds = A['body_kind']
    tb = int(A['task_tool_body'])
    for a, b in zip(A['pair_a'], A['pair_b']):
        assert not (kinds[a] in (2, 4) and kinds[b] in (2, 4))         # no static-static pairs
        if tb in (a, b):
            o = b if a == tb else a
            if kinds[o] == 0:
                assert not (71 <= 64 + A['body_index'][o] <= 85)       # tool vs links 71..85 off (world_creation.py:357-360)
    assert int(A['hc_n']) == 7 and list(A['hc_joint'][:7]) == list(range(7, 14))
    m = A['hc_mass'][0]
    assert np.allclose(m[[2, 4, 6]], 78.4 * np.array([0.033, 0.019, 0.0065]))   # human_creation.py:213
    assert np.all(m[[0, 1, 3, 5]] == 0)
    # the arm's self-collision partners exclude its own shoulder (human_creation.py:283-285)
    chain_bodies = set(int(b) for b in A['hc_body'] if b >= 0)
    sh = [k for k, l in enumerate(A['human_slot_link']) if l == 6][0]
    sh_body = [b for b in range(len(kinds)) if kinds[b] == 3 and A['body_index'][b] == sh][0]
    for a, b in zip(A['pair_a'], A['pair_b']):
        if a in chain_bodies or b in chain_bodies:
            assert sh_body not in (a, b)


@pytest.mark.skipif(not os.path.isdir(REF), reason='reference assets not mounted (GPU box)')
def test_committed_scratch_scene_matches_compiler():
    import tempfile
    from avr import model_compiler as MC
    with tempfile.TemporaryDirectory() as d:
        path, A = MC.compile_scratch(d)
        committed = np.load(os.path.join(MC.DATA_DIR, 'scratch_itch_pr2.npz'))
        assert set(A) == set(committed.files)
        for k in A:
            assert np.array_equal(np.asarray(A[k]), committed[k]), k


# ----------------------------------------------------------------------------- CPU: reset + oracle glue
def test_reset_states(sc, states):
    from avr import reset_scratch as RSS, geom as G
    A, md = sc
    S, meta = states
    assert np.all(np.isfinite(S))
    nd = md.n_dof
    for k, m in enumerate(meta):
        st = S[k]
        bp = st[SI.S_RBASE:SI.S_RBASE + 3]
        assert -1.25 <= bp[0] <= -0.75 and -0.9 <= bp[1] <= 0.1 and bp[2] == 0     # env.py:507-508 + pos_offset
        assert m['base_ok']
        # tool handle COM on link 76's COM frame (world_creation.py:332-345)
        CP, CQ, _, _ = RSS.arm_fk(A, st[None, :nd], bp[None], st[None, SI.S_RBASE + 3:SI.S_RBASE + 7])
        tb = st[SI.S_FREE:SI.S_FREE + 7]
        handle = G.tf_mul(tb[:3], tb[3:], A['task_tool_pivot'], [0, 0, 0, 1])[0]
        assert np.allclose(handle, CP[0, int(A['task_tool_link'])], atol=1e-9)
        # target on the limb capsule's surface (util.point_on_capsule)
        on = st[SI.S_TASK + SI.T_ONARM:SI.S_TASK + SI.T_ONARM + 3]
        g = 0 if m['gender'] == 'male' else 1
        rad = {9: A['task_limbs'][g][0][2], 11: A['task_limbs'][g][1][2]}[m['limb']]
        assert np.hypot(on[0], on[1]) == pytest.approx(rad)
        # reactive arm motors: gain 0.01, impulse human_strength * dt (world_creation.py:171-179)
        assert np.allclose(st[SI.S_KP + nd:SI.S_KP + nd + 7], 0.01)
        assert np.allclose(st[SI.S_MAXIMP + nd:SI.S_MAXIMP + nd + 7], 0.02 * m['strength'])
        assert st[SI.S_TASK + SI.T_TREMOR] == (m['impairment'] == 'tremor')
        lo = st[SI.S_HCH + 2 * SI.HC_N:SI.S_HCH + 2 * SI.HC_N + 7]
        assert np.allclose(lo, A['hc_lower'][:7] * m['limit_scale'])


def test_oracle_observation_layout(sc, states):
    A, md = sc
    S, meta = states
    o = oracle(md, len(S))
    o.set_state(S)
    obs = o.settle(0)
    assert obs.shape == (len(S), 30)
    assert np.allclose(obs[:, 13:20], S[:, SI.S_Q:SI.S_Q + 7], atol=1e-6)            # left arm q
    assert np.allclose(np.linalg.norm(obs[:, 3:7], axis=1), 1, atol=1e-6)           # tool orientation
    tgt = S[:, SI.S_TASK + SI.T_TARGET:SI.S_TASK + SI.T_TARGET + 3]
    assert np.allclose(obs[:, 0:3] - obs[:, 7:10], obs[:, 10:13] + 0 * tgt, atol=1e-6)   # (tool-torso)-(tool-target) = target-torso
    assert np.all(obs[:, 29] == 0)                                                   # _get_obs([0], ...) at reset


def test_oracle_reward_without_contact(sc, states):
    """No contact: reward = -|target - tool| - 0.01 sum(a^2) - 0.25 |v_tool| (scratch_itch.py:60-72,
    env.py:412-448), with the caller's unclipped action."""
    from avr import geom as G
    A, md = sc
    S, meta = states
    o = oracle(md, len(S))
    o.set_state(S)
    a = np.full((len(S), 7), 1.5, np.float32)
    a[:, ::2] = -2.0
    obs, r, d, info = o.step(a)
    St = o.get_state()
    assert np.all(St[:, SI.S_TASK + SI.T_NCP] == 0)
    tb = St[:, SI.S_FREE:SI.S_FREE + 13]
    for k in range(len(S)):
        Rm = G.quat_to_mat(tb[k, 3:7])
        tip = Rm @ A['task_tool_tip']
        tool = tb[k, :3] + tip
        v = tb[k, 7:10] + np.cross(tb[k, 10:13], tip)
        tgt = St[k, SI.S_TASK + SI.T_TARGET:SI.S_TASK + SI.T_TARGET + 3]
        ref = -np.linalg.norm(tgt - tool) - 0.01 * np.sum(a[k].astype(np.float64) ** 2) - 0.25 * np.linalg.norm(v)
        assert r[k] == pytest.approx(ref, abs=1e-6)
        assert info[k, 0] == 0 and info[k, 1] == 0
    assert np.all(St[:, SI.S_TASK + SI.T_ITER] == 1)


def test_oracle_tremor_targets_alternate(sc):
    import scratch_util as U
    A, md = sc
    S, meta = U.reset_states(A, md, range(4), impairment='tremor')
    o = oracle(md, 4)
    o.set_state(S)
    nd = md.n_dof
    base = S[:, SI.S_HCH:SI.S_HCH + 7]
    trem = S[:, SI.S_HCH + SI.HC_N:SI.S_HCH + SI.HC_N + 7]
    assert np.any(trem != 0)
    for t in range(2):
        o.step(np.zeros((4, 7), np.float32))
        St = o.get_state()
        sg = 1 if t % 2 == 0 else -1                                  # env.py:331
        assert np.allclose(St[:, SI.S_QTGT + nd:SI.S_QTGT + nd + 7], base + sg * trem)
        assert np.allclose(St[:, SI.S_KP + nd:SI.S_KP + nd + 7], 0.05)  # human_gains (scratch_itch.py:45)


def test_oracle_contact_regime_rewards_tool_force(sc, states):
    import scratch_util as U
    A, md = sc
    S, meta = states
    C = U.contact_states(A, md, S, meta)
    o = oracle(md, len(S))
    o.set_state(C)
    obs, r, d, info = o.step(np.zeros((len(S), 7), np.float32))
    St = o.get_state()
    touching = St[:, SI.S_TASK + SI.T_NCP] > 0
    assert touching.sum() >= 2
    assert np.all(info[touching, 0] >= 0) and np.any(info[:, 0] > 0)   # total_force_on_human
    assert np.any(obs[:, 29] > 0)                                        # tool force (obs[-1])
    assert np.all(np.isfinite(r)) and np.all(St[:, SI.S_TASK + SI.T_FLAGS] == 0)


# ----------------------------------------------------------------------------- GPU
def _sim(md, n, **kw):
    from avr import _lib
    return _lib.Sim(md, n, **kw)


@pytest.mark.gpu
def test_scratch_kernel_resources(sc):
    A, md = sc
    sim = _sim(md, 4)
    ki = sim.kernel_info()
    assert all(k['scratch_bytes'] == 0 for k in ki.values())
    assert ki['b']['lds_bytes'] <= 40 * 1024 and ki['pairs']['lds_bytes'] <= 10240
    sim.close()


@pytest.mark.gpu
def test_scratch_one_substep_matches_oracle(sc, states):
    A, md = sc
    S, meta = states
    S32 = S.astype(np.float32)
    n, nd = len(S), md.n_dof + 7
    sim, o = _sim(md, n), oracle(md, n)
    sim.set_state(S32); o.set_state(S32.astype(np.float64))
    sim.substep(0.02); o.substep(0.02)
    G, C = sim.get_state(), o.get_state()
    assert np.abs(G[:, :nd] - C[:, :nd]).max() < 1e-5
    assert np.abs(G[:, SI.S_FREE:SI.S_FREE + 13] - C[:, SI.S_FREE:SI.S_FREE + 13]).max() < 1e-4
    sim.close()


@pytest.mark.gpu
def test_scratch_200_steps_within_1e3(sc, states):
    """Random actions, every impairment: per-DoF |dq| <= 1e-3 rad over 200 gym steps; obs, reward
    and info per step against the oracle."""
    from avr import _lib
    A, md = sc
    S, meta = states
    S32 = S.astype(np.float32)
    n, nd = len(S), md.n_dof + 7
    sim, o = _sim(md, n), oracle(md, n)
    sim.set_state(S32); o.set_state(S32.astype(np.float64))
    assert np.abs(sim.settle(0) - o.settle(0)).max() < 1e-5
    worst = wobs = wrew = wf = 0.0
    for t in range(200):
        a = _lib.random_actions(1001, np.arange(n), t)
        g = sim.step(a)
        c = o.step(a)
        wobs = max(wobs, np.abs(g[0][:, :29] - c[0][:, :29]).max())          # kinematic part of the obs
        wf = max(wf, (np.abs(g[0][:, 29] - c[0][:, 29]) / (1.0 + np.abs(c[0][:, 29]))).max())   # tool force
        wrew = max(wrew, np.abs(g[1] - c[1]).max())
        assert np.array_equal(g[2], c[2])
        assert np.array_equal(g[3][:, 1], c[3][:, 1])
        if t % 20 == 19:
            worst = max(worst, np.abs(sim.get_state()[:, :nd] - o.get_state()[:, :nd]).max())
    assert worst < 1e-3, worst
    assert wobs < 2e-3 and wrew < 2e-3 and wf < 5e-2, (wobs, wrew, wf)
    sim.close()


@pytest.mark.gpu
def test_scratch_contact_regime(sc, states):
    import scratch_util as U
    from avr import _lib
    A, md = sc
    S, meta = states
    C32 = U.contact_states(A, md, S, meta).astype(np.float32)
    n, nd = len(S), md.n_dof + 7
    sim, o32, o64 = _sim(md, n), oracle(md, n, 'f32'), oracle(md, n)
    sim.set_state(C32); o32.set_state(C32.astype(np.float64)); o64.set_state(C32.astype(np.float64))
    w32 = w64 = 0.0
    contacts = 0
    for t in range(10):
        a = _lib.random_actions(1001, np.arange(n), t) * 0.2
        g = sim.step(a)
        o32.step(a)
        c = o64.step(a)
        G = sim.get_state()
        contacts += int(np.count_nonzero(G[:, SI.S_TASK + SI.T_NCP]))
        w32 = max(w32, np.abs(G[:, :nd] - o32.get_state()[:, :nd]).max())
        w64 = max(w64, np.abs(G[:, :nd] - o64.get_state()[:, :nd]).max())
    assert contacts > 0
    assert w32 < 1e-3 and w64 < 5e-3, (w32, w64)
    sim.close()


@pytest.mark.gpu
def test_scratch_state_getters(sc, states):
    """avr_get_q / avr_get_link_pose / avr_get_contact_summary against the state block and FK."""
    import scratch_util as U
    from avr import reset_scratch as RSS
    A, md = sc
    S, meta = states
    C32 = U.contact_states(A, md, S, meta).astype(np.float32)
    n = len(S)
    sim = _sim(md, n)
    sim.set_state(C32)
    sim.step(np.zeros((n, 7), np.float32))
    St = sim.get_state()
    q, qd = sim.get_q()
    nd = sim.n_dof()
    assert nd == 21
    assert np.array_equal(q, St[:, SI.S_Q:SI.S_Q + nd]) and np.array_equal(qd, St[:, SI.S_QD:SI.S_QD + nd])
    link = int(A['task_tool_link'])
    P = sim.get_link_pose(link)
    CP, CQ, _, _ = RSS.arm_fk(A, St[:, :md.n_dof].astype(np.float64), St[:, SI.S_RBASE:SI.S_RBASE + 3].astype(np.float64),
                              St[:, SI.S_RBASE + 3:SI.S_RBASE + 7].astype(np.float64))
    assert np.abs(P[:, :3] - CP[:, link]).max() < 1e-5
    assert np.abs(np.abs(np.sum(P[:, 3:] * CQ[:, link], 1)) - 1).max() < 1e-5
    assert np.allclose(sim.get_link_pose(-1), St[:, SI.S_RBASE:SI.S_RBASE + 7])
    cs = sim.get_contact_summary()
    assert np.array_equal(cs[:, 0], St[:, SI.S_TASK + SI.T_NCP])
    imp = np.zeros(n)
    for e in range(n):
        k = int(St[e, SI.S_TASK + SI.T_NCP])
        imp[e] = St[e, SI.S_CP + ABI.CP_IMP:SI.S_CP + ABI.CP_WORDS * k:ABI.CP_WORDS].sum() / 0.02
    assert np.allclose(cs[:, 1], imp, rtol=1e-5, atol=1e-5)
    with pytest.raises(RuntimeError):
        sim.get_link_pose(99)
    sim.close()


@pytest.mark.gpu
def test_scratch_part_b_row_paths_bit_identical(sc, states):
    """Part B of the PR2 tasks stages every row -- the non-contact rows with their 21-DoF robot
    parts as well as the contact rows -- in LDS when a block's four envs fit, and reads them from
    global memory otherwise (AVR_B4_GLOBAL=1 forces that for every block): the same rows in the
    same order with the same arithmetic, so both agree bit for bit, with and without contacts."""
    import scratch_util as U
    from avr import _lib
    A, md = sc
    S, meta = states
    C32 = U.contact_states(A, md, S, meta).astype(np.float32)
    X = np.concatenate([S.astype(np.float32), C32])
    outs = []
    for g in ('0', '1'):
        old = os.environ.pop('AVR_B4_GLOBAL', None)
        os.environ['AVR_B4_GLOBAL'] = g
        try:
            sim = _sim(md, len(X))
        finally:
            os.environ.pop('AVR_B4_GLOBAL')
            if old is not None:
                os.environ['AVR_B4_GLOBAL'] = old
        sim.set_state(X)
        steps = [sim.step(_lib.random_actions(1001, np.arange(len(X)), t) * 0.5) for t in range(5)]
        outs.append((sim.get_state(), steps))
        sim.close()
    (G0, s0), (G1, s1) = outs
    assert np.array_equal(G0, G1)
    for a, b in zip(s0, s1):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert np.count_nonzero(G0[:, SI.S_TASK + SI.T_NCP]) > 0
