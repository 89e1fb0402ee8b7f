"""The PR2 tasks (ScratchItchPR2-v0 = BASELINE configs[2]; BedBathingPR2-v0, the PR2 variant of
configs[3]) at the bench's launch shape and over contact horizons, against the CPU oracle.

  * launch shape: 4096 envs in four concurrent env groups with graph replay -- the shape bench.py
    times -- from a pool of reset states and contact states (the scratcher pressed onto the arm /
    the cloth pressed onto a wipe target), tiled; 32 sampled envs (every group, part-B block
    boundaries included) against the fp64 oracle over 5 gym steps: joint angles, observations,
    rewards, done and the task bookkeeping (success counts, wipe bits) per step;
  * contact regime: 128 envs x 200 gym steps starting in contact, small random actions (x 0.2,
    so the tool stays on the person), GPU vs the fp64 oracle.  Contact trajectories diverge at
    the rounding level (chaos), so the episode outcomes are compared statistically, as FeedingJaco's
    (test_gpu_parity.py): mean episode reward (paired difference within 3 standard errors +
    tolerance), scratches / wiped targets (task_success counters, scratch_itch.py:66-70 and
    bed_bathing.py:97-125), contact-step counts and the final task_success flags.
"""
import numpy as np
import pytest

from avr import _abi as ABI

pytestmark = pytest.mark.gpu

SI, BB = ABI.SI, ABI.BB
PICK = np.array([0, 1, 31, 32, 33, 511, 512, 1023, 1024, 1025, 1055, 1056, 1500, 2047, 2048, 2049, 2079, 2080,
                 2500, 3071, 3072, 3073, 3103, 3104, 3500, 3800, 4000, 4063, 4064, 4090, 4094, 4095])


def _oracle(md, n, precision):
    from oracle.oracle import Oracle
    o = Oracle(md, n, precision)
    o.set_threads(8)
    return o


def _pool(task, n_reset):
    """(A, md, L, pool of reset + contact states (float32), is-contact mask)."""
    if task == ABI.TASK_SCRATCH:
        import scratch_util as U
        A, md = U.scene()
        S, meta = U.reset_states(A, md, range(n_reset))
        C = U.contact_states(A, md, S, meta)
        L = SI
    else:
        import bedbath_util as U
        from avr import reset_bedbath as RBB
        A = ABI.load_scene(ABI.TASK_BEDBATH)
        md = ABI.ModelDesc(A)
        S, meta = RBB.batch_reset_states(A, md, 1001, list(range(n_reset)), attempts=12, iters=80)
        C, _ = U.wipe_states(A, md, S, strict=False)
        L = BB
    P = np.concatenate([S, C]).astype(np.float32)
    return A, md, L, P, np.r_[np.zeros(len(S), bool), np.ones(len(C), bool)]


def _wipe_bits(St, L):
    return St[:, L.S_TASK + L.T_WIPE:L.S_TASK + L.T_WIPE + 6]


@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH], ids=['ScratchItchPR2', 'BedBathingPR2'])
def test_launch_shape_sampled_envs_match_oracle(task):
    from avr import _lib
    A, md, L, P, _ = _pool(task, 16)
    E = 4096
    P = P[:31] if len(P) % 2 == 0 else P    # (an odd pool: the picks at block boundaries see different states)
    S = np.tile(P, (E // len(P) + 1, 1))[:E]
    sim = _lib.Sim(md, E)
    assert sim.env_groups() == 4
    sim.set_state(S)
    o, op = _oracle(md, len(PICK), 'f64'), _oracle(md, len(PICK), 'f64')
    o.set_state(S[PICK].astype(np.float64)); op.set_state(S[PICK].astype(np.float64))
    nd = md.n_dof + (int(A['hc_n']) if task == ABI.TASK_SCRATCH else 0)
    od = L.OBS_DIM - 1                     # the kinematic part of the obs (the last word is the tool force)
    n = len(PICK)
    w = dict(dq=np.zeros(n), obs=np.zeros(n), rew=np.zeros(n), force=np.zeros(n))
    spread = np.zeros(n)
    same = np.ones(n, bool)
    ncp = 0
    rng = np.random.default_rng(9)
    for t in range(5):
        a = _lib.random_actions(1001, np.arange(E), t) * 0.2
        ob, r, d, i = sim.step(a)
        oc, rc, dc, ic = o.step(a[PICK])
        op.step((a[PICK] + 1e-4 * rng.standard_normal((n, a.shape[1]))).astype(np.float32))
        G, C = sim.get_state()[PICK], o.get_state()
        w['dq'] = np.maximum(w['dq'], np.abs(G[:, :nd] - C[:, :nd]).max(1))
        w['obs'] = np.maximum(w['obs'], np.abs(ob[PICK, :od] - oc[:, :od]).max(1))
        w['rew'] = np.maximum(w['rew'], np.abs(r[PICK] - rc) / (1.0 + np.abs(rc)))
        w['force'] = np.maximum(w['force'], np.abs(ob[PICK, od] - oc[:, od]) / (1.0 + np.abs(oc[:, od])))
        spread = np.maximum(spread, np.abs(op.get_state()[:, :nd] - C[:, :nd]).max(1))
        assert np.array_equal(d[PICK], dc)
        same &= i[PICK, 1] == ic[:, 1]                                            # task_success
        same &= G[:, L.S_TASK + L.T_SUCCESS] == C[:, L.S_TASK + L.T_SUCCESS].astype(np.float32)
        if task == ABI.TASK_BEDBATH:
            same &= np.all(_wipe_bits(G, L) == _wipe_bits(C, L).astype(np.float32), axis=1)
        ncp += int(np.count_nonzero(G[:, L.S_TASK + L.T_NCP]))
    sim.close()
    # a pick whose own oracle moves by more than 1e-3 under a 1e-4 perturbation of its actions sits
    # at a contact bifurcation (e.g. the scratcher pressed hard into the arm: a wrist joint ends at
    # 0.86 or 0.36 rad depending on the fifth decimal of the action); the rest are held to the
    # one-step tolerances, up to two picks: the fp32 GJK / EPA misses ~1 % of penetrating
    # box-capsule queries (test_narrowphase_pairs.py), and a contact pick makes tens per step
    calm = spread < 1e-3
    ok = same & (w['dq'] < 1e-3) & (w['obs'] < 2e-3) & (w['rew'] < 2e-3) & (w['force'] < 5e-2)
    print('launch shape', task, {k: float(v[calm & ok].max()) for k, v in w.items()}, 'sensitive picks', int((~calm).sum()),
          'calm picks off', [(int(PICK[k]), float(w['dq'][k])) for k in np.nonzero(calm & ~ok)[0]], 'contact env-steps', ncp)
    assert ncp > 0 and calm.sum() >= n // 2, spread
    assert (calm & ~ok).sum() <= 2, w


def _episode(task, sim_or_oracle, L, ids, steps, gpu):
    from avr import _lib
    n = len(ids)
    R = np.zeros(n)
    contact_steps = np.zeros(n)
    for t in range(steps):
        a = _lib.random_actions(1001, ids, t) * 0.2
        ob, r, d, i = sim_or_oracle.step(a)
        R += r
        contact_steps += ob[:, L.OBS_DIM - 1] > 0          # tool force in the obs (scratch_itch.py:108, bed_bathing.py:133)
    St = sim_or_oracle.get_state()
    return R, contact_steps, St, i


@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH], ids=['ScratchItchPR2', 'BedBathingPR2'])
def test_contact_regime_episode_statistics_vs_fp64_oracle(task):
    from avr import _lib
    A, md, L, P, is_c = _pool(task, 16)
    C = P[is_c]
    n = 128
    S = np.tile(C, (n // len(C) + 1, 1))[:n]        # distinct action streams per env id
    ids = np.arange(n)
    sim = _lib.Sim(md, n)
    sim.set_state(S)
    o = _oracle(md, n, 'f64')
    o.set_state(S.astype(np.float64))
    Rg, Kg, G, ig = _episode(task, sim, L, ids, 200, True)
    Rc, Kc, Cs, ic = _episode(task, o, L, ids, 200, False)
    sim.close()
    d = Rg - Rc
    se = d.std(ddof=1) / np.sqrt(n)
    sg, sc = G[:, L.S_TASK + L.T_SUCCESS], Cs[:, L.S_TASK + L.T_SUCCESS]
    print('contact regime', task, 'reward mean gpu %.4f oracle %.4f diff %.4f se %.4f' % (Rg.mean(), Rc.mean(), d.mean(), se),
          'success mean %.3f %.3f' % (sg.mean(), sc.mean()), 'contact steps %.2f %.2f' % (Kg.mean(), Kc.mean()),
          'task_success %.3f %.3f' % (ig[:, 1].mean(), ic[:, 1].mean()))
    assert np.all(np.isfinite(Rg)) and np.all(G[:, L.S_TASK + L.T_FLAGS].astype(np.int64) & 0x1f == 0)
    assert Kg.mean() > 5 and Kc.mean() > 5            # the episodes do run in contact
    assert abs(d.mean()) < 3 * se + 0.05 * abs(Rc.mean()) + 0.5, (d.mean(), se)
    assert abs(sg.mean() - sc.mean()) <= 0.1 * max(sc.mean(), 1.0) + 0.5, (sg.mean(), sc.mean())
    assert abs(Kg.mean() - Kc.mean()) <= 0.1 * Kc.mean() + 2.0, (Kg.mean(), Kc.mean())
    assert abs(ig[:, 1].mean() - ic[:, 1].mean()) <= 0.1
