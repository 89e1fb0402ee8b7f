"""The PR2 tasks (ScratchItchPR2-v0 = BASELINE configs[2]; BedBathingPR2-v0, the PR2 variant of
configs[3]) at the bench's launch shape and over contact horizons, against the CPU oracle.

  * launch shape: 4096 envs in four concurrent env groups with graph replay -- the shape bench.py
    times -- from a pool of reset states and contact states (the scratcher pressed onto the arm /
    the cloth pressed onto a wipe target), tiled; 32 sampled envs (every group, part-B block
    boundaries included) against the fp64 oracle over 5 gym steps: joint angles, observations,
    rewards, done and the task bookkeeping (success counts, wipe bits) per step;
  * contact regime: 512 envs x 200 gym steps starting in contact, small random actions (x 0.2,
    so the tool stays on the person), GPU vs the fp64 oracle.  Contact trajectories diverge at
    the rounding level (chaos), so the episode outcomes are compared statistically, as FeedingJaco's
    (test_gpu_parity.py): mean episode reward, scratches / wiped targets (the task_success
    counters, scratch_itch.py:66-70 and bed_bathing.py:97-125) and contact-step counts, each as a
    paired difference within three standard errors.
"""
import numpy as np
import pytest

from avr import _abi as ABI
from ensemble_util import ensembles, launch_shape_verdict

pytestmark = pytest.mark.gpu

SI, BB = ABI.SI, ABI.BB


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


def _picks(n_pool, n_first_contact):
    """32 picks of the 4096-env launch (env e holds pool state e mod n_pool): every env group's
    first and last env, part-B block boundaries, and one env of every contact state spread over
    the four groups; the rest of the 32 from further contact envs."""
    reset = [0, 1024, 2048, 3072]
    contact = [n_first_contact + k + n_pool * (8 * k + 3) for k in range(n_pool - n_first_contact)]
    ends = [1023, 2047, 3071, 4095]
    P = sorted(set(reset + contact + ends))
    extra = (n_first_contact + k % (n_pool - n_first_contact) + n_pool * (5 * k + 1) for k in range(10 ** 4))
    for e in extra:
        if len(P) >= 32:
            break
        if e < 4096 and e not in P:
            P = sorted(P + [e])
    P = np.array(P[:32])
    assert len(P) == 32 and P.max() < 4096
    return P


def _perturbed(S, L, nd, rng, eps):
    """S with the joint angles and the tool's position moved by eps N(0, 1): rounding-level
    perturbations that show how far fp32 rounding alone can carry a state in a few steps."""
    X = S.astype(np.float64).copy()
    X[:, L.S_Q:L.S_Q + nd] += eps * rng.standard_normal((len(X), nd))
    X[:, L.S_FREE:L.S_FREE + 3] += eps * rng.standard_normal((len(X), 3))
    return X


@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH], ids=['ScratchItchPR2', 'BedBathingPR2'])
def test_launch_shape_sampled_envs_match_oracle(task):
    """32 sampled envs of the bench's launch against the fp64 oracle over 5 gym steps.  The GPU is
    one fp32 realisation of each env.  Two 16-member oracle ensembles started from rounding-level
    perturbations of the same states (1e-6 on the joint angles and the tool position) say what
    each pick is: the fp64 ensemble whether the physics amplifies such a perturbation (a contact
    bifurcation: the pick is chaotic), the fp32 ensemble -- the kernel's own arithmetic, the lane
    GJK's stall rule included -- how far fp32 rounding carries it.  Calm picks are held to the
    one-step tolerances (1e-3 rad, obs / reward 2e-3, force 5e-2); chaotic picks to twice the larger
    ensemble deviation; the task bookkeeping must be exact wherever both ensembles keep it exact.
    No pick is excepted."""
    from avr import _lib
    A, md, L, P, is_c = _pool(task, 16)
    E = 4096
    n_pool, n_first_contact = len(P), int(np.argmax(is_c))
    PICK = _picks(n_pool, n_first_contact)
    S = np.tile(P, (E // n_pool + 1, 1))[:E]
    n = len(PICK)
    n_contact_picks = int(is_c[PICK % n_pool].sum())
    nd = md.n_dof + (int(A['hc_n']) if task == ABI.TASK_SCRATCH else 0)

    def book(X, info, C, ic):       # the task bookkeeping: task_success, the success counter, (BedBathing) wipe bits
        b = [info[:, 1] == ic[:, 1], X[:, L.S_TASK + L.T_SUCCESS] == C[:, L.S_TASK + L.T_SUCCESS]]
        if task == ABI.TASK_BEDBATH:
            b.append(np.all(_wipe_bits(X, L) == _wipe_bits(C, L), axis=1))
        return np.all(b, axis=0)

    acts = lambda t: _lib.random_actions(1001, np.arange(E), t)[PICK] * 0.2
    dev, ens_same, traj = ensembles(md, S[PICK], L, nd, lambda X, rng: _perturbed(X, L, nd, rng, 1e-6), 5, acts, book)
    sim = _lib.Sim(md, E)
    assert sim.env_groups() == 4
    sim.set_state(S)
    od = L.OBS_DIM - 1                     # the kinematic part of the obs (the last word is the tool force)
    keys = ('dq', 'obs', 'rew', 'force')
    w = {k: np.zeros(n) for k in keys}     # GPU vs fp64
    same = np.ones(n, bool)
    both_same = ens_same['f32'] & ens_same['f64']
    ncp = 0
    for t in range(5):
        a = _lib.random_actions(1001, np.arange(E), t) * 0.2
        ob, r, d, i = sim.step(a)
        oc, rc, dc, ic, C = traj[t]
        G = sim.get_state()[PICK]
        w['dq'] = np.maximum(w['dq'], np.abs(G[:, :nd] - C[:, :nd]).max(1))
        w['obs'] = np.maximum(w['obs'], np.abs(ob[PICK, :od] - oc[:, :od]).max(1))
        w['rew'] = np.maximum(w['rew'], np.abs(r[PICK] - rc) / (1.0 + np.abs(rc)))
        w['force'] = np.maximum(w['force'], np.abs(ob[PICK, od] - oc[:, od]) / (1.0 + np.abs(oc[:, od])))
        assert np.array_equal(d[PICK], dc)
        # exact bookkeeping wherever both ensembles keep it exact (a scratch or a wiped target at a
        # force threshold flips with the rounding: there the ensembles show it too)
        same &= ~both_same | book(G.astype(np.float64), i[PICK], C, ic)
        ncp += int(np.count_nonzero(G[:, L.S_TASK + L.T_NCP]))
    sim.close()
    tol = dict(dq=1e-3, obs=2e-3, rew=2e-3, force=5e-2)
    ok, chaotic, bound = launch_shape_verdict(w, dev, tol, n // 2)
    ok &= same
    print('launch shape', task, 'picks', n, 'contact picks', n_contact_picks, 'contact env-steps', ncp)
    print('  chaotic picks (fp64 ensemble >= 5e-4 rad): (pick, fp64 ens, fp32 ens, GPU) dq',
          [(int(PICK[k]), float(dev['f64']['dq'][k]), float(dev['f32']['dq'][k]), float(w['dq'][k])) for k in np.nonzero(chaotic)[0]])
    print('  calm picks: max GPU dev', {k: float(w[k][~chaotic].max()) for k in keys},
          'max fp32 ensemble dev', {k: float(dev['f32'][k][~chaotic].max()) for k in keys},
          'max fp64 ensemble dev', {k: float(dev['f64'][k][~chaotic].max()) for k in keys})
    print('  per pick (pick, GPU dq, fp32 ens dq, fp64 ens dq):',
          [(int(PICK[k]), float('%.3g' % w['dq'][k]), float('%.3g' % dev['f32']['dq'][k]), float('%.3g' % dev['f64']['dq'][k])) for k in range(n)])
    print('  failing picks', [(int(PICK[k]), bool(same[k]), {q: (float(w[q][k]), float(bound[q][k])) for q in keys}) for k in np.nonzero(~ok)[0]],
          'picks whose bookkeeping an ensemble flips', [int(PICK[k]) for k in np.nonzero(~both_same)[0]])
    assert n_contact_picks >= 16 and ncp >= 60, (n_contact_picks, ncp)
    assert ok.all()


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
    """512 envs x 200 gym steps from the contact states (distinct action streams per env) on the GPU
    and on the fp32 and fp64 oracles.  Contact trajectories part at the rounding level (chaos), so
    episode outcomes are compared as paired statistics: the mean episode reward, the scratch / wipe
    counter (task_success before the threshold, scratch_itch.py:66-70, bed_bathing.py:97-125) and
    the contact-step count, each within three standard errors of the paired differences plus the
    fp32 oracle's own mean difference from fp64, against both oracles.  Precision is not neutral
    here: BedBathing's fp32 oracle wipes ~2 % more targets than its fp64 build, mostly through fp32
    GJK stops on thin hull-capsule simplices that the kernel hands to its double GJK (gjk_lane), so
    the GPU may sit anywhere between the two oracles (measured: at the fp64 oracle)."""
    from avr import _lib
    A, md, L, P, is_c = _pool(task, 16)
    C = P[is_c]
    n = 512
    S = np.tile(C, (n // len(C) + 1, 1))[:n]
    ids = np.arange(n)
    sim = _lib.Sim(md, n)
    sim.set_state(S)
    o = _oracle(md, n, 'f64')
    o.set_state(S.astype(np.float64))
    o32 = _oracle(md, n, 'f32')
    o32.set_state(S.astype(np.float64))
    Rg, Kg, G, ig = _episode(task, sim, L, ids, 200, True)
    Rc, Kc, Cs, ic = _episode(task, o, L, ids, 200, False)
    R3, K3, C3, i3 = _episode(task, o32, L, ids, 200, False)
    sim.close()
    sg, sc, s3 = (X[:, L.S_TASK + L.T_SUCCESS].astype(np.float64) for X in (G, Cs, C3))

    def paired(a, b):
        d = a - b
        return d.mean(), d.std(ddof=1) / np.sqrt(len(d))
    print('contact regime', task, 'reward mean gpu %.4f fp32 %.4f fp64 %.4f' % (Rg.mean(), R3.mean(), Rc.mean()),
          'success counter %.3f %.3f %.3f' % (sg.mean(), s3.mean(), sc.mean()), 'contact steps %.2f %.2f %.2f' % (Kg.mean(), K3.mean(), Kc.mean()))
    assert np.all(np.isfinite(Rg)) and np.all(G[:, L.S_TASK + L.T_FLAGS].astype(np.int64) & 0x1f == 0)
    assert Kg.mean() > 5 and Kc.mean() > 5            # the episodes do run in contact
    assert sc.mean() > 0.05                           # and score (scratches / wiped targets)
    for name, g, c64, c32 in (('reward', Rg, Rc, R3), ('success', sg, sc, s3), ('contact steps', Kg, Kc, K3)):
        d32, se32 = paired(g, c32)
        d64, se64 = paired(g, c64)
        p, _ = paired(c32, c64)
        print('  %s: gpu - fp32 %.4f (se %.4f), gpu - fp64 %.4f (se %.4f), fp32 - fp64 %.4f' % (name, d32, se32, d64, se64, p))
        assert abs(d32) <= 3 * se32 + abs(p) + 1e-9, (name, d32, se32, p)
        assert abs(d64) <= 3 * se64 + abs(p) + 1e-9, (name, d64, se64, p)
