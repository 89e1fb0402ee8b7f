"""The PR2 outside the left arm's subtree (base casters, torso, head, laser, right arm) is held at
its reset pose.  The reference simulates those 37 joints with PyBullet's default
velocity motors (world_creation.py:187 loads the PR2 with every joint motorised at target
velocity 0, max impulse `default_motor_impulse` per sub-step) in zero gravity
(scratch_itch.py:259, bed_bathing.py:344), so a joint stays at rest exactly as long as the contact
load on it stays within that motor's limit: with every joint of the fixed-base chain at rest, the
static joint impulses that hold a contact impulse f at x are tau_j = a_j . ((x - o_j) x f) on the
revolute ancestors and a_j . f on the prismatic ones, and the solver's motor rows reach them.

This test measures that load on the oracle (the fp64 CPU restatement the kernels are checked
against) over full-amplitude random actions, from reset states and from contact states (tool
pressed on the arm / cloth pressed on a wipe target): every contact point on the robot-fixed
geometry, sampled at the end of each gym step (the manifold's last sub-step), bounded with its
friction and torsional parts at their limits (|f_t| <= sqrt(2) mu lambda, torsion <= coefficient x
lambda).  The bound must stay below the motor limit with a margin, i.e. holding these joints
still is what the reference's motors do on these rollouts.
"""
import numpy as np
import pytest

from avr import _abi as ABI
from avr import geom as G

SI, BB = ABI.SI, ABI.BB
J_REVOLUTE, J_PRISMATIC = 1, 2


def _pool(task, n_reset):
    if task == ABI.TASK_SCRATCH:
        import scratch_util as U
        A, md = U.scene()
        S, meta = U.reset_states(A, md, range(n_reset))
        return A, md, SI, np.concatenate([S, U.contact_states(A, md, S, meta)])
    import bedbath_util as U
    from avr import reset_bedbath as RBB
    from oracle.oracle import Oracle
    A = ABI.load_scene(ABI.TASK_BEDBATH)
    md = ABI.ModelDesc(A)

    def run(S, frames):                  # the reset's arm settle on the oracle (no GPU here)
        o = Oracle(md, len(S))
        o.set_state(S)
        o.settle(frames)
        return o.get_state()
    settled = RBB.settled_arms(A, md, runner=run)
    S, _ = RBB.batch_reset_states(A, md, 1001, list(range(n_reset)), attempts=12, iters=80, settled=settled)
    C, _ = U.wipe_states(A, md, S, strict=False)
    return A, md, BB, np.concatenate([S, C])


def frozen_joint_load(A, L, St, links=None):
    """Largest bound on a frozen PR2 joint's holding impulse over the contact points of states St
    (n, words): (max over joints and envs, per-env max, number of contact points on the fixed
    geometry); links: a dict counting those points per URDF link."""
    par, jt, jo, ja = A['pr2_parent'], A['pr2_jtype'], A['pr2_jorigin'], A['pr2_jaxis']
    sb, kind, link = A['shape_body'], A['body_kind'], A['shape_urdf_link']
    fric, roll, spin = A['body_friction'], A['body_rolling'], A['body_spinning']
    per_env = np.zeros(len(St))
    n_pts = 0
    for e, st in enumerate(St):
        bq = st[L.S_RBASE + 3:L.S_RBASE + 7]
        for c in range(L.MAX_CONTACTS):
            cp = st[L.S_CP + ABI.CP_WORDS * c:L.S_CP + ABI.CP_WORDS * (c + 1)]
            lam = float(cp[ABI.CP_IMP])
            if cp[ABI.CP_LIFE] <= 0 or lam <= 0:
                continue
            sa_, sb_ = int(cp[ABI.CP_SA]), int(cp[ABI.CP_SB])
            ba, bb = sb[sa_], sb[sb_]
            if kind[ba] != 4:                  # KIND_RSTATIC is always body A of its pairs
                assert kind[bb] != 4
                continue
            n_pts += 1
            if links is not None:
                links[int(link[sa_])] = links.get(int(link[sa_]), 0) + 1
            x = cp[ABI.CP_LA:ABI.CP_LA + 3]                     # base_footprint frame
            n = G.quat_rotate(G.quat_conj(bq), cp[ABI.CP_N:ABI.CP_N + 3])
            mu = min(fric[ba] * fric[bb], 10.0)
            tors = min(roll[ba] * fric[bb] + roll[bb] * fric[ba], 10.0)
            tors = np.hypot(min(spin[ba] * fric[bb] + spin[bb] * fric[ba], 10.0), np.sqrt(2) * tors)
            j = int(link[sa_])
            while j >= 0:
                a = ja[j]
                if jt[j] == J_REVOLUTE:
                    r = x - jo[j]
                    t = abs(a @ np.cross(r, n)) + np.sqrt(2) * mu * np.linalg.norm(np.cross(a, r)) + tors
                elif jt[j] == J_PRISMATIC:
                    t = abs(a @ n) + np.sqrt(2) * mu
                else:
                    t = 0.0
                per_env[e] = max(per_env[e], t * lam)
                j = int(par[j])
    return float(per_env.max(initial=0.0)), per_env, n_pts


def test_frozen_joint_table_matches_the_scene():
    for task in (ABI.TASK_SCRATCH, ABI.TASK_BEDBATH):
        A = ABI.load_scene(task)
        jt = A['pr2_jtype']
        # 37 motorised joints outside the left arm's subtree (the right arm's 7 arm joints among them)
        assert (jt > 0).sum() >= 30 and np.all(jt[[42, 43, 44, 46, 47, 49, 50]] == J_REVOLUTE)
        assert np.all(jt[64:86] == 0)                                   # left subtree: simulated
        rs = np.nonzero(A['body_kind'][A['shape_body']] == 4)[0]
        assert len(rs) and np.all(A['shape_urdf_link'][rs] >= 0)
        assert np.all(A['shape_urdf_link'][A['body_kind'][A['shape_body']] != 4] == -1)
        assert np.allclose(np.linalg.norm(A['pr2_jaxis'][jt > 0], axis=1), 1.0)


@pytest.mark.parametrize('task', [ABI.TASK_SCRATCH, ABI.TASK_BEDBATH], ids=['ScratchItchPR2', 'BedBathingPR2'])
def test_frozen_branches_stay_within_default_motor_limit(task):
    from oracle.oracle import Oracle
    A, md, L, P = _pool(task, 8)
    n = 48
    S = np.tile(P, (n // len(P) + 1, 1))[:n].astype(np.float64)
    o = Oracle(md, n, 'f64')
    o.set_threads(8)
    o.set_state(S)
    rng = np.random.default_rng(5)
    worst, pts, loaded, links = 0.0, 0, 0, {}
    T = 200                                 # one episode (scratch_itch.py / bed_bathing.py: 200 steps)
    for t in range(T):
        if t % 10 == 0:                     # held for 10 steps: the arm sweeps its workspace
            a = rng.uniform(-1, 1, (n, 7)).astype(np.float32)
        o.step(a)
        w, pe, k = frozen_joint_load(A, L, o.get_state(), links)
        worst = max(worst, w)
        pts += k
        loaded += int((pe > 0).sum())
    cap = md.params['default_motor_impulse']
    print('frozen PR2 branches', task, 'contact points on the fixed geometry', pts, 'by URDF link', links,
          'env-steps loading a frozen joint', loaded, 'of', n * T, 'max holding impulse bound %.4g (motor limit %g)' % (worst, cap))
    assert worst < 0.5 * cap
