"""Rounding-level ensembles of the CPU oracle for the launch-shape parity tests
(test_pr2_launch_shape.py, test_gpu_parity.py): which sampled envs sit at a contact bifurcation
(the fp64 oracle itself amplifies a 1e-6 perturbation) and how far the kernel's fp32 arithmetic
alone carries each env (the fp32 oracle, which restates the kernel's GJK stall rule)."""
import numpy as np


def _oracle(md, n, precision):
    from oracle.oracle import Oracle
    o = Oracle(md, n, precision)
    o.set_threads(8)
    return o


def ensembles(md, S0, L, nd, perturb, steps, actions, book, members=16, settle=0, seed=9):
    """fp32 and fp64 oracle ensembles of the picks S0 (members 1.. started from rounding-level
    perturbations: perturb(S, rng)), `settle` frames, then `steps` gym steps of actions(t).  Returns
    per precision the largest deviation from the unperturbed fp64 oracle per pick over the steps --
    dq (joint angles), obs (kinematic part), rew (relative), force (relative) -- and whether the
    whole ensemble kept the bookkeeping of the fp64 oracle (book(X, info, C, ic)); plus the fp64
    oracle's own trajectory [(obs, rew, done, info, state)] per step.  The fp32 ensemble is the
    kernel's arithmetic (the oracle restates the lane GJK's stall rule and double rerun); the fp64
    ensemble says whether the physics itself amplifies a 1e-6 perturbation (a contact bifurcation)."""
    n = len(S0)
    rng = np.random.default_rng(seed)
    o = _oracle(md, n, 'f64')
    o.set_state(S0.astype(np.float64))
    o.settle(settle)
    ens = {}
    for prec in ('f32', 'f64'):
        e = _oracle(md, n * members, prec)
        X = np.concatenate([S0.astype(np.float64) if (j == 0 and prec == 'f32') else perturb(S0, rng) for j in range(members)])
        e.set_state(X)
        e.settle(settle)
        ens[prec] = e
    keys = ('dq', 'obs', 'rew', 'force')
    dev = {p: {k: np.zeros(n) for k in keys} for p in ens}
    same = {p: np.ones(n, bool) for p in ens}
    od = L.OBS_DIM - 1
    traj = []
    for t in range(steps):
        a = actions(t)
        oc, rc, dc, ic = o.step(a)
        C = o.get_state()
        traj.append((oc, rc, dc, ic, C))
        for p, e in ens.items():
            eo, er, _, ei = e.step(np.tile(a, (members, 1)))
            X = e.get_state()
            for j in range(members):
                sl = slice(j * n, (j + 1) * n)
                d = dev[p]
                d['dq'] = np.maximum(d['dq'], np.abs(X[sl, :nd] - C[:, :nd]).max(1))
                d['obs'] = np.maximum(d['obs'], np.abs(eo[sl, :od] - oc[:, :od]).max(1))
                d['rew'] = np.maximum(d['rew'], np.abs(er[sl] - rc) / (1.0 + np.abs(rc)))
                d['force'] = np.maximum(d['force'], np.abs(eo[sl, od] - oc[:, od]) / (1.0 + np.abs(oc[:, od])))
                if book is not None:
                    same[p] &= book(X[sl], ei[sl], C, ic)
    return dev, same, traj


def launch_shape_verdict(w, dev, tol, n_chaotic_max):
    """A pick is chaotic only if the fp64 ensemble itself moves by >= half the joint tolerance: the
    physics amplifies a 1e-6 perturbation.  Calm picks are held to the one-step tolerances; chaotic
    picks to twice the larger of the two ensembles' deviations from the unperturbed fp64 oracle.
    Returns (ok per pick, chaotic per pick, bound)."""
    keys = tuple(tol)
    chaotic = dev['f64']['dq'] >= 0.5 * tol['dq']
    bound = {k: np.where(chaotic, np.maximum(tol[k], 2.0 * np.maximum(dev['f32'][k], dev['f64'][k])), tol[k]) for k in keys}
    ok = np.all([w[k] <= bound[k] for k in keys], axis=0)
    assert chaotic.sum() <= n_chaotic_max, 'the fp64 ensemble calls too many picks chaotic: %d' % chaotic.sum()
    return ok, chaotic, bound
