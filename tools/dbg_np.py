"""Narrowphase pair check (GPU avr_narrowphase_query vs the oracle's, f64 and f32) on perturbed
poses of one shape pair taken from a saved state; reports normal / depth disagreements and, for
the worst, the true penetration from a direction search on the support functions."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'assistive-vr-gym_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
from avr import _abi as ABI, geom as G
from oracle.oracle import Oracle

np.set_printoptions(precision=5, suppress=True, linewidth=200)
task = int(os.environ.get('TASK', 1))
A = ABI.load_scene(task)
md = ABI.ModelDesc(A)
L = ABI.SI if task == 1 else ABI.BB
st = np.load(os.environ.get('STATE', 'gpurun_out/dbg_state_t1_k28_n2.npy'))[0].astype(np.float64)
sa, sb = int(os.environ.get('SA', 49)), int(os.environ.get('SB', 166))
N = int(os.environ.get('N', 512))


def body_pose(b):
    k, i = A['body_kind'][b], A['body_index'][b]
    if k == 1: return st[L.S_FREE + 13 * i:L.S_FREE + 13 * i + 7]
    if k == 3: return st[L.S_HUMAN + 7 * i:L.S_HUMAN + 7 * i + 7]
    raise ValueError(k)


pa0, pb = body_pose(A['shape_body'][sa]), body_pose(A['shape_body'][sb])
rng = np.random.default_rng(1)
X = np.zeros((N, 14))
for k in range(N):
    s = 0 if k == 0 else 1
    dp = s * rng.uniform(-0.015, 0.015, 3)
    ax = rng.standard_normal(3); ax /= np.linalg.norm(ax)
    dq = G.quat_axis_angle(ax, s * rng.uniform(-0.1, 0.1))
    X[k, :3] = pa0[:3] + dp
    X[k, 3:7] = G.quat_mul(dq, pa0[3:])
    X[k, 7:] = pb
pairs = np.tile([sa, sb], (N, 1))
res = {}
for prec in ('f64', 'f32'):
    o = Oracle(md, 1, prec)
    R = np.zeros((N, 8))
    for k in range(N):
        r, out = o.narrowphase(sa, X[k, :7], sb, X[k, 7:], 0.02)
        R[k, 0] = r; R[k, 1:] = out
    res[prec] = R
if os.environ.get('NOGPU'):
    res['gpu'] = res['f32']
else:
    from avr import _lib
    sim = _lib.Sim(md, 1)
    res['gpu'] = sim.narrowphase(pairs, X).astype(np.float64)
    sim.close()


def ang(a, b):
    return np.degrees(np.arccos(np.clip((a * b).sum(1), -1, 1)))


pen = res['f64'][:, 7] < 0
for name in ('gpu', 'f32'):
    R = res[name]
    both = (R[:, 0] == 1) & (res['f64'][:, 0] == 1)
    a = ang(R[:, 1:4], res['f64'][:, 1:4])
    dd = np.abs(R[:, 7] - res['f64'][:, 7])
    print(name, 'vs f64: contact agree', float(np.mean((R[:, 0] > 0) == (res['f64'][:, 0] > 0))),
          'penetrating', int(pen.sum()), 'normal > 2 deg', int((a[both] > 2).sum()), 'depth diff > 1e-4', int((dd[both] > 1e-4).sum()),
          'worst angle', float(a[both].max()) if both.any() else 0)
    bad = np.nonzero(both & ((a > 2) | (dd > 1e-4)))[0][:5]
    for k in bad:
        print('   pose', k, name, R[k, [0, 1, 2, 3, 7]], 'f64', res['f64'][k, [0, 1, 2, 3, 7]])
