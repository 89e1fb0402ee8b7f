"""The narrowphase of one shape pair at a launch-shape pool state, GPU (avr_narrowphase_query)
against the fp64 and fp32 oracles, plus a jittered neighbourhood of that pose: which queries
the GPU answers differently from both oracles.

  TASK=1 K=27 SA=50 SB=165 python tools/dbg_np_state.py
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [os.path.join(ROOT, 'assistive-vr-gym_amd'), ROOT, os.path.join(ROOT, 'tests')]
from avr import _abi as ABI, _lib, geom as G  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
import test_pr2_launch_shape as T  # noqa: E402

np.set_printoptions(precision=6, suppress=True, linewidth=200)
TASK = int(os.environ.get('TASK', 1))
K = int(os.environ.get('K', 27))
SA, SB = int(os.environ.get('SA', 50)), int(os.environ.get('SB', 165))
N = int(os.environ.get('N', 4000))
A, md, L, P, is_c = T._pool(TASK, 16)
st = P[K].astype(np.float64)


def body_pose(b):
    kind, idx = int(A['body_kind'][b]), int(A['body_index'][b])
    if kind == ABI.BODY_FREE:
        return st[L.S_FREE + 13 * idx:L.S_FREE + 13 * idx + 7]
    if kind == ABI.BODY_HUMAN:
        return st[L.S_HUMAN + 7 * idx:L.S_HUMAN + 7 * idx + 7]
    raise SystemExit('body %d kind %d: not a free / human body' % (b, kind))


pa, pb = body_pose(int(A['shape_body'][SA])), body_pose(int(A['shape_body'][SB]))
rng = np.random.default_rng(1)
X = np.zeros((N, 14))
X[:, :7], X[:, 7:] = pa, pb
for k in range(1, N):
    q = G.quat_axis_angle(rng.standard_normal(3), rng.uniform(0, 0.05))
    X[k, 3:7] = G.quat_mul(q, pa[3:7])
    X[k, 3:7] /= np.linalg.norm(X[k, 3:7])
    X[k, :3] = pa[:3] + rng.uniform(-0.005, 0.005, 3)
pairs = np.tile([SA, SB], (N, 1)).astype(np.int32)
sim = _lib.Sim(md, 1)
g = sim.narrowphase(pairs, X.astype(np.float32)).astype(np.float64)
sim.close()
res = {}
for prec in ('f64', 'f32'):
    o = Oracle(md, 1, prec)
    R = np.zeros((N, 8))
    for k in range(N):
        r, out = o.narrowphase(SA, X[k, :7], SB, X[k, 7:], 0.02)
        R[k, 0], R[k, 1:] = r, out
    res[prec] = R
    o.close()


def off(R, ref):
    both = (R[:, 0] > 0) & (ref[:, 0] > 0)
    ang = np.degrees(np.arccos(np.clip((R[:, 1:4] * ref[:, 1:4]).sum(1), -1, 1)))
    return ((R[:, 0] > 0) != (ref[:, 0] > 0)) | (both & ((ang > 2) | (np.abs(R[:, 7] - ref[:, 7]) > 1e-4))), ang


print('pool state %d pair (%d, %d): GPU rc %d n %s d %.6f | f64 rc %d n %s d %.6f | f32 rc %d n %s d %.6f' % (
    K, SA, SB, g[0, 0], g[0, 1:4], g[0, 7], res['f64'][0, 0], res['f64'][0, 1:4], res['f64'][0, 7], res['f32'][0, 0], res['f32'][0, 1:4], res['f32'][0, 7]))
og, ag = off(g, res['f64'])
o32, a32 = off(res['f32'], res['f64'])
print('jittered %d: GPU off %d, fp32 oracle off %d, GPU-only %d, both %d' % (N, og.sum(), o32.sum(), (og & ~o32).sum(), (og & o32).sum()))
for k in np.nonzero(og & ~o32)[0][:12]:
    print('  q%-5d GPU n %s d %.6f | f64 n %s d %.6f | angle %.2f deg' % (k, g[k, 1:4], g[k, 7], res['f64'][k, 1:4], res['f64'][k, 7], ag[k]))
np.save(os.path.join(ROOT, 'gpurun_out', 'np_state_%d_%d_%d.npy' % (K, SA, SB)), X[np.nonzero(og & ~o32)[0]])
