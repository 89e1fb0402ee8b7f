"""Diagnostic: per-phase cycle breakdown of the step kernel (AVR_PROF build, libavr_prof.so)."""
import ctypes as C, os, sys, subprocess, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
so = os.path.join(ROOT, 'assistive-vr-gym_amd', 'avr', sys.argv[2] if len(sys.argv) > 2 else 'libavr_prof.so')
_lib.LIB_PATH = so
lib = _lib.load(so)
lib.avr_set_profile_buffer.argtypes = [C.c_void_p, C.c_void_p]
import torch
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
TASK = int(os.environ.get('TASK', '0'))        # 0 FeedingJaco, 1 ScratchItchPR2, 2 BedBathingPR2
A = ABI.load_scene(TASK); md = ABI.ModelDesc(A)
L = md.layout
if TASK == 0:
    S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(min(N, 256))), impairment=os.environ.get('IMPAIRMENT', 'random'))
else:
    import bench
    S, _ = bench.reset_pool(TASK, A, md, list(range(min(N, 64))), os.environ.get('IMPAIRMENT', 'random'))
S = np.tile(S, ((N + len(S) - 1) // len(S), 1))[:N]
sim = _lib.Sim(md, N)
SLOTS = 48
prof = torch.zeros(N * SLOTS, dtype=torch.int64, device='cuda')
lib.avr_set_profile_buffer(sim.h, prof.data_ptr())
sim.set_state(S.astype(np.float32)); sim.settle(100 if TASK == 0 else 0)
names = ['fk', 'bodies+broad', 'childpairs', 'narrow+mf', '#culleditems', '#xcd-mismatch', 'dyn', 'nc_rows', 'c_rows', 'solve', 'integrate', '#cooppairs', 'task', 'collide', '#shapepairs', '#bodypairs', ' lane-narrow', ' coop', ' manifold', '#coop sph-hull', '#coop hull-hull', '#coop other', '#coop bighull', '-',
         ' M entries', ' cholesky', ' M^-1 cols', ' bias (RNEA)', '#coop GJK it', '#coop cycles', '#coop max cyc', '-',
         '#np sph-hull', '#np other', '#np refill trips', '#np ph_steps', '#np GJK it', '#np GJK it max', '#np GJK pairs', '#np closed form',
         '  mf match', '  mf add', '  mf refresh', '-', '-', '-', '-', '-']
for t in range(int(os.environ.get('PROF_STEPS', '3'))):
    prof.zero_()
    t0 = time.time(); sim.step(_lib.random_actions(1001, np.arange(N), t)); el = time.time() - t0
    p = prof.cpu().numpy().reshape(N, SLOTS).astype(np.float64)
    tot = p[:, [0, 13, 6, 7, 8, 9, 10, 12]].sum(1).mean()   # (coop part) is inside narrow+mf
    print('step %d wall %.1f ms, mean cycles/env %.3g' % (t, el * 1e3, tot))
    for k, nm in enumerate(names):
        if nm == '-':
            continue
        if nm.startswith('#'):
            print('  %-13s per env-step mean %.1f (per substep %.1f), max %.0f' % (nm, p[:, k].mean(), p[:, k].mean() / 10, p[:, k].max()))
            continue
        print('  %-13s %6.2f%%  mean %.3g  max %.3g' % (nm, 100 * p[:, k].mean() / tot, p[:, k].mean(), p[:, k].max()))
St = sim.get_state()
print('ncp mean', St[:, L.S_TASK + L.T_NCP].mean(), 'flags', np.unique(St[:, L.S_TASK + L.T_FLAGS]))
# the envs with the slowest contact-row phase: their contact count and robot endpoints (last step)
c_rows = p[:, 8]
top = np.argsort(-c_rows)[:6]
bk = A['body_kind'] if 'body_kind' in A else None
cpw = ABI.CP_WORDS if hasattr(ABI, 'CP_WORDS') else None
for e in top:
    ncp = int(St[e, L.S_TASK + L.T_NCP])
    nrob = -1
    if bk is not None and cpw is not None and hasattr(L, 'S_CP'):
        cp = St[e, L.S_CP:L.S_CP + cpw * ncp].reshape(ncp, cpw)
        sb = A['shape_body']
        kinds = [(int(bk[sb[int(r[ABI.CP_SA])]]), int(bk[sb[int(r[ABI.CP_SB])]])) for r in cp]
        nrob = sum(1 for a, b in kinds if a == ABI.BODY_ROBOT or b == ABI.BODY_ROBOT)
        print('slow c_rows env %d: %.3g cycles/env-step, contacts %d, robot contacts %d, (kind A, kind B) %s, bodies %s'
              % (e, c_rows[e], ncp, nrob, kinds, [(int(sb[int(r[ABI.CP_SA])]), int(sb[int(r[ABI.CP_SB])])) for r in cp]))
    else:
        print('slow c_rows env %d: %.3g cycles/env-step, contacts %d' % (e, c_rows[e], ncp))
# kernel a's slowest envs (the launch's tail): their phases against the median env's (last step)
ka = p[:, 3] + p[:, 6] + p[:, 7] + p[:, 8]
med = np.median(p, axis=0)
cols = [(3, 'narrow+mf'), (17, 'coop'), (40, 'mf match'), (41, 'mf add'), (42, 'mf refresh'), (18, 'mf pool'), (6, 'dyn'), (7, 'nc_rows'), (8, 'c_rows'), (24, 'M'), (25, 'chol'), (26, 'Minv'), (27, 'bias')]
print('kernel a per env-step cycles: median %.3g, p99 %.3g, max %.3g' % (np.median(ka), np.percentile(ka, 99), ka.max()))
print('  median env   ' + ' '.join('%s %.3g' % (nm, med[k]) for k, nm in cols))
for e in np.argsort(-ka)[:8]:
    print('  env %4d %.3g ncp %2d ' % (e, ka[e], int(St[e, L.S_TASK + L.T_NCP])) + ' '.join('%s %.3g' % (nm, p[e, k]) for k, nm in cols))
