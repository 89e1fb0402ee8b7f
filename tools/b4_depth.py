"""Diagnostic: part-B results vs pipeline depth of the contact sweeps, one sub-step from a settled
state (AVR_LIB selects the build)."""
import os, sys, subprocess
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
if len(sys.argv) > 1 and sys.argv[1] == 'child':
    from avr import _abi as ABI, reset as RS, _lib
    A = ABI.load_scene(); md = ABI.ModelDesc(A)
    S0 = np.load('/tmp/b4d_settled.npy')
    b = _lib.Sim(md, len(S0)); b.set_state(S0); b.substep(0.01)
    np.save(sys.argv[2], b.get_state()); b.close()
    sys.exit(0)
from avr import _abi as ABI, reset as RS, _lib
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states(A, md, 1001, list(range(16)), impairment='none')
b = _lib.Sim(md, 16); b.set_state(S.astype(np.float32)); b.settle(30); np.save('/tmp/b4d_settled.npy', b.get_state()); b.close()
L = os.path.join(ROOT, 'assistive-vr-gym_amd', 'avr')
runs = [('dc1', ROOT + '/exp/libavr_dc1.so'), ('dc2', L + '/libavr.so'), ('dc3', ROOT + '/exp/libavr_dc3.so'), ('dc4', ROOT + '/exp/libavr_dc4.so')]
out = {}
for name, lib in runs:
    f = '/tmp/b4d_%s.npy' % name
    subprocess.check_call([sys.executable, __file__, 'child', f], env=dict(os.environ, AVR_LIB=lib), stderr=subprocess.DEVNULL)
    out[name] = np.load(f)
ks = list(out)
print({'%s-%s' % (a, c): int(np.count_nonzero(out[a] != out[c])) for i, a in enumerate(ks) for c in ks[i + 1:]})
G2, G3 = out['dc2'], out['dc3']
for e in range(0):
    d = np.nonzero(G2[e] != G3[e])[0]
    if len(d):
        n = int(G2[e, ABI.S_TASK + ABI.T_NCP])
        imp2 = G2[e, ABI.S_CP + 12: ABI.S_CP + 16 * n: 16]; imp3 = G3[e, ABI.S_CP + 12: ABI.S_CP + 16 * n: 16]
        di = np.nonzero(imp2 != imp3)[0]
        print('env', e, 'ncp', n, 'words', len(d), 'first', d[:6], 'imp diffs at contacts', di[:10], 'max', np.abs(imp2 - imp3).max(), 'min idx', d.min())
