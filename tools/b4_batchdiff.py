"""Diagnostic: env 37 alone vs in a batch of 64 (tests/test_gpu_parity.py batch independence):
which state words differ after settle / steps, for the LDS and the forced-global part-B paths."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states(A, md, 1001, list(range(16)), impairment='random')
S = np.tile(S, (4, 1)).astype(np.float32)
def run(glob, n, Sx, off, frames):
    os.environ['AVR_B4_GLOBAL'] = glob
    b = _lib.Sim(md, n, env_offset=off); b.set_state(Sx); b.settle(frames)
    G = b.get_state(); b.close(); return G
for frames in (2, 3, 5):
    bl = run('0', 64, S, 0, frames)[37]; bg = run('1', 64, S, 0, frames)[37]
    ol = run('0', 1, S[37:38], 37, frames)[0]; og = run('1', 1, S[37:38], 37, frames)[0]
    S37 = np.tile(S[37:38], (64, 1))
    cl = run('0', 64, S37, 0, frames); cg = run('1', 64, S37, 0, frames)
    f = lambda a, b: int(np.count_nonzero(a != b))
    print('frames %d: batchL-batchG %d  aloneL-aloneG %d  batchG-aloneG %d  batchL-aloneL %d  copiesL spread %d copiesG spread %d copiesL-aloneL %d' % (
        frames, f(bl, bg), f(ol, og), f(bg, og), f(bl, ol), int(np.count_nonzero(cl != cl[0])), int(np.count_nonzero(cg != cg[0])), f(cl[0], ol)), flush=True)
