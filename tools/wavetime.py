"""Diagnostic: wave timeline of the last sub-step kernels A and B (AVR_WAVETIME build,
libavr_wt.so): per-wave durations (p50/p90/p99/max), kernel span, and how the span splits into
'all waves busy' vs the tail.  python tools/wavetime.py [n_envs] [lib]"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd')); sys.path.insert(0, ROOT)
from avr import _abi as ABI, reset as RS, _lib
so = sys.argv[2] if len(sys.argv) > 2 and os.path.isabs(sys.argv[2]) else os.path.join(ROOT, "assistive-vr-gym_amd", "avr", sys.argv[2] if len(sys.argv) > 2 else "libavr_wt.so")
_lib.LIB_PATH = so
lib = _lib.load(so)
lib.avr_set_profile_buffer.argtypes = [C.c_void_p, C.c_void_p]
import torch
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
A = ABI.load_scene(); md = ABI.ModelDesc(A)
S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(min(N, 256))), impairment=os.environ.get('IMPAIRMENT', 'random'))
S = np.tile(S, ((N + len(S) - 1) // len(S), 1))[:N]
sim = _lib.Sim(md, N)
buf = torch.zeros(5 * N * 2, dtype=torch.int64, device='cuda')
lib.avr_set_profile_buffer(sim.h, buf.data_ptr())
sim.set_state(S.astype(np.float32)); sim.settle(20)
for t in range(3):
    sim.step(_lib.random_actions(1001, np.arange(N), t))
    raw = buf.cpu().numpy().reshape(5, N, 2)
    p = raw[:2].astype(np.float64) * 10.0   # 100 MHz ticks -> ns
    for k, nm in enumerate(('A', 'B')):
        sel = p[k, :, 0] > 0        # B: one record per block (its group-0 env)
        s0, s1 = p[k, sel, 0], p[k, sel, 1]
        d = (s1 - s0) / 1e3
        span = (s1.max() - s0.min()) / 1e3
        t0 = s0.min()
        last_start = (s0.max() - t0) / 1e3
        order = np.argsort(-d)
        print('step %d kernel %s: span %.1f us, wave us p50 %.1f p90 %.1f p99 %.1f max %.1f mean %.1f, last wave starts at %.1f us; slowest envs %s'
              % (t, nm, span, np.percentile(d, 50), np.percentile(d, 90), np.percentile(d, 99), d.max(), d.mean(), last_start,
                 order[:6].tolist()))
        if nm == 'B':
            w = raw[2, sel]
            nnc, nc, lds, nrows = w[:, 0] & 0xffff, (w[:, 0] >> 16) & 0xffff, (w[:, 0] >> 32) & 1, w[:, 1] & 0xffff
            print('   B blocks %d: in LDS %.3f; nnc_max mean %.1f max %d; nc_max mean %.1f max %d; rows_max mean %.1f max %d'
                  % (len(d), lds.mean(), nnc.mean(), nnc.max(), nc.mean(), nc.max(), nrows.mean(), nrows.max()))
            c = np.polyfit(nrows.astype(np.float64), d, 1)
            print('   B us ~ %.3f * rows_max + %.1f (corr %.3f); slowest blocks: us %s rows %s lds %s'
                  % (c[0], c[1], np.corrcoef(nrows, d)[0, 1], np.round(d[order[:6]], 1).tolist(), nrows[order[:6]].tolist(), lds[order[:6]].tolist()))
            hist = np.histogram(d, bins=10)
            print('   B duration histogram', hist[0].tolist(), np.round(hist[1], 1).tolist())
    npd = raw[3].astype(np.float64) * 10.0 / 1e3
    print('   NP block us: list0 mean %.1f p90 %.1f max %.1f; list1 mean %.1f p90 %.1f max %.1f'
          % (npd[:, 0].mean(), np.percentile(npd[:, 0], 90), npd[:, 0].max(), npd[:, 1].mean(), np.percentile(npd[:, 1], 90), npd[:, 1].max()))
    cp = raw[4].astype(np.float64) * 10.0 / 1e3
    cd = cp[:, 1] - cp[:, 0]
    print('   coop block us: span %.1f, starts spread %.1f, duration mean %.2f p99 %.1f max %.1f, blocks > 3 us: %d'
          % (cp[:, 1].max() - cp[:, 0].min(), cp[:, 0].max() - cp[:, 0].min(), cd.mean(), np.percentile(cd, 99), cd.max(), int((cd > 3).sum())))
    St = sim.get_state()
ncp = St[:, ABI.S_TASK + ABI.T_NCP]
print('ncp of slowest A envs', ncp[order[:6]], 'mean ncp', ncp.mean())
np.save(os.path.join(ROOT, 'gpurun_out', 'wavetime_%d.npy' % N), raw)
