"""Kernel timeline of a rocprofv3 --kernel-trace rocpd database: per queue, the idle gap between a
kernel's end and the next kernel's start, and how much of the traced span has at least one kernel
running.   python tools/timeline.py <db-dir> [skip_first_fraction]"""
import glob
import sqlite3
import sys

import numpy as np


def main(d, skip=0.3):
    f = sorted(glob.glob(d + '/**/*.db', recursive=True))[0]
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute('pragma table_info(kernels)')]
    print('columns:', cols)
    q = 'queue_id' if 'queue_id' in cols else ('stream_id' if 'stream_id' in cols else None)
    rows = c.execute('select start, end, name%s from kernels order by start' % (', ' + q if q else '')).fetchall()
    rows = rows[int(len(rows) * skip):]          # past the warmup / reset part
    s = np.array([r[0] for r in rows], float); e = np.array([r[1] for r in rows], float)
    names = [r[2].split('(')[0].split('::')[-1] for r in rows]
    qs = np.array([r[3] for r in rows]) if q else np.zeros(len(rows))
    span = e.max() - s.min()
    # union of busy intervals
    busy, cur_s, cur_e = 0.0, s[0], e[0]
    for a, b in zip(s[1:], e[1:]):
        if a > cur_e:
            busy += cur_e - cur_s; cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    busy += cur_e - cur_s
    print('dispatches %d, span %.3f ms, some kernel running %.1f %%' % (len(rows), span / 1e6, 100 * busy / span))
    for qq in np.unique(qs):
        m = qs == qq
        ss, ee = s[m], e[m]
        gaps = ss[1:] - ee[:-1]
        nm = [n for n, k in zip(names, m) if k]
        print('queue %s: %d dispatches, gap us median %.2f mean %.2f p90 %.2f; gap share of the queue span %.1f %%'
              % (qq, m.sum(), np.median(gaps) / 1e3, gaps.mean() / 1e3, np.percentile(gaps, 90) / 1e3,
                 100 * np.clip(gaps, 0, None).sum() / (ee.max() - ss.min())))
        per = {}
        for k in range(len(gaps)):
            per.setdefault(nm[k + 1], []).append(gaps[k])
        print('   mean gap before each kernel (us):', {k: round(float(np.mean(v)) / 1e3, 2) for k, v in per.items()})


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.3)
