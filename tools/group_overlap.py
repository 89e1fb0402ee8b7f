"""Env-group overlap in a rocprofv3 kernel trace (tools/gpu_group_overlap.sh): per gym step, when
each env group's take_step starts relative to the first group's, how long each group's launch chain
runs, and how many sub-step kernels run at once on average.

    python3 tools/group_overlap.py <rocprofv3 output dir> [kernel namespace, default avr_feeding]
"""
import glob
import os
import sqlite3
import sys

import numpy as np


def main(d, ns='avr_feeding'):
    f = sorted(glob.glob(os.path.join(d, '**', '*.db'), recursive=True))[0]
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute('pragma table_info(kernels)')]
    qcol = next((k for k in ('stream_id', 'queue_id') if k in cols), None)
    print('columns', cols)
    rows = c.execute('select name, start, "end", %s from kernels order by start' % (qcol or '0')).fetchall()
    rows = [r for r in rows if r[0].startswith(ns + '::')]
    takes = [r for r in rows if 'avr_take_step_kernel' in r[0]]
    # a gym step: take_step launches of all groups within 3 ms of the first
    steps, cur = [], []
    for r in takes:
        if cur and r[1] - cur[0][1] > 3e6:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    offs = [[(r[1] - s[0][1]) / 1e3 for r in s] for s in steps if len(s) > 1]
    print('groups per step (median)', np.median([len(s) for s in steps]))
    print('take_step start offsets us (median over steps, by order):', np.median(np.array([o for o in offs if len(o) == len(offs[-1])]), 0).round(1))
    for s0, s1 in zip(steps[:-1], steps[1:]):
        pass
    # concurrency: time-weighted number of running kernels between the first and last kernel of the
    # traced window after warm-up
    t0, t1 = steps[min(3, len(steps) - 1)][0][1], steps[-1][0][1]
    ev = []
    for r in rows:
        if r[1] >= t0 and r[2] <= t1:
            ev += [(r[1], 1), (r[2], -1)]
    ev.sort()
    busy = np.zeros(8)
    n, last = 0, t0
    for t, dlt in ev:
        busy[min(n, 7)] += t - last
        n += dlt
        last = t
    busy /= busy.sum()
    print('share of time with k kernels running, k = 0..7:', busy.round(3))
    if len(steps) > 4:
        dt = np.diff([s[0][1] for s in steps[3:]]) / 1e3
        print('step period us median %.0f' % np.median(dt))
    if os.environ.get('DUMP'):
        mid = len(rows) // 2
        base = rows[mid][1]
        for r in rows[mid:mid + int(os.environ['DUMP'])]:
            print('s%-2s %9.1f %7.1f %s' % (r[3], (r[1] - base) / 1e3, (r[2] - r[1]) / 1e3, r[0].split('::')[1][:28]))
    if qcol:
        qs = sorted(set(r[3] for r in rows))
        print(qcol, 'values', qs[:16])


if __name__ == '__main__':
    main(sys.argv[1], *(sys.argv[2:3]))
