"""Median per-dispatch counter values per kernel from rocprofv3 rocpd databases.

    python tools/pmc_query.py <dir-with-*.db> [kernel-substring ...]
"""
import glob
import os
import sqlite3
import sys

import numpy as np


def main(d, kernels):
    for f in sorted(glob.glob(os.path.join(d, '**', '*.db'), recursive=True)):
        c = sqlite3.connect(f)
        names = [r[0] for r in c.execute('select distinct counter_name from counters_collection')]
        for k in kernels:
            vals = {}
            for n in names:
                v = [r[0] for r in c.execute("select value from counters_collection where counter_name=? and kernel_name like ?", (n, '%' + k + '%'))]
                if v:
                    vals[n] = float(np.median(v))
            if vals:
                print(os.path.basename(f), k, ' '.join('%s=%.4g' % kv for kv in sorted(vals.items())))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:] or ['substep_a', 'substep_b'])
