"""Per-kernel average durations from a rocprofv3 kernel-trace database (rocpd .db)."""
import glob
import sqlite3
import sys

db = sys.argv[1] if sys.argv[1].endswith('.db') else glob.glob(sys.argv[1] + '/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute('pragma table_info(kernels)')]
name = 'kernel_name' if 'kernel_name' in cols else 'name'
rows = c.execute('select %s, count(*), avg(end - start), sum(end - start) from kernels group by %s order by 4 desc' % (name, name)).fetchall()
tot = sum(r[3] for r in rows)
for n, k, a, s in rows[:8]:
    print('%-40s n=%5d avg %8.1f us  %5.1f%%' % (n[:40], k, a / 1e3, 100 * s / tot))
