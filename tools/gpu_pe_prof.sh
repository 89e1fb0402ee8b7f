set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/pe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pe/kt -o kt -- python3 bench.py --policy-eval > gpurun_out/pe/pe.json 2> gpurun_out/pe/pe.err || exit 11
python3 - <<'PY' > gpurun_out/pe/summary.txt
import glob, sqlite3, numpy as np
f = sorted(glob.glob('gpurun_out/pe/kt/**/*.db', recursive=True))[0]
c = sqlite3.connect(f)
rows = c.execute('select name, duration, start, "end" from kernels order by start').fetchall() if 0 else c.execute('select name, duration from kernels').fetchall()
by = {}
for n, d in rows: by.setdefault(n.split('(')[0][:90], []).append(d)
tot = sum(sum(v) for v in by.values())
for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print('%-90s %6d avg %8.1f us tot %7.1f ms' % (n, len(v), np.mean(v)/1e3, sum(v)/1e6))
print('total kernel ms', tot/1e6)
PY
rm -rf gpurun_out/pe/kt
timeout -k 10 300 python3 bench.py --task DressingJaco-v0 --facade --steps 600 > gpurun_out/pe/facade_dressing.json 2> gpurun_out/pe/fd.err || exit 12
