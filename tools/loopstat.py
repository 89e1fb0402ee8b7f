"""Diagnostic: instruction mix of the loops of one kernel in a gfx950 .s file.
python tools/loopstat.py k.s <kernel-symbol-prefix> [min_instrs]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key)
i = s.index(':', s.index('\n' + key if ('\n' + key) in s else key)) + 1
body = s[i:s.index('.Lfunc_end', i)]
lines = body.split('\n')
labels = {l.split(':')[0]: n for n, l in enumerate(lines) if re.match(r'^\.LBB\d+_\d+:', l)}
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
seen = set()
for n, l in enumerate(lines):
    m = re.search(r's_cbranch_\w+ (\.LBB\d+_\d+)|s_branch (\.LBB\d+_\d+)', l)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    j = labels.get(t)
    if j is None or j >= n or (j, n) in seen:
        continue
    seen.add((j, n))
    ins = [x.split()[0] for x in lines[j:n + 1] if x.startswith('\t') and not x.strip().startswith(';') and not x.strip().startswith('.')]
    if len(ins) < mn:
        continue
    c = Counter(ins)
    print('loop %s [%d..%d] instrs %d valu %d salu %d ds %d vmem %d smem %d nop %d waitcnt %d' % (
        t, j, n, len(ins), sum(v for k, v in c.items() if k.startswith('v_')), sum(v for k, v in c.items() if k.startswith('s_') and not k.startswith(('s_nop', 's_waitcnt', 's_load', 's_cbranch', 's_branch'))),
        sum(v for k, v in c.items() if k.startswith('ds_')), sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_', 'flat_', 'scratch_'))),
        sum(v for k, v in c.items() if k.startswith('s_load')), c.get('s_nop', 0), c.get('s_waitcnt', 0)))
