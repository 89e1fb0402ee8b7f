"""Per-kernel medians of the counters in one rocprofv3 --pmc run (rocpd database), for the
FeedingJaco step kernels:  python tools/pmc_counters_summary.py <db_dir> COUNTER [COUNTER ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rocpd_summary as R  # noqa: E402

d, names = sys.argv[1], sys.argv[2:]
sub = [os.path.join(d, x) for x in sorted(os.listdir(d)) if os.path.isdir(os.path.join(d, x))]
c = R.db(d) or next((R.db(s) for s in sub if R.db(s)), None)
if c is None:
    raise SystemExit('no rocpd database under %s' % d)
cnt = R.counters(c, names)
for k, v in cnt.items():
    print(k, ' '.join('%s=%.4g' % (n, v[n]) for n in names if n in v))
    w, ia = v.get('SQ_WAVE_CYCLES'), v.get('SQ_WAIT_INST_ANY')
    if w and ia is not None:
        print('   wait-for-instruction share of wave cycles %.3f' % (ia / w))
    rq, h = v.get('SQC_ICACHE_REQ'), v.get('SQC_ICACHE_HITS')
    if rq and h is not None:
        print('   instruction-cache hit rate %.3f' % (h / rq))
