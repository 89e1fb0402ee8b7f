"""Summarise rocprofv3 rocpd databases (ROCm 7.2 default output) into profiles/.

    python tools/rocpd_summary.py <prof_dir> <round_tag> [envs] [task]

task: FeedingJaco-v0 (default) or ScratchItchPR2-v0 (launch multiplicities differ: 10 sub-steps
per env-step vs 5).  Kernel names carry the task namespace (avr_feeding:: / avr_scratch::).

<prof_dir>/kt/*.db     --kernel-trace --stats run  -> profiles/<tag>_kernel_stats.csv
<prof_dir>/fetch/*.db  --pmc FETCH_SIZE            -> } profiles/pmc_traffic.json and
<prof_dir>/write/*.db  --pmc WRITE_SIZE            -> } profiles/<tag>_pmc.json
<prof_dir>/sq/*.db     --pmc SQ_* instruction mix  -> }
FETCH_SIZE is doubled (gfx950: it reports half the bytes of 128-B requests, MI355X_MICROARCH.md
HBM section); WRITE_SIZE is taken as is.  Counter values are per dispatch, in KiB.
"""
import glob
import json
import os
import sqlite3
import sys

import numpy as np

# launches per env-step: one take_step, one task launch and, per sub-step, the five sub-step kernels
# (FeedingJaco: 5 frames x 2 sub-steps; ScratchItchPR2: 5 frames x 1 sub-step)
SUBSTEPS = {'FeedingJaco-v0': 10, 'ScratchItchPR2-v0': 5, 'BedBathingPR2-v0': 5}


def step_kernels(task):
    if task == 'DressingJaco-v0':          # one launch per gym step (csrc/avr_dressing.hip)
        return {'avr_dress_step_kernel': 1}
    n = SUBSTEPS[task]
    k = {'avr_take_step_kernel': 1, 'avr_substep_pairs_kernel': n, 'avr_narrowphase_kernel': n,
         'avr_substep_a_kernel': n, 'avr_substep_b4_kernel': n, 'avr_task_kernel': 1}
    if task == 'BedBathingPR2-v0':        # the closest distance's stalled pairs (round 6, avr_glue_bedbath.hip)
        k['avr_bb_stall_kernel'] = 1
    return k


STEP_KERNELS = step_kernels('FeedingJaco-v0')


def db(d):
    f = sorted(glob.glob(os.path.join(d, '*.db')))
    return sqlite3.connect(f[0]) if f else None


def kernel_stats(c):
    rows = c.execute('select name, duration from kernels').fetchall()
    by = {}
    for n, d in rows:
        by.setdefault(n.split('(')[0], []).append(d)
    out = []
    tot = sum(sum(v) for v in by.values())
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v = np.array(v, float)
        out.append((n, len(v), v.sum(), v.mean(), np.median(v), v.min(), v.max(), 100 * v.sum() / tot))
    return out


def counters(c, names):
    """{kernel: {counter: median per-dispatch value}} for the step's kernels."""
    res = {}
    for k in STEP_KERNELS:
        for n in names:
            v = [r[0] for r in c.execute("select value from counters_collection where counter_name=? and (kernel_name like ? or kernel_name like ?)",
                                         (n, k + '(%', '%::' + k + '(%'))]
            if v:
                res.setdefault(k, {})[n] = float(np.median(v))
    return res


def per_step(cnt, name, groups=1):
    """sum over the kernels of one env-step (launch multiplicities of STEP_KERNELS, once per env
    group); None unless every step kernel has the counter."""
    if not cnt or any(name not in cnt.get(k, {}) for k in STEP_KERNELS):
        return None
    return sum(cnt[k][name] * STEP_KERNELS[k] * groups for k in STEP_KERNELS)


def main(pdir, tag, envs=4096, groups=None, task='FeedingJaco-v0'):
    global STEP_KERNELS
    STEP_KERNELS = step_kernels(task)
    # the bench runs min(4, envs / 1024) env groups: every kernel of the step is dispatched once
    # per group, over that group's share of the envs
    groups = groups or (1 if task == 'DressingJaco-v0' else max(1, min(4, envs // 1024)))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.environ.get('AVR_PROF_OUT') or os.path.join(root, 'profiles')   # (on the GPU box: a gpurun_out/ dir)
    os.makedirs(prof, exist_ok=True)
    # kt: the bench as the driver runs it (env groups); kt1: the same bench with one env group,
    # whose launches are the ones bench.py's per-kernel event pass times
    for sub, name in (('kt', '%s_kernel_stats.csv'), ('kt1', '%s_kernel_stats_1group.csv')):
        c = db(os.path.join(pdir, sub))
        if not c:
            continue
        st = kernel_stats(c)
        with open(os.path.join(prof, name % tag), 'w') as f:
            f.write('kernel,calls,total_ns,avg_ns,median_ns,min_ns,max_ns,pct\n')
            for r in st:
                f.write('%s,%d,%.0f,%.1f,%.1f,%.0f,%.0f,%.2f\n' % r)
        print(name % tag)
        for r in st:
            print('%-28s calls %4d avg %10.3f ms  median %10.3f ms  %5.1f%%' % (r[0], r[1], r[3] / 1e6, r[4] / 1e6, r[7]))
    out = {'task': task, 'kernels_per_step': STEP_KERNELS, 'envs': envs, 'env_groups': groups,
           'dispatches_per_step': {k: v * groups for k, v in STEP_KERNELS.items()}}   # (only kernels that run in a step)
    cf, cw, cs = db(os.path.join(pdir, 'fetch')), db(os.path.join(pdir, 'write')), db(os.path.join(pdir, 'sq'))
    fetch = counters(cf, ['FETCH_SIZE']) if cf else {}
    write = counters(cw, ['WRITE_SIZE']) if cw else {}
    out['FETCH_SIZE_KiB_raw_per_launch'] = {k: v['FETCH_SIZE'] for k, v in fetch.items()}
    out['WRITE_SIZE_KiB_per_launch'] = {k: v['WRITE_SIZE'] for k, v in write.items()}
    if cs:
        out['sq_per_launch'] = counters(cs, ['SQ_WAVES', 'SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_SMEM', 'SQ_INSTS_LDS', 'SQ_WAIT_ANY',
                                             'SQ_ACTIVE_INST_ANY', 'SQ_WAVE_CYCLES'])
    f_step, w_step = per_step(fetch, 'FETCH_SIZE', groups), per_step(write, 'WRITE_SIZE', groups)
    if f_step is not None and w_step is not None:
        fb, wb = 2 * f_step * 1024, w_step * 1024
        out['hbm_read_bytes_per_step'] = fb
        out['hbm_write_bytes_per_step'] = wb
        out['hbm_bytes_per_step'] = fb + wb
        out['hbm_bytes_per_env_step'] = (fb + wb) / envs
        out['correction'] = 'FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; median per-dispatch value x dispatches per step (launches x env groups)'
        json.dump(out, open(os.path.join(prof, {'FeedingJaco-v0': 'pmc_traffic.json', 'ScratchItchPR2-v0': 'pmc_scratch.json', 'DressingJaco-v0': 'pmc_dressing.json'}.get(task, 'pmc_bedbath.json')), 'w'), indent=1)
    json.dump(out, open(os.path.join(prof, '%s_pmc.json' % tag), 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4096,
         task=sys.argv[4] if len(sys.argv) > 4 else 'FeedingJaco-v0')
