#!/usr/bin/env python3
"""Benchmark: env-steps/s on MI355X.  Default: FeedingJaco-v0 at 4096 envs (BASELINE.json
configs[1]); --task ScratchItchPR2-v0 runs configs[2]; --task BedBathingPR2-v0 is the PR2 variant
of configs[3] (BASELINE's BedBathingSawyer-v0 does not exist in the reference):
32768 envs over 8 GPUs = torchrun --nproc-per-node 8 bench.py --task BedBathingPR2-v0 --gpus 8.

One "step" = one gym step of every env (take_step + 5 x stepSimulation (FeedingJaco: 2 sub-steps
each, ScratchItch: 1) + task glue) = one launch sequence of the gfx950 kernels.  Synthetic random
actions are drawn on the device (Philox4x32-10 keyed by (seed=1001, global env id, step),
examples/random_actions.py semantics).  Inputs are resident in HBM before the timed region; host
buffers are not touched inside it.

  python bench.py [--task T] [--gpus N] [--steps K] [--warmup W] [--envs E_per_gpu]
  torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU: envs shard across ranks (global env id = rank*E + e, independent units -> weak
scaling); rollouts (obs, reward, done, info) are collected with an RCCL all-gather over xGMI
every --gather-every steps (the only data-path collective).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


# algorithmic bytes per env-step = persistent state read + written once + read-only
# per-env params + action in + obs, reward, done, info out.  FeedingJaco: 605 words (2420 B) each
# way + 144 + 28 + 116 = 5128 B.  ScratchItchPR2: 563 words (2252 B) each way + 120 + 28 + 136.
TASKS = {
    'FeedingJaco-v0': dict(task=0, bytes=2420 * 2 + 144 + 28 + 116, settle=100, substeps=10, iters=10, pool=1024,
                           workload='FeedingJaco-v0, %d envs/GPU, rigid-only, random actions'),
    'ScratchItchPR2-v0': dict(task=1, bytes=2252 * 2 + 120 + 28 + 136, settle=0, substeps=5, iters=50, pool=128,
                              workload='ScratchItchPR2-v0, %d envs/GPU, human-capsule contact + tool force reward, random actions'),
    # BedBathingPR2 (SURVEY 8(d) recipe, ScratchItch's state minus the scratch target plus the wipe bit
    # set: 2252 + 28 B each way) + obs 24 + reward + done + 2 info + action in
    'BedBathingPR2-v0': dict(task=2, bytes=2280 * 2 + 120 + 28 + 112, settle=0, substeps=5, iters=50, pool=128,
                             workload='BedBathingPR2-v0, %d envs/GPU, wiping targets + tool-human closest distance, random actions'),
    # DressingJaco (build-defined, include/avr_dressing.h): the 1104-word state block in and out once
    # (it stays in registers / LDS across the 100 cloth sub-steps of one launch) + action + obs 24,
    # reward, done, info 2; BASELINE configs[4] runs 2048 envs
    'DressingJaco-v0': dict(task=3, bytes=1104 * 4 * 2 + 28 + 112, settle=0, substeps=100, iters=0, pool=128, envs=2048,
                            workload='DressingJaco-v0, %d envs/GPU, mass-spring sleeve (128 particles) with penalty cloth-arm contact, random actions'),
}
VALU_CYC = 2.0          # v_fma_f32 wave64 issue throughput, cycles (MI355X_MICROARCH.md cycle table)
SIMDS, CLOCK_HZ = 1024, 2.4e9


def layout_bytes_per_env_step(L):
    """What this build's state layout actually moves per env-step (state block in and out once,
    it stays resident across the sub-steps; actions are generated on the device)."""
    return 2 * L.STATE_WORDS * 4 + (L.OBS_DIM + 1 + L.INFO_DIM) * 4 + 1


def reset_pool(task, A, md, ids, impairment, device=0):
    """Reset states of the bench's env pool; the PR2 tasks' base-pose search runs on the device
    (avr_base_search) with the reference's 100 attempts of 200 IK iterations, on this rank's GPU."""
    if task == 3:
        from avr import reset_dressing as RD
        return RD.batch_reset_states(A, md, 1001, ids)
    if task in (1, 2):
        from avr import _lib
        sim = _lib.Sim(md, 1, device=device)
        try:
            if task == 2:
                from avr import reset_bedbath as RBB
                return RBB.batch_reset_states(A, md, 1001, ids, sim=sim, device=device)
            from avr import reset_scratch as RSS
            return RSS.batch_reset_states(A, md, 1001, ids, impairment=impairment, sim=sim)
        finally:
            sim.close()
    from avr import reset as RS
    return RS.batch_reset_states_fast(A, md, 1001, ids, impairment=impairment)


def cpu_baseline(name, md, A, seconds, threads, impairment):
    """Oracle (the CPU restatement, fp64) on the host cores; bounded sample of 4 envs per thread."""
    import numpy as np
    from oracle.oracle import Oracle
    from avr import _lib
    T = TASKS[name]
    n = max(threads * 4, 8)
    S, _ = reset_pool(T['task'], A, md, list(range(n)), impairment)
    o = Oracle(md, n)
    o.set_threads(threads)
    o.set_state(S)
    o.settle(T['settle'])
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = _lib.random_actions(1001, np.arange(n), steps)
        o.step(a)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds and steps >= 2:
            break
    return dict(value=n * steps / el, unit='env-steps/s', cores=threads, host_cpus=os.cpu_count(), kind='port',
                short='%d envs x %d steps, fp64 oracle, %d OpenMP threads' % (n, steps, threads),
                sample='%s, %d envs x %d gym steps (%.1f s) after a %d-frame settle; fp64 oracle, OpenMP over envs on %d threads '
                       '(the GPU box\'s CPU share, OMP_NUM_THREADS; os.cpu_count() reports the whole host)' % (
                           name, n, steps, el, T['settle'], threads))


def pmc_summary(name, kernels, ms_per_step, E):
    """HBM traffic and SQ issue figures from the committed rocprofv3 PMC summary of this task's
    bench (profiles/pmc_<task>.json, tools/rocpd_summary.py), if its kernel set and env count match."""
    fname = {'FeedingJaco-v0': 'pmc_traffic.json', 'ScratchItchPR2-v0': 'pmc_scratch.json', 'BedBathingPR2-v0': 'pmc_bedbath.json',
             'DressingJaco-v0': 'pmc_dressing.json'}[name]
    path = os.path.join(ROOT, 'profiles', fname)
    if not os.path.exists(path):
        return None
    try:
        tj = json.load(open(path))
    except Exception:
        return None
    # (the summary may list kernels the event pass folds into another kind: BedBathing's
    # avr_bb_stall_kernel runs inside the task kernel's interval)
    if tj.get('envs') != E or tj.get('task', 'FeedingJaco-v0') != name or not set(kernels) <= set(tj.get('kernels_per_step', {})):
        return None
    out = dict(traffic=tj.get('hbm_bytes_per_step'), source='profiles/' + fname)
    sq = tj.get('sq_per_launch', {})
    disp = tj.get('dispatches_per_step', {})
    if sq and disp:
        valu = sum(sq[k]['SQ_INSTS_VALU'] * disp.get(k, 0) for k in sq)
        out['valu_busy_chip'] = valu * VALU_CYC / (SIMDS * CLOCK_HZ * ms_per_step * 1e-3)
        per = {}
        for k, c in sq.items():
            wc = max(c.get('SQ_WAVE_CYCLES', 0.0), 1.0)
            per[k] = dict(issue_frac=c.get('SQ_ACTIVE_INST_ANY', 0.0) / wc, wait_frac=c.get('SQ_WAIT_ANY', 0.0) / wc,
                          valu_insts_per_wave=c['SQ_INSTS_VALU'] / max(c.get('SQ_WAVES', 1.0), 1.0))
        out['sq'] = per
    return out


def facade_bench(args):
    """Trainer-side throughput: AVRTorchVecEnv.step with device actions, auto-reset on (every env
    ends its episode at the 200-step TimeLimit, then resets: FeedingJaco with the device IK whose
    host draws are prefetched while the previous episode steps).  Reports env-steps/s with the
    rollovers inside the timed region and the same loop's rate between rollovers."""
    import numpy as np
    import torch
    from avr import env as EV
    E = args.envs if args.envs is not None else TASKS[args.task].get('envs', 4096)
    dev = torch.device('cuda', 0)
    v = EV.AVRTorchVecEnv(args.task, E, device=0, impairment=args.impairment)
    t0 = time.perf_counter()
    v.reset()
    torch.cuda.synchronize(dev)
    t_reset = time.perf_counter() - t0
    act = torch.empty(E, v.L.ACT_DIM, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1001)
    for _ in range(args.warmup):
        act.uniform_(-1, 1, generator=gen)
        v.step(act)
    torch.cuda.synchronize(dev)
    roll, t_roll, t_drain = 0, [], []
    c0 = v.sim.graph_captures()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if args.fresh_actions:      # a new action tensor every step, as a policy's output is
            act = torch.rand(E, v.L.ACT_DIM, device=dev, generator=gen) * 2 - 1
        else:
            act.uniform_(-1, 1, generator=gen)
        due = bool((v.iteration + 1 >= v.max_steps).any())
        if due:
            # a rollover step synchronises inside step(): drain the steps queued ahead of it first,
            # so that rollover_ms is the rollover step itself (its launches + the masked reset)
            td = time.perf_counter()
            torch.cuda.synchronize(dev)
            t_drain.append(time.perf_counter() - td)
        ts = time.perf_counter()
        _, _, _, info = v.step(act)
        if 'terminal_observation' in info:
            roll += 1
            t_roll.append(time.perf_counter() - ts)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    captures = v.sim.graph_captures() - c0
    # the same loop over steps that end no episode (synchronised at both ends, after the next
    # episode's reset draws are ready so that no prefetch runs beside it)
    if v._prefetch:
        v._prefetch.wait()
    K = max(1, min(100, v.max_steps - int(v.iteration.max()) - 1))
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    host_ms = []
    for k in range(K):
        act.uniform_(-1, 1, generator=gen)
        th = time.perf_counter()
        v.step(act)
        host_ms.append((time.perf_counter() - th) * 1e3)
    torch.cuda.synchronize(dev)
    no_roll = (time.perf_counter() - t1) / K
    out = {'metric': 'facade env-steps/sec (AVRTorchVecEnv, auto-reset at the 200-step TimeLimit)', 'value': E * args.steps / el,
           'unit': 'env-steps/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': el / args.steps * 1e3,
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
           'data': 'synthetic: torch uniform(-1, 1) actions on the device; resets drawn per env and episode',
           'config': {'workload': args.task + ', %d envs, gym facade with rollover' % E, 'task': args.task, 'envs_per_gpu': E,
                      'impairment': args.impairment,
                      'reset_ik': ('device IK' if (v.device_ik or v.device_dress_ik) else 'device base-pose search' if v.device_search else 'host')},
           'rollovers_timed': roll, 'env_steps_per_s_between_rollovers': E / no_roll, 'between_rollovers_steps': K,
           'between_rollovers_host_ms_per_step': [round(float(np.median(host_ms)), 3), round(float(np.max(host_ms)), 3)],
           'rollover_ms': float(np.mean(t_roll) * 1e3) if roll else None,
           'rollover_scope': 'one rollover step: its launches, the synchronisation and the masked device reset, after the steps '
                             'queued ahead of it were drained (drain_ms_before_rollover, not part of rollover_ms)',
           'drain_ms_before_rollover': float(np.mean(t_drain) * 1e3) if t_drain else None,
           'fresh_action_tensor_per_step': bool(args.fresh_actions), 'graph_captures_in_timed_loop': captures,
           'first_reset_s': t_reset,
           'ik_accept_rate': float(v.last_ik_ok.mean()) if v.last_ik_ok is not None else None,
           'last_rollover_breakdown_s': v.reset_timing,
           'flagged_envs': int(np.count_nonzero(v.flags()))}
    print(json.dumps(out), flush=True)
    v.close()


def progress(msg):
    """A progress line on stderr (long GPU-box runs must keep writing: DESIGN.md section 6)."""
    sys.stderr.write('[bench %.0fs] %s\n' % (time.perf_counter() - T_START, msg))
    sys.stderr.flush()


T_START = time.perf_counter()


def run_task(name, args, steps, warmup, world, rank, local, dist, gloo, dev, cpu_seconds):
    """Time `steps` gym steps of task `name` (E = args.envs per GPU) after `warmup` untimed ones;
    returns the JSON object of its bench line (cpu_baseline when cpu_seconds > 0)."""
    import numpy as np
    progress('%s: reset pool' % name)
    import torch
    from avr import _abi as ABI, _lib
    from avr import dist as D
    T = TASKS[name]
    settle = T['settle'] if args.settle is None else args.settle
    if T['task'] == 3:
        from avr import reset_dressing as RD
        A = RD.dressing_scene()
    else:
        A = ABI.load_scene(T['task'])
    md = ABI.ModelDesc(A)
    L = md.layout
    E = args.envs if args.envs is not None else T.get('envs', 4096)
    # reset pool: distinct initial states for global env ids; tiled if pool < E
    pool = min(args.reset_pool or T['pool'], E)
    base_id, _ = D.shard(E, rank)
    S_pool, meta = reset_pool(T['task'], A, md, [base_id + i for i in range(pool)], args.impairment, device=local)
    n_tremor = sum(m['impairment'] == 'tremor' for m in meta)
    import hashlib
    pool_sha = hashlib.sha1(S_pool.astype(np.float32).tobytes()).hexdigest()[:12]
    S = np.tile(S_pool, ((E + pool - 1) // pool, 1))[:E]
    progress('%s: reset pool ready (%d distinct states)' % (name, pool))
    sim = _lib.Sim(md, E, device=local, seed=1001, env_offset=base_id)
    sim.set_state(S.astype(np.float32))
    sim.settle(settle)

    obs = torch.zeros(E, L.OBS_DIM, device=dev)
    rew = torch.zeros(E, device=dev)
    done = torch.zeros(E, dtype=torch.uint8, device=dev)
    info = torch.zeros(E, L.INFO_DIM, device=dev)
    ext = torch.cuda.ExternalStream(sim.stream(), device=dev)
    G = args.gather_every
    W = D.roll_width(L.OBS_DIM)
    roll = torch.zeros(G, E, W, device=dev)
    gathered = torch.zeros(world * G * E * W, device='cpu' if gloo else dev) if world > 1 else None

    def one_step(t, k):
        sim.step_random_device(t, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), info.data_ptr())
        if world > 1:
            with torch.cuda.stream(ext):
                j = k % G
                D.pack_rollout(roll, j, obs, rew, info, done)
                if j == G - 1:
                    D.gather_rollouts(roll.cpu() if gloo else roll, out=gathered)

    # the timed steps as rollouts (avr_rollout_random_device: the same steps, bit for bit, with
    # the env groups joined at the end of each rollout instead of after every step); multi-GPU:
    # rollouts of G steps with per-step outputs (stacked), packed and all-gathered after each
    if not args.step_sync:
        so, sr, sd, si = (torch.zeros(G, E, L.OBS_DIM, device=dev), torch.zeros(G, E, device=dev),
                          torch.zeros(G, E, dtype=torch.uint8, device=dev), torch.zeros(G, E, L.INFO_DIM, device=dev)) if world > 1 else (None,) * 4

    def run_steps(t0, n):
        if args.step_sync:
            for k in range(n):
                one_step(t0 + k, k)
            return
        if world == 1:
            sim.rollout_random_device(t0, n, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), info.data_ptr())
            return
        for c in range(0, n, G):
            m = min(G, n - c)
            sim.rollout_random_device(t0 + c, m, so.data_ptr(), sr.data_ptr(), sd.data_ptr(), si.data_ptr(), stacked=True)
            with torch.cuda.stream(ext):
                D.pack_rollout_stacked(roll, so, sr, si, sd, m)
                D.gather_rollouts(roll.cpu() if gloo else roll, out=gathered)

    run_steps(0, warmup)
    progress('%s: warmed up, timing %d steps' % (name, steps))
    sim.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ext)
    run_steps(warmup, steps)
    ev1.record(ext)
    sim.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device='cpu' if gloo else dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    t_next = warmup + steps
    # the per-step API's rate beside the rollout headline (avr_step_random_device, env groups
    # joined after every step): what a policy in the loop gets (enjoy_vr.py:106-116, a PPO
    # rollout), which needs every step's observation before it can act
    step_sync = None
    if world == 1 and not args.step_sync and args.sync_steps > 0:
        for k in range(2):                 # untimed: the per-step graph is captured on first use
            one_step(t_next + k, k)
        t_next += 2
        sim.sync()
        torch.cuda.synchronize(dev)
        ts = time.perf_counter()
        for k in range(args.sync_steps):
            one_step(t_next + k, k)
        sim.sync()
        torch.cuda.synchronize(dev)
        es = time.perf_counter() - ts
        t_next += args.sync_steps
        step_sync = {'value': E * args.sync_steps / es, 'ms_per_step': es / args.sync_steps * 1e3, 'steps': args.sync_steps}
    # per-kernel launch durations (HIP events between the launches of a step, on the sim
    # stream), from a separate short pass so the timed loop above carries no event overhead
    P = min(10, steps)
    sim.profile_kernels(True)
    for k in range(P):
        one_step(t_next + k, k)
    kt = sim.kernel_times()
    sim.profile_kernels(False)
    kernels = {k: {'avg_ms': v[0] / max(v[1], 1), 'launches_per_step': v[1] / P, 'ms_per_step': v[0] / P} for k, v in kt.items() if v[1] > 0}
    step_kernel_ms = sum(v['ms_per_step'] for v in kernels.values())
    dominant = max(kernels, key=lambda k: kernels[k]['ms_per_step'])
    St = sim.get_state()
    flags = St[:, L.S_TASK + L.T_FLAGS].astype(np.int64)
    value = world * E * steps / el
    bpe = T['bytes']
    achieved = bpe * E / (step_kernel_ms * 1e-3) / 1e9
    ms_per_step = el / steps * 1e3
    pmc = pmc_summary(name, [k for k, v in kt.items() if v[1] > 0], ms_per_step, E)
    traffic = pmc['traffic'] if pmc else None
    # the bound: the larger of the two roofline fractions the path could sit on (HBM bytes vs the
    # dense matrix-core peak; the path issues no MFMA, so its MFMA fraction is 0)
    fracs = {'hbm': achieved / HBM_PEAK_GBS, 'mfma': 0.0}
    bound = max(fracs, key=fracs.get)
    # what actually limits the kernels, from the PMC SQ counters of the dominant kernel: issue-
    # or wait-dominated wave lifetime (None without a matching PMC summary)
    limiter = None
    if pmc and pmc.get('sq', {}).get(dominant):
        q = pmc['sq'][dominant]
        limiter = 'latency (waves waiting %.0f%% of their cycles, issuing %.0f%%)' % (100 * q['wait_frac'], 100 * q['issue_frac']) \
            if q['wait_frac'] > q['issue_frac'] else 'instruction issue (%.0f%% of wave cycles)' % (100 * q['issue_frac'])
    out = {
        'metric': 'env-steps/sec at N parallel envs, 1/2/4/8 MI355X; max |dq| vs PyBullet',
        'value': value,
        'unit': 'env-steps/s',
        'n_gpus': world,
        'steps': steps,
        'warmup': warmup,
        'ms_per_step': ms_per_step,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic: random actions U(-1,1)^7 (Philox, device), reset states from the reset path (%d distinct per GPU, tiled)' % pool,
        'config': {'workload': T['workload'] % E, 'task': name, 'envs_per_gpu': E, 'impairment': args.impairment,
                   'parallelism': 'env-sharded x%d' % world, 'env_groups': sim.env_groups(),
                   'stepping': 'per-step joins' if args.step_sync else ('rollout' if world == 1 else 'rollout x%d steps' % G)},
        'step_sync': step_sync,
        'roofline': {'bound': bound, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic, 'limiter': limiter,
                     'valu_busy': pmc.get('valu_busy_chip') if pmc else None,
                     'bytes_per_env_step': bpe, 'dominant_kernel': dominant,
                     'dominant_avg_ms': kernels[dominant]['avg_ms']},
        # fault bits only (bits 0-4); bit 5 (an env under the EPA budget) is informational
        'nan_or_overflow_envs': int(np.count_nonzero(flags & _lib.FLAGS_FAULT_MASK)),
    }
    # the long-form record (per-kernel tables, PMC issue shares, the scope of each figure) goes to
    # a side file, so that the printed line stays within the driver's record
    detail = {'task': name, 'value': value, 'ms_per_step': ms_per_step, 'roofline_fracs': fracs,
              'traffic_GBs': (traffic * 1e-9 / (step_kernel_ms * 1e-3)) if traffic else None,
              'sq_by_kernel': pmc.get('sq') if pmc else None, 'pmc_source': pmc['source'] if pmc else None,
              'layout_bytes_per_env_step': layout_bytes_per_env_step(L), 'step_kernel_ms': step_kernel_ms,
              'stream_ms_per_step': kern_ms, 'kernels': kernels, 'scope': SCOPE,
              'config': dict(out['config'], tremor_fraction=n_tremor / pool, global_envs=world * E,
                             substeps_per_env_step=T['substeps'], solver_iterations=T['iters'],
                             rollout_gather_every=G if world > 1 else None,
                             dist_backend=args.dist_backend if world > 1 else None),
              'flagged_envs_by_bit': {fname: int(np.count_nonzero(flags & (1 << b))) for b, fname in enumerate(
                  ('nan_or_singular_mass', 'contact_pool_full', 'aabb_pairs_full', 'shape_pairs_full', 'nc_rows_full', 'coop_capped'))},
              'reset_pool_sha1': pool_sha,
              # the contact load at the end of the run (contact points per env), which sets the
              # narrowphase, kernel-a and part-B work and traffic per env-step
              'contact_points_per_env': {'mean': float(St[:, L.S_TASK + L.T_NCP].mean()), 'max': float(St[:, L.S_TASK + L.T_NCP].max()),
                                         'envs_in_contact': float((St[:, L.S_TASK + L.T_NCP] > 0).mean())} if hasattr(L, 'T_NCP') else None}
    sim.close()
    if rank == 0 and world == 1 and cpu_seconds > 0:
        # the host threads this process may use: OMP_NUM_THREADS (the GPU box's CPU share, 16 per
        # GPU; os.cpu_count() reports the whole machine there), else every CPU of this host
        threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
        progress('%s: CPU baseline (%.0f s on %d threads)' % (name, cpu_seconds, threads))
        cb = cpu_baseline(name, md, A, cpu_seconds, max(1, threads), args.impairment)
        detail['cpu_baseline'] = cb
        out['cpu_baseline'] = {k: cb[k] for k in ('value', 'unit', 'cores', 'kind')}
        out['cpu_baseline']['sample'] = cb['short']
    elif rank == 0:
        out['cpu_baseline'] = None
    return out, detail


# the other single-GPU configs BASELINE.json names (configs[2], the PR2 variant of configs[3],
# configs[4] as the build-defined DressingJaco),
# timed after the headline in the same default run: extra keys of the one JSON line
OTHER_TASKS = ('ScratchItchPR2-v0', 'BedBathingPR2-v0', 'DressingJaco-v0')
OTHER_KEYS = ('value', 'ms_per_step', 'steps', 'step_sync', 'nan_or_overflow_envs', 'cpu_baseline')
ROOF_KEYS = ('frac', 'achieved', 'traffic', 'valu_busy', 'limiter', 'dominant_kernel', 'dominant_avg_ms')
# what each figure covers (kept out of the printed line, written to the detail file)
SCOPE = ('one env-step = one gym step of one env: 1 take_step + S x (pairs, narrowphase, a, b4) + 1 task launch '
         '(DressingJaco: one dress_step launch); achieved = algorithmic bytes of the step (SURVEY 8(d)) / summed launch '
         'durations, measured with HIP events on the sim stream in a separate pass with one env group; the timed loop runs '
         'env_groups concurrent launch sequences; traffic = PMC HBM bytes per step (FETCH_SIZE x 2 + WRITE_SIZE) and '
         'valu_busy = PMC VALU instructions x %.0f cycles / (%d SIMDs x %.1f GHz x ms_per_step), both from the task\'s committed '
         'rocprofv3 summary under profiles/' % (VALU_CYC, SIMDS, CLOCK_HZ / 1e9))
DETAIL_PATH = os.environ.get('AVR_BENCH_DETAIL', os.path.join(ROOT, 'gpurun_out', 'bench_detail.json'))


def compact_other(o):
    c = {k: o[k] for k in OTHER_KEYS}
    c['envs'] = o['config']['envs_per_gpu']
    c['roofline'] = {k: o['roofline'][k] for k in ROOF_KEYS}
    return c


def write_detail(details):
    try:
        os.makedirs(os.path.dirname(DETAIL_PATH), exist_ok=True)
        with open(DETAIL_PATH, 'w') as f:
            json.dump(details, f, indent=1)
        return os.path.relpath(DETAIL_PATH, ROOT)
    except OSError:
        return None


def policy_eval_run(name, E, steps=200):
    """enjoy_vr.py's evaluation loop (avr.policy_eval.evaluate: policy forward on the normalised
    obs, then AVRTorchVecEnv.step with the policy's fresh action tensor) for one `steps`-step trial
    in each of E envs: (evaluate's result, seconds including env creation and reset)."""
    import torch
    from avr import policy_eval as PE, _abi as ABI
    L = ABI.LAYOUTS[TASKS[name]['task']]
    torch.manual_seed(0)
    pol = PE.ActorCritic(L.OBS_DIM, L.ACT_DIM)
    rms = PE.RunningMeanStd((L.OBS_DIM,))
    t0 = time.perf_counter()
    r = PE.evaluate(name, pol, rms, n_envs=E, steps=steps, deterministic=False, device=0)
    return r, time.perf_counter() - t0


def policy_eval_bench(args):
    """policy_eval_run for 200 steps in each of --envs envs; env-steps/s of the stepping loop
    (env creation and reset excluded)."""
    import numpy as np
    name = args.task
    E = args.envs if args.envs is not None else TASKS[name].get('envs', 4096)
    r, total = policy_eval_run(name, E)
    out = {'metric': 'policy-eval env-steps/sec (avr.policy_eval.evaluate: enjoy_vr.py loop, fresh action tensor per step)',
           'value': E * 200 / r['loop_s'], 'unit': 'env-steps/s', 'n_gpus': 1, 'steps': 200, 'warmup': 0,
           'ms_per_step': r['loop_s'] / 200 * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
           'data': 'synthetic policy (random-init MLP actor-critic), stochastic actions',
           'config': {'workload': '%s, %d envs, policy evaluation harness' % (name, E), 'task': name, 'envs_per_gpu': E},
           'graph_captures': r['graph_captures'], 'policy_graph': r.get('policy_graph'), 'total_s_with_env_creation_and_reset': total,
           'mean_return': float(np.mean(r['returns']))}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--task', default='FeedingJaco-v0', choices=sorted(TASKS))
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--envs', type=int, default=None, help='envs per GPU (default: the config\'s, 4096; DressingJaco 2048)')
    ap.add_argument('--settle', type=int, default=None, help='reset settle frames (FeedingJaco 100, ScratchItch 0)')
    ap.add_argument('--gather-every', type=int, default=16)
    ap.add_argument('--step-sync', action='store_true',
                    help='time avr_step_random_device per step (env groups joined after every step) instead of rollouts')
    ap.add_argument('--sync-steps', type=int, default=20,
                    help='N=1 rollout runs: also time this many per-step API steps (--step-sync mode) on the same handle, '
                         'reported as step_sync (0 = skip)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--other-steps', type=int, default=20,
                    help='steps of each other single-GPU task (ScratchItchPR2, BedBathingPR2) timed after the FeedingJaco '
                         'headline at N=1 (extra keys of the JSON line; 0 = skip)')
    ap.add_argument('--reset-pool', type=int, default=None,
                    help='distinct host reset states, tiled over the envs (IK is host-side; FeedingJaco 1024, ScratchItch 128)')
    ap.add_argument('--facade', action='store_true',
                    help='time the gym facade (avr.env.AVRTorchVecEnv: device tensors, TimeLimit 200 with auto-reset) '
                         'instead of the bare step; --steps should span rollovers (e.g. 600)')
    ap.add_argument('--fresh-actions', action='store_true',
                    help='--facade: a new action tensor every step (as a policy returns), not one refilled tensor')
    ap.add_argument('--policy-eval', action='store_true',
                    help='time avr.policy_eval.evaluate (enjoy_vr.py harness: synthetic MLP policy, VecNormalize eval) at --envs '
                         'envs for 200 steps')
    ap.add_argument('--policy-eval-steps', type=int, default=200,
                    help='N=1 FeedingJaco runs: also time this many steps of the policy-evaluation loop (policy in the '
                         'loop, per-step observations), reported as policy_eval (0 = skip)')
    ap.add_argument('--dist-backend', default='nccl', choices=('nccl', 'gloo'),
                    help="torch.distributed backend for --gpus > 1: nccl (RCCL over xGMI, the product path); gloo only "
                         "rehearses the multi-rank flow where ranks share a GPU (rollouts gathered through host memory)")
    ap.add_argument('--impairment', default='random',
                    help="human impairment per env: 'random' is the tasks' own setting (feeding.py:175, scratch_itch.py:178)")
    args = ap.parse_args()
    if args.facade:
        return facade_bench(args)
    if args.policy_eval:
        return policy_eval_bench(args)

    import torch

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    gloo = args.dist_backend == 'gloo'
    if gloo:        # rehearsal: ranks may share the GPUs there are
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if gloo:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    cpu_s = 0.0 if args.no_cpu_baseline else args.cpu_seconds
    out, det = run_task(args.task, args, args.steps, args.warmup, world, rank, local, dist, gloo, dev, cpu_s)
    details = [det]
    if rank == 0 and world == 1 and args.task == 'FeedingJaco-v0' and args.other_steps > 0:
        out['other_tasks'] = {}
        for name in OTHER_TASKS:
            o, det = run_task(name, args, args.other_steps, args.warmup, world, rank, local, dist, gloo, dev, min(cpu_s, 5.0))
            out['other_tasks'][name] = compact_other(o)
            details.append(det)
    if rank == 0 and world == 1 and args.task == 'FeedingJaco-v0' and args.policy_eval_steps > 0:
        # the trainer-facing rate: a policy in the loop needs every step's observation (enjoy_vr.py:106-116)
        progress('FeedingJaco-v0: policy-eval loop')
        E = args.envs if args.envs is not None else TASKS[args.task].get('envs', 4096)
        r, _ = policy_eval_run(args.task, E, args.policy_eval_steps)
        out['policy_eval'] = {'value': E * args.policy_eval_steps / r['loop_s'], 'ms_per_step': r['loop_s'] / args.policy_eval_steps * 1e3,
                              'steps': args.policy_eval_steps, 'envs': E,
                              'loop': 'avr.policy_eval.evaluate: random-init MLP actor-critic forward + AVRTorchVecEnv.step per step'}
    if rank == 0:
        out['detail'] = write_detail(details)
        print(json.dumps(out, separators=(',', ':')), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
