#!/usr/bin/env python3
"""Benchmark: FeedingJaco-v0 env-steps/s on MI355X (BASELINE.json configs[1]).

One "step" = one gym step of every env (take_step + 5 x stepSimulation x 2 sub-steps + task
glue) = one launch of the gfx950 step kernel.  Synthetic random actions are drawn on the device
(Philox4x32-10 keyed by (seed=1001, global env id, step), examples/random_actions.py semantics).
Inputs are resident in HBM before the timed region; host buffers are not touched inside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E_per_gpu]
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


# algorithmic bytes per FeedingJaco env-step = persistent state read + written once
# (605 words, 2420 B each way) + read-only per-env params (144 B) + action in (28 B) + obs,
# reward, done, info out (116 B).
ALGO_BYTES_PER_ENV_STEP = 2420 * 2 + 144 + 28 + 116      # 5128


def layout_bytes_per_env_step(ABI):
    """What this build's state layout actually moves per env-step (state block in and out once,
    it stays in LDS across the 10 sub-steps; actions are generated on the device)."""
    return 2 * ABI.STATE_WORDS * 4 + (ABI.OBS_DIM + 1 + ABI.INFO_DIM) * 4 + 1


def cpu_baseline(md, A, RS, seconds, threads, impairment):
    """Oracle (the CPU restatement, fp64) on the host cores; bounded sample."""
    import numpy as np
    from oracle.oracle import Oracle
    from avr import _lib
    n = max(threads * 2, 8)
    S, _ = RS.batch_reset_states_fast(A, md, 1001, list(range(n)), impairment=impairment)
    o = Oracle(md, n)
    o.set_threads(threads)
    o.set_state(S)
    o.settle(100)
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = _lib.random_actions(1001, np.arange(n), steps)
        o.step(a)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds and steps >= 2:
            break
    return dict(value=n * steps / el, unit='env-steps/s', cores=threads, kind='port',
                sample='FeedingJaco-v0, %d envs x %d gym steps (%.1f s) after a 100-frame settle; fp64 oracle, OpenMP over envs' % (n, steps, el))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--envs', type=int, default=4096, help='envs per GPU')
    ap.add_argument('--settle', type=int, default=100)
    ap.add_argument('--gather-every', type=int, default=16)
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--reset-pool', type=int, default=1024,
                    help='distinct host reset states, tiled over the envs (IK is host-side)')
    ap.add_argument('--impairment', default='random',
                    help="human impairment per env: 'random' is FeedingJaco-v0's own setting (feeding.py:175)")
    args = ap.parse_args()

    import numpy as np
    import torch
    from avr import _abi as ABI, reset as RS, _lib
    from avr import dist as D

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)

    A = ABI.load_scene()
    md = ABI.ModelDesc(A)
    E = args.envs
    # reset pool: distinct initial states for global env ids; tiled if pool < E
    pool = min(args.reset_pool, E)
    base_id, _ = D.shard(E, rank)
    S_pool, meta = RS.batch_reset_states_fast(A, md, 1001, [base_id + i for i in range(pool)], impairment=args.impairment)
    n_tremor = sum(m['impairment'] == 'tremor' for m in meta)
    import hashlib
    pool_sha = hashlib.sha1(S_pool.astype(np.float32).tobytes()).hexdigest()[:12]
    S = np.tile(S_pool, ((E + pool - 1) // pool, 1))[:E]
    sim = _lib.Sim(md, E, device=local, seed=1001, env_offset=base_id)
    sim.set_state(S.astype(np.float32))
    sim.settle(args.settle)

    obs = torch.zeros(E, ABI.OBS_DIM, device=dev)
    rew = torch.zeros(E, device=dev)
    done = torch.zeros(E, dtype=torch.uint8, device=dev)
    info = torch.zeros(E, ABI.INFO_DIM, device=dev)
    ext = torch.cuda.ExternalStream(sim.stream(), device=dev)
    G = args.gather_every
    roll = torch.zeros(G, E, D.ROLL_WIDTH, device=dev)
    gathered = torch.zeros(world * G * E * D.ROLL_WIDTH, device=dev) if world > 1 else None

    def one_step(t, k):
        sim.step_random_device(t, obs.data_ptr(), rew.data_ptr(), done.data_ptr(), info.data_ptr())
        if world > 1:
            with torch.cuda.stream(ext):
                j = k % G
                D.pack_rollout(roll, j, obs, rew, info, done)
                if j == G - 1:
                    D.gather_rollouts(roll, out=gathered)

    for w in range(args.warmup):
        one_step(w, w)
    sim.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(ext)
    for k in range(args.steps):
        one_step(args.warmup + k, k)
    ev1.record(ext)
    sim.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    # per-kernel launch durations (HIP events between the launches of a step, on the sim
    # stream), from a separate short pass so the timed loop above carries no event overhead
    P = min(10, args.steps)
    sim.profile_kernels(True)
    for k in range(P):
        one_step(args.warmup + args.steps + k, k)
    kt = sim.kernel_times()
    sim.profile_kernels(False)
    kernels = {k: {'avg_ms': v[0] / max(v[1], 1), 'launches_per_step': v[1] / P, 'ms_per_step': v[0] / P} for k, v in kt.items()}
    step_kernel_ms = sum(v['ms_per_step'] for v in kernels.values())
    dominant = max(kernels, key=lambda k: kernels[k]['ms_per_step'])
    St = sim.get_state()
    flags = St[:, ABI.S_TASK + ABI.T_FLAGS].astype(np.int64)
    value = world * E * args.steps / el
    bpe = ALGO_BYTES_PER_ENV_STEP
    achieved = bpe * E / (step_kernel_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            # only a profile of this build's kernel set counts (kernels_per_step names them)
            if tj.get('envs') == E and set(tj.get('kernels_per_step', {})) == set(sim.kernel_kinds):
                traffic = tj.get('hbm_bytes_per_step')
        except Exception:
            traffic = None
    out = {
        'metric': 'env-steps/sec at N parallel envs, 1/2/4/8 MI355X; max |dq| vs PyBullet',
        'value': value,
        'unit': 'env-steps/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': el / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic: random actions U(-1,1)^7 (Philox, device), reset states from the host IK path (%d distinct per GPU, tiled)' % pool,
        'config': {'workload': 'FeedingJaco-v0, %d envs/GPU, rigid-only, random actions' % E, 'envs_per_gpu': E,
                   'impairment': args.impairment, 'tremor_fraction': n_tremor / pool,
                   'global_envs': world * E, 'substeps_per_env_step': 10, 'solver_iterations': 10,
                   'parallelism': 'env-sharded x%d' % world, 'rollout_gather_every': G if world > 1 else None,
                   'env_groups': sim.env_groups()},
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                     # the HBM roofline is the bound the contract names; the kernels sit far below
                     # it and are limited by VALU issue and memory latency
                     'limiter': 'valu-issue/latency' if achieved / HBM_PEAK_GBS < 0.05 else 'hbm',
                     'traffic_GBs': (traffic * 1e-9 / (step_kernel_ms * 1e-3)) if traffic else None,
                     'scope': 'one env-step = 1 take_step + 10 x (substep_pairs, narrowphase, coop, substep_a, substep_b4) + 1 task launch; '
                              'achieved = algorithmic bytes of the step / summed launch durations, measured in a separate pass with '
                              'one env group (per-kernel events need one stream); the timed loop runs env_groups concurrent launch '
                              'sequences, so its stream time per step is below the summed durations; '
                              'traffic = PMC HBM bytes of the step (profiles/pmc_traffic.json), traffic_GBs = traffic / summed launch durations',
                     'bytes_per_env_step': bpe, 'layout_bytes_per_env_step': layout_bytes_per_env_step(ABI),
                     'step_kernel_ms': step_kernel_ms, 'stream_ms_per_step': kern_ms,
                     'dominant_kernel': dominant, 'kernels': kernels},
        'nan_or_overflow_envs': int(np.count_nonzero(flags)),
        'flagged_envs_by_bit': {name: int(np.count_nonzero(flags & (1 << b))) for b, name in enumerate(
            ('nan_or_singular_mass', 'contact_pool_full', 'aabb_pairs_full', 'shape_pairs_full', 'nc_rows_full'))},
        'reset_pool_sha1': pool_sha,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1))
        threads = max(1, min(threads, 16))
        out['cpu_baseline'] = cpu_baseline(md, A, RS, args.cpu_seconds, threads, args.impairment)
    elif rank == 0:
        out['cpu_baseline'] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
