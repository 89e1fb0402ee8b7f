"""Gym facade on the GPU: FeedingEnv's reset/step contract (feeding.py:56-142, env.py:274-351)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_env_contract():
    from avr import env as E
    e = E.make('FeedingJaco-v0')
    obs = e.reset()
    assert obs.shape == (25,) and obs.dtype == np.float64 and np.all(np.isfinite(obs))
    obs, r, done, info = e.step(e.action_space.sample(np.random.default_rng(0)))
    assert obs.shape == (25,) and isinstance(r, float) and isinstance(done, bool)
    for k in ('total_force_on_human', 'task_success', 'action_robot_len', 'action_human_len', 'obs_robot_len', 'obs_human_len'):
        assert k in info
    assert info['action_robot_len'] == 7 and info['obs_robot_len'] == 25
    e.close()


def test_vec_env_time_limit_and_auto_reset():
    from avr import env as E, _lib
    n = 8
    v = E.AVRVecEnv('FeedingJaco-v0', n)
    o = v.reset()
    assert o.shape == (n, 25)
    for t in range(E.MAX_EPISODE_STEPS):
        o, r, d, info = v.step(_lib.random_actions(1001, np.arange(n), t))
        assert np.all(np.isfinite(o)) and np.all(np.isfinite(r))
        if t < E.MAX_EPISODE_STEPS - 1:
            assert not d.any()
    assert d.all()                                       # TimeLimit(200)
    assert 'terminal_observation' in info
    assert np.all(v.episode == 1)
    St = v.get_state()
    from avr import _abi as ABI
    assert np.all(St[:, ABI.S_TASK + ABI.T_ITER] == 0)  # auto-reset restarted the episodes
    assert np.all(v.flags() & 1 == 0)
    v.close()


def test_observation_layout():
    """obs = [spoon-torso(3), spoon quat(4), spoon-target(3), arm q(7), head-torso(3), head quat(4), force(1)]."""
    from avr import env as E, _abi as ABI
    v = E.AVRVecEnv('FeedingJaco-v0', 2)
    o = v.reset()
    St = v.get_state()
    q_arm = St[:, ABI.S_Q:ABI.S_Q + 7]
    assert np.allclose(o[:, 10:17], q_arm, atol=1e-6)
    assert np.allclose(np.linalg.norm(o[:, 3:7], axis=1), 1, atol=1e-5)
    assert np.allclose(np.linalg.norm(o[:, 20:24], axis=1), 1, atol=1e-5)
    sp = St[:, ABI.S_FREE:ABI.S_FREE + 3]
    tgt = St[:, ABI.S_TASK + ABI.T_TARGET:ABI.S_TASK + ABI.T_TARGET + 3]
    assert np.allclose(o[:, 7:10], sp - tgt, atol=1e-5)
    v.close()


def test_device_reset_ik_and_prefetch_over_two_rollovers():
    """Auto-reset with the device IK twice in a row: the second rollover uses the prefetched draws
    of episode 2, which equal a fresh reset_inputs of that episode (same states as computed
    synchronously)."""
    from avr import env as E, _lib, _abi as ABI, reset as RS
    n = 16
    v = E.AVRVecEnv('FeedingJaco-v0', n)
    v.reset()
    assert v.last_ik_ok.mean() > 0.8
    for ep in range(2):
        for t in range(E.MAX_EPISODE_STEPS):
            o, r, d, info = v.step(_lib.random_actions(1001, np.arange(n), ep * 1000 + t))
        assert d.all() and np.all(v.episode == ep + 1)
    St = v.get_state()
    Si, t7, init, q0, meta = RS.reset_inputs(v.A, v.md, v.seed, list(range(n)), impairment='random', episodes=[2] * n, stream='philox')
    # the human / bowl / task words of episode 2 are the host draws (before the settle moved nothing static)
    H = slice(ABI.S_HUMAN, ABI.S_HUMAN + 7 * 4)
    static = [m['impairment'] != 'tremor' for m in meta]
    assert np.allclose(St[static, H], Si[static, H], atol=1e-5)
    assert np.all(v.flags() == 0)
    v.close()


def test_torch_vec_env_matches_host_vec_env():
    import torch
    from avr import env as E, _lib
    n = 8
    h = E.AVRVecEnv('FeedingJaco-v0', n, auto_reset=False)
    g = E.AVRTorchVecEnv('FeedingJaco-v0', n, auto_reset=False)
    oh = h.reset()
    og = g.reset()
    assert isinstance(og, torch.Tensor) and og.is_cuda
    np.testing.assert_array_equal(oh, og.cpu().numpy())
    for t in range(5):
        a = _lib.random_actions(1001, np.arange(n), t)
        xh = h.step(a)
        xg = g.step(torch.from_numpy(a).cuda())
        assert np.array_equal(xg[2].cpu().numpy(), g.iteration >= g.max_steps)
        np.testing.assert_array_equal(xh[0], xg[0].cpu().numpy())
        np.testing.assert_array_equal(xh[1], xg[1].cpu().numpy())
        np.testing.assert_array_equal(xh[3]['total_force_on_human'], xg[3]['total_force_on_human'].cpu().numpy())
    h.close(); g.close()


def test_scratch_itch_facade():
    from avr import env as E
    e = E.make('ScratchItchPR2-v0')
    o = e.reset()
    assert o.shape == (30,) and np.all(np.isfinite(o))
    o, r, d, info = e.step(e.action_space.sample(np.random.default_rng(0)))
    assert o.shape == (30,) and info['obs_robot_len'] == 30 and info['action_robot_len'] == 7
    assert np.isfinite(r) and not d
    e.close()


def test_torch_vec_env_rollover_follows_device_done():
    """The host iteration mirror decides rollovers: at step 200 the device's done is set for every
    env, the terminal observation is the pre-reset one and the returned obs is the reset's."""
    import torch
    from avr import env as E
    n = 8
    g = E.AVRTorchVecEnv('FeedingJaco-v0', n)
    g.reset()
    gen = torch.Generator(device='cuda'); gen.manual_seed(3)
    a = torch.empty(n, 7, device='cuda')
    for t in range(E.MAX_EPISODE_STEPS):
        a.uniform_(-1, 1, generator=gen)
        o, r, d, info = g.step(a)
        assert bool(d.all()) == (t == E.MAX_EPISODE_STEPS - 1) and bool(d.any()) == bool(d.all())
    assert 'terminal_observation' in info and not torch.equal(info['terminal_observation'], o)
    assert np.all(g.iteration == 0) and np.all(g.episode == 1)
    np.testing.assert_array_equal(o.cpu().numpy(), g._obs)
    g.close()


def test_bed_bathing_facade():
    from avr import env as E
    e = E.make('BedBathingPR2-v0')
    o = e.reset()
    assert o.shape == (24,) and np.all(np.isfinite(o)) and o[23] == 0
    o, r, d, info = e.step(e.action_space.sample(np.random.default_rng(0)))
    assert o.shape == (24,) and info['obs_robot_len'] == 24 and info['action_robot_len'] == 7
    assert np.isfinite(r) and r < 0 and not d
    e.close()


def test_fresh_action_tensor_each_step_replays_one_graph():
    """A caller that hands a new action tensor every step (policy_eval.evaluate: the policy's
    output) replays one captured graph: the actions are copied into the handle's own buffer in
    stream order, so the graph key holds no caller action pointer (avr_capi.hip run_step).  The
    results are bit-identical to stepping with one persistent action tensor."""
    import torch
    from avr import env as E, _lib
    n = 8
    g1 = E.AVRTorchVecEnv('FeedingJaco-v0', n, auto_reset=False)
    g2 = E.AVRTorchVecEnv('FeedingJaco-v0', n, auto_reset=False)
    g1.reset(); g2.reset()
    keep = torch.empty(n, 7, device='cuda')
    c0 = g1.sim.graph_captures()
    for t in range(6):
        a = _lib.random_actions(1001, np.arange(n), t)
        fresh = torch.from_numpy(a).cuda() * 1.0          # a new device buffer every step
        keep.copy_(torch.from_numpy(a))
        x1 = g1.step(fresh)
        del fresh                                          # (its memory may be reused at once)
        x2 = g2.step(keep)
        np.testing.assert_array_equal(x1[0].cpu().numpy(), x2[0].cpu().numpy())
        np.testing.assert_array_equal(x1[1].cpu().numpy(), x2[1].cpu().numpy())
    assert g1.sim.graph_captures() - c0 <= 1, 'the step re-captured its graph for new action buffers'
    np.testing.assert_array_equal(g1.get_state(), g2.get_state())
    g1.close(); g2.close()


def test_graph_cache_keeps_several_output_keys():
    """Steps alternating between two output-buffer sets capture two graphs once each (a few keys
    are cached) and match direct launches bit for bit."""
    import torch
    from avr import env as E, _lib
    n = 8
    v = E.AVRVecEnv('FeedingJaco-v0', n, auto_reset=False)
    v.reset()
    S0 = v.get_state()
    sim = v.sim
    outs = [(torch.zeros(n, 25, device='cuda'), torch.zeros(n, device='cuda'), torch.zeros(n, dtype=torch.uint8, device='cuda'),
             torch.zeros(n, 2, device='cuda')) for _ in range(2)]
    c0 = sim.graph_captures()
    for t in range(6):
        o = outs[t % 2]
        sim.step_random_device(t, *(x.data_ptr() for x in o))
    sim.sync()
    assert sim.graph_captures() - c0 == 2
    S_graph = sim.get_state()
    sim.set_state(S0)
    for t in range(6):
        sim.step(_lib.random_actions(1001, np.arange(n), t))
    np.testing.assert_array_equal(S_graph, sim.get_state())
    v.close()


def test_negative_step_index_rejected():
    from avr import env as E
    v = E.AVRVecEnv('FeedingJaco-v0', 2, auto_reset=False)
    with pytest.raises(RuntimeError, match='step index'):
        v.sim.step_random_device(-1)
    v.close()


def test_calls_keep_the_callers_current_device():
    """Every C-API entry point runs on its handle's device and restores the caller's current
    device (lazily allocated scratch lands on the handle's GPU).  With two GPUs: a handle on
    device 1 used while device 0 is current."""
    import torch
    from avr import env as E
    ndev = torch.cuda.device_count()
    dev = 1 if ndev > 1 else 0
    torch.cuda.set_device(0)
    v = E.AVRVecEnv('FeedingJaco-v0', 4, device=dev, auto_reset=False)
    assert torch.cuda.current_device() == 0
    v.reset()                                # device IK: lazily allocated scratch
    assert torch.cuda.current_device() == 0
    assert np.all(v.flags() & 1 == 0)
    q, _ = v.sim.get_q()
    assert np.all(np.isfinite(q)) and torch.cuda.current_device() == 0
    v.close()
