"""Multi-GPU plumbing for the vectorised envs.

Envs are independent units: GPU `rank` owns the contiguous block of global env ids
[rank * E, (rank + 1) * E).  Reset randomness and synthetic actions are keyed by the global env
id, so a run's per-env results do not depend on the GPU count.  The only data-path collective is
the rollout collection: each rank packs its (obs, reward, info, done) rows for G steps and one
all_gather_into_tensor (RCCL over xGMI on MI355X; gloo in the CPU tests) concatenates them in
rank order = global env order.
"""
import torch

from . import _abi as ABI

ROLL_WIDTH = ABI.OBS_DIM + 1 + ABI.INFO_DIM + 1   # FeedingJaco: obs, reward, info, done


def roll_width(obs_dim):
    """Columns of one env's rollout row: obs, reward, info, done."""
    return obs_dim + 1 + ABI.INFO_DIM + 1


def shard(envs_per_rank, rank):
    """(global id of the rank's first env, count)."""
    return rank * envs_per_rank, envs_per_rank


def pack_rollout(roll, j, obs, rew, info, done):
    """roll[j] (E, W) <- one step of outputs (device tensors, no host sync); W = roll_width(obs_dim)."""
    od = obs.shape[1]
    roll[j, :, :od] = obs
    roll[j, :, od] = rew
    roll[j, :, od + 1:od + 1 + ABI.INFO_DIM] = info
    roll[j, :, -1] = done.to(roll.dtype)


def pack_rollout_stacked(roll, obs, rew, info, done, m):
    """roll[:m] (m, E, W) <- m steps of stacked outputs ([G, E, ...] device tensors); the rows past m
    keep their previous contents (a short last chunk)."""
    od = obs.shape[2]
    roll[:m, :, :od] = obs[:m]
    roll[:m, :, od] = rew[:m]
    roll[:m, :, od + 1:od + 1 + ABI.INFO_DIM] = info[:m]
    roll[:m, :, -1] = done[:m].to(roll.dtype)


def gather_rollouts(roll, out=None, group=None):
    """All-gather every rank's roll (G, E, W) -> (G, world*E, W) in global env order."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    G, E, W = roll.shape
    flat = torch.empty(world * G * E * W, dtype=roll.dtype, device=roll.device) if out is None else out
    dist.all_gather_into_tensor(flat, roll.contiguous().reshape(-1), group=group)
    return flat.reshape(world, G, E, W).permute(1, 0, 2, 3).reshape(G, world * E, W)
