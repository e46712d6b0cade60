"""Multi-GPU helpers: one process per GPU, environments sharded by global id.

Environments are independent, so the step itself has no exchange: rank r owns the contiguous
global ids [r * n, (r + 1) * n) (``env_base``) and every random draw is keyed by the global id,
which makes results independent of the number of GPUs.  The only collective is OPTIONAL and off
the data path: ``all_gather_outputs`` packs (tip x/y/z, done | success << 1 | (reward = -1) << 2)
into 16 B per env and all-gathers it over RCCL (backend "nccl" on ROCm, xGMI between the GPUs of a node) for a
single-process trainer that wants every shard's outputs.
"""
import os

PACK_WIDTH = 4   # float32 words per env: tip x, y, z, flags (done | success << 1 | (reward = -1) << 2)


def world():
    """(rank, world_size, local_rank) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(num_envs_per_rank, rank):
    """Global id of this rank's first environment."""
    return int(num_envs_per_rank) * int(rank)


def pack_step_outputs(achieved_goal, reward, done, success, out=None):
    """[n, 4] float32 tensor: tip (3, f64 -> f32), done | success << 1 | (reward = -1) << 2.
    The env's reward is sparse, -1 or 0 (ctr_reach_env.py:160-170), so one bit carries it."""
    import torch
    n = achieved_goal.shape[0]
    if out is None:
        out = torch.empty((n, PACK_WIDTH), dtype=torch.float32, device=achieved_goal.device)
    out[:, 0:3] = achieved_goal
    out[:, 3] = done.to(torch.float32) + 2.0 * success.to(torch.float32) + 4.0 * (reward < 0).to(torch.float32)
    return out


def unpack_step_outputs(packed):
    """(tip [n, 3] f32, reward [n] f32, done [n] bool, success [n] bool) of packed rows."""
    import torch
    flags = packed[:, 3].round().to(torch.int32)
    reward = ((flags >> 2) & 1).to(torch.float32).neg_().add_(0.0)     # -1 or +0 (not -0)
    return packed[:, 0:3], reward, (flags & 1).bool(), (flags & 2).bool()


def all_gather_outputs(packed, group=None, async_op=False):
    """All-gather every rank's packed [n, 4] block into [world * n, 4] (rank-major = global id
    order).  Uses all_gather_into_tensor: one RCCL ring/tree call for the whole step.

    async_op=True returns (out, work): the collective runs on RCCL's own stream, ordered after
    the packing on the current stream, so the next ctr_step overlaps it; ``work.wait()`` before
    reading ``out``, and keep ``packed`` unchanged until then."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    if packed.is_cuda and dist.get_backend(group) == "gloo":
        # gloo rehearsal of the RCCL path (several ranks on one GPU): gather host copies
        host = packed.cpu()
        out = torch.empty((ws * packed.shape[0], packed.shape[1]), dtype=packed.dtype)
        dist.all_gather_into_tensor(out, host, group=group)
        out = out.to(packed.device)
        return (out, _DoneWork()) if async_op else out
    out = torch.empty((ws * packed.shape[0], packed.shape[1]), dtype=packed.dtype, device=packed.device)
    work = dist.all_gather_into_tensor(out, packed.contiguous(), group=group, async_op=async_op)
    return (out, work) if async_op else out


class _DoneWork(object):
    """A completed collective (the synchronous gloo rehearsal path)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


def max_over_ranks(value, device=None, group=None):
    """Max of a python float over ranks (bench timing); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
