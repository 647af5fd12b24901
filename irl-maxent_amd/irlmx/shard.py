"""Instance sharding across GPUs (one process per GPU, torch.distributed).

Independent instances split into contiguous blocks, one block per rank, with
no collective on the data path: each rank builds its own
instances' tables on its device and runs them; only timing (max over ranks)
and, when a caller wants all results on one rank, a final gather cross ranks.
"""

import numpy as np
import torch
import torch.distributed as dist


def shard_range(n_total, world, rank):
    """Contiguous [lo, hi) block of instances owned by `rank` (sizes differ by at most 1)."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_over_ranks(x, device=None):
    """Max of a float over all ranks (the bench's timing reduction)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    backend = dist.get_backend()
    dev = device if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_rank0(local, n_total):
    """Concatenate every rank's [n_local, ...] result on rank 0 (CPU tensors; None elsewhere)."""
    local = local.detach().cpu()
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    world, rank = dist.get_world_size(), dist.get_rank()
    parts = [None] * world if rank == 0 else None
    dist.gather_object(local, parts, dst=0)
    if rank != 0:
        return None
    out = torch.cat(parts, dim=0)
    assert out.shape[0] == n_total
    return out


def instance_slips(ids, n_total):
    """The bench's per-instance slip probabilities: p_slip_b = 0.1 + 0.2 * b / B."""
    return 0.1 + 0.2 * np.asarray(ids, dtype=np.float64) / n_total
