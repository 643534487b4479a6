"""Multi-GPU sharding of the pair / query batch.

Every (start, goal) pair and every planner query is independent and the weights (2.3 MB)
and B tables are replicated, so each rank evaluates a contiguous slice
[lo, hi) of the batch with no data-path collective.  The one exchange is the optional
all-gather of per-rank outputs (τ+∇τ rows or planner paths) that hands every rank the
whole result: `torch.distributed` over RCCL ("nccl" backend = RCCL over xGMI on ROCm),
or gloo for the CPU tests.
"""
import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torchrun environment (1-process default)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend=None, device=None, force=False):
    """Initialise the default process group when launched with WORLD_SIZE > 1 (or, with
    `force`, also at world size 1: a one-rank RCCL communicator, so the collective path can be
    exercised and timed on a single GPU).

    backend "nccl" is RCCL on ROCm (over xGMI inside a node); pass the rank's HIP `device`
    (already made current) so the communicator binds to it.  Returns (rank, world_size) as
    the process group reports them, which must equal the environment's."""
    rank, ws, _ = world()
    if (ws > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {"device_id": device} if (device is not None and backend == "nccl") else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=ws, **kw)
    if dist.is_initialized():
        got = (dist.get_rank(), dist.get_world_size())
        if got != (rank, ws):
            raise RuntimeError("process group reports rank/world %s, environment %s"
                               % (got, (rank, ws)))
    return rank, ws


def shard_range(n, rank, world_size):
    """Contiguous balanced slice [lo, hi) of n items for `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n, world_size)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def all_gather_rows(local, n_total, group=None, force=False):
    """Concatenate every rank's row-slice (shard_range order) into the full (n_total, ...)
    tensor on every rank.  Shards are padded to the largest one so the collective is a
    single all_gather_into_tensor.  At world size 1 the local block is returned as is, unless
    `force` (and a process group exists): then the collective runs anyway (a copy through
    RCCL), which is how the single-GPU tests and bench exercise and time the RCCL path."""
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    if ws == 1 and not (force and dist.is_initialized()):
        return local
    chunk = -(-n_total // ws)
    if n_total == chunk * ws:                 # equal shards: gather straight into the result
        if local.shape[0] != chunk:
            raise ValueError("rank holds %d rows, expected %d" % (local.shape[0], chunk))
        out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    pad = torch.zeros((chunk,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((chunk * ws,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    pieces = []
    for r in range(ws):
        lo, hi = shard_range(n_total, r, ws)
        pieces.append(out[r * chunk:r * chunk + (hi - lo)])
    return torch.cat(pieces)
