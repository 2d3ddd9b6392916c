"""Window sharding across ranks (one process per GPU).

Windows of a clip are independent (lipsync_pipeline.py:500-575 slices its own
latents, faces and audio per window; DDIM with eta=0 carries no state across
windows), so a clip shards as whole windows.  Rank r owns the contiguous block
[r*per, (r+1)*per) of the clip's windows, per = ceil(n / W): the busiest rank holds
ceil(n / W) windows, as with any balanced split, and the rank-major result of the one
all-gather is already clip order -- no reordering copy after the exchange.  The only
exchange is that all-gather of the decoded frames after the loop, which puts every
window back in clip order on every rank.
"""
import math

import torch
import torch.distributed as dist


def world_and_rank(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def windows_per_rank(n_windows: int, world: int) -> int:
    """Windows of the busiest rank (the slab size every rank contributes to the gather)."""
    return math.ceil(n_windows / world) if n_windows > 0 else 0


def rank_windows(n_windows: int, world: int, rank: int):
    """Window indices owned by `rank`: a contiguous block of windows_per_rank windows
    (the last ranks hold fewer, or none, when n_windows % world != 0)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    per = windows_per_rank(n_windows, world)
    return list(range(min(n_windows, rank * per), min(n_windows, (rank + 1) * per)))


def gather_bytes(n_windows: int, world: int, window_bytes: int) -> int:
    """Bytes gather_windows allocates on the busiest rank for n_windows windows of
    window_bytes: the receive buffer (world * per windows) plus, when some rank holds
    fewer than per windows, that rank's zero-padded send slab.  Nothing when world == 1
    (the input is returned)."""
    if world == 1:
        return 0
    per = windows_per_rank(n_windows, world)
    pad = per if n_windows < world * per else 0
    return (world * per + pad) * window_bytes


def gather_windows(local: torch.Tensor, n_windows: int, group=None) -> torch.Tensor:
    """All-gather per-rank window outputs into clip order.

    local: (len(rank_windows(n_windows, W, r)), *S), the rank's block in order.
    Returns (n_windows, *S) on every rank -- a view of the one receive buffer, whose
    rank-major layout is clip order (no index_select copy).  One collective: the
    per-rank slabs are padded to windows_per_rank windows so a single
    all_gather_into_tensor (RCCL over xGMI) moves them."""
    world, rank = world_and_rank(group)
    n_local = len(rank_windows(n_windows, world, rank))
    if local.shape[0] != n_local:
        raise ValueError(f"rank {rank} holds {local.shape[0]} windows, expected {n_local}")
    if world == 1:
        return local
    per = windows_per_rank(n_windows, world)
    S = tuple(local.shape[1:])
    if n_local == per:
        buf = local.contiguous()
    else:
        buf = local.new_zeros((per,) + S)
        buf[:n_local] = local
    out = local.new_empty((world * per,) + S)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:  # gloo (CPU tests): same layout through the list form
        dist.all_gather(list(out.chunk(world)), buf, group=group)
    return out[:n_windows]
