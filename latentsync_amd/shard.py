"""Window sharding across ranks (one process per GPU).

Windows of a clip are independent (lipsync_pipeline.py:500-575 slices its own
latents, faces and audio per window; DDIM with eta=0 carries no state across
windows), so a clip shards as whole windows: rank r runs windows r, r+W, r+2W, ...
(round-robin keeps ranks within one window of each other on ragged counts).
The only exchange is one all-gather of the decoded frames after the loop, which
puts every window back in clip order on every rank.
"""
import math

import torch
import torch.distributed as dist


def world_and_rank(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def rank_windows(n_windows: int, world: int, rank: int):
    """Window indices owned by `rank` (round-robin)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return list(range(rank, n_windows, world))


def gather_windows(local: torch.Tensor, n_windows: int, group=None) -> torch.Tensor:
    """All-gather per-rank window outputs into clip order.

    local: (len(rank_windows(n_windows, W, r)), *S) in the order rank_windows
    returns.  Returns (n_windows, *S) on every rank.  One collective: the
    per-rank slabs are padded to ceil(n_windows / W) windows so a single
    all_gather_into_tensor (RCCL over xGMI) moves them."""
    world, rank = world_and_rank(group)
    n_local = len(rank_windows(n_windows, world, rank))
    if local.shape[0] != n_local:
        raise ValueError(f"rank {rank} holds {local.shape[0]} windows, expected {n_local}")
    if world == 1:
        return local
    per = math.ceil(n_windows / world)
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
    order = torch.tensor([(i % world) * per + i // world for i in range(n_windows)], device=out.device)
    return out.index_select(0, order)
