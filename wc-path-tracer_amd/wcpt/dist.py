"""Row-block sharding of a frame across ranks.

Every pixel is independent: its seed depends only on the global (x, y, frame) (pathTracer.comp:304) and the
accumulation is per pixel (:314-323), so rank r of N renders rows [r*H/N, (r+1)*H/N) of the global frame with
unchanged pixel indices and the union is bit-identical to a single-device render. The only exchange is the
gather of the row blocks to the presenting rank (RCCL over xGMI with the "nccl" backend; gloo on CPU).
"""
from __future__ import annotations


def row_block(height: int, world: int, rank: int) -> tuple[int, int]:
    """(y0, rows) of `rank`'s block; blocks differ by at most one row."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    y0 = rank * height // world
    y1 = (rank + 1) * height // world
    return y0, y1 - y0


def gather_frame(shard, height: int, world: int, rank: int, dst: int = 0):
    """Gather equal-size padded row blocks ([ceil(H/N), W, 4] tensors) to `dst` and assemble the frame.
    Returns the [H, W, 4] frame on dst and None elsewhere."""
    import torch
    import torch.distributed as dist

    if world == 1:
        y0, rows = row_block(height, 1, 0)
        return shard[:rows]
    parts = [torch.empty_like(shard) for _ in range(world)] if rank == dst else None
    dist.gather(shard, parts, dst=dst)
    if rank != dst:
        return None
    blocks = []
    for r in range(world):
        _, rows = row_block(height, world, r)
        blocks.append(parts[r][:rows])
    return torch.cat(blocks, dim=0)
