"""Row-block sharding of a frame across ranks.

Every pixel is independent: its seed depends only on the global (x, y, frame) (pathTracer.comp:304) and the
accumulation is per pixel (:314-323), so rank r of N renders rows [r*H/N, (r+1)*H/N) of the global frame with
unchanged pixel indices and the union is bit-identical to a single-device render. The only exchange is the
gather of the row blocks to the presenting rank (RCCL over xGMI with the "nccl" backend; gloo on CPU).

The gather can carry RGB only: the kernel writes alpha = 1.0 for every pixel (pathTracer.comp:323,
`vec4(acc, 1)`), so the presenting rank restores it and the frame is bit-identical with 3/4 of the bytes on
the wire.
"""
from __future__ import annotations


def row_block(height: int, world: int, rank: int) -> tuple[int, int]:
    """(y0, rows) of `rank`'s block; blocks differ by at most one row."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    y0 = rank * height // world
    y1 = (rank + 1) * height // world
    return y0, y1 - y0


def row_stripes(height: int, world: int, rank: int, stripe: int = 0) -> tuple[int, int]:
    """(y_first, rows) of `rank` under interleaved stripes of `stripe` rows (include/wcpt.h wcpt_row_stripes): rank r
    takes stripes r, r + world, ... of ceil(height / stripe); only the frame's last stripe can be short. stripe 0 is
    row_block."""
    if stripe == 0:
        return row_block(height, world, rank)
    if world < 1 or not 0 <= rank < world or stripe & (stripe - 1):
        raise ValueError(f"bad rank {rank} of {world} / stripe {stripe}")
    total = -(-height // stripe)
    count = (total - 1 - rank) // world + 1 if total > rank else 0
    rows = count * stripe
    if count and (total - 1 - rank) % world == 0 and height % stripe:
        rows -= stripe - height % stripe
    return rank * stripe, rows


def frame_rows(height: int, world: int, rank: int, stripe: int = 0) -> list[int]:
    """The frame rows of `rank`'s local rows 0, 1, ... (row_map.h: y_first + ly + (ly // stripe) * (period - stripe))."""
    y0, rows = row_stripes(height, world, rank, stripe)
    if stripe == 0:
        return list(range(y0, y0 + rows))
    gap = world * stripe - stripe
    return [y0 + ly + (ly // stripe) * gap for ly in range(rows)]


def pack_rgb(block):
    """The RGB channels of a [rows, W, 4] block as a contiguous [rows, W, 3] tensor (alpha is always 1.0)."""
    return block[..., :3].contiguous()


def assemble(parts, height: int, world: int):
    """Frame [H, W, 4] from the ranks' padded row blocks ([ceil(H/N), W, 4] or RGB-only [.., 3])."""
    import torch

    blocks = [parts[r][:row_block(height, world, r)[1]] for r in range(world)]
    frame = torch.cat(blocks, dim=0)
    if frame.shape[-1] == 3:
        alpha = torch.ones(frame.shape[:-1] + (1,), dtype=frame.dtype, device=frame.device)
        frame = torch.cat([frame, alpha], dim=-1)
    return frame


def gather_frame(shard, height: int, world: int, rank: int, dst: int = 0, rgb_only: bool = False):
    """Gather equal-size padded row blocks ([ceil(H/N), W, 4] tensors) to `dst` and assemble the frame; with
    rgb_only the blocks travel as RGB and alpha (always 1.0) is restored on dst.
    Returns the [H, W, 4] frame on dst and None elsewhere."""
    import torch
    import torch.distributed as dist

    if world == 1:
        y0, rows = row_block(height, 1, 0)
        return shard[:rows]
    send = pack_rgb(shard) if rgb_only else shard
    parts = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, parts, dst=dst)
    if rank != dst:
        return None
    return assemble(parts, height, world)
