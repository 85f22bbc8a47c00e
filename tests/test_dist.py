"""Multi-rank path on CPU (gloo, world_size 2 and 3): row-block partition + gather reproduce the single-rank
frame bit for bit. The per-rank renderer here is the CPU oracle; on GPUs bench.py runs the
same partition with libwcpt.so per rank and the gather over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wcpt.dist import gather_frame, row_block


def test_row_block_partition():
    for H in (1, 7, 135, 1080, 2160, 1081):
        for N in (1, 2, 3, 4, 8):
            if N > H:
                continue
            blocks = [row_block(H, N, r) for r in range(N)]
            assert blocks[0][0] == 0
            assert sum(r for _, r in blocks) == H
            for (a, ra), (b, _) in zip(blocks, blocks[1:]):
                assert a + ra == b
            assert max(r for _, r in blocks) - min(r for _, r in blocks) <= 1
    assert row_block(1080, 8, 7) == (945, 135)
    with pytest.raises(ValueError):
        row_block(10, 2, 2)


def test_row_stripes_partition_the_frame():
    """Interleaved row stripes (include/wcpt.h wcpt_row_stripes, its Python mirror and the row map
    of row_map.h): for every height, rank count and stripe size the ranks' frame rows cover the frame exactly once, the
    library's split equals the mirror's, and every rank's rows fit the map's closed form."""
    import ctypes as C
    from wcpt import _lib
    from wcpt.dist import frame_rows, row_stripes
    y0, rows = C.c_uint32(), C.c_uint32()
    for H in (1, 7, 17, 45, 135, 1080, 1081, 2160):
        for N in (1, 2, 3, 4, 7, 8):
            for S in (0, 1, 2, 8, 16, 64):
                stripes = -(-H // S) if S else H
                if stripes < N:
                    continue
                seen = []
                for r in range(N):
                    assert _lib.lib.wcpt_row_stripes(H, N, r, S, C.byref(y0), C.byref(rows)) == 0
                    assert (y0.value, rows.value) == row_stripes(H, N, r, S)
                    fr = frame_rows(H, N, r, S)
                    assert len(fr) == rows.value > 0 and fr == sorted(fr)
                    seen += fr
                assert sorted(seen) == list(range(H)), (H, N, S)
    # 1080 rows, 8 ranks, stripes of 8: 135 stripes -> ranks 0-6 hold 17 (136 rows), rank 7 holds 16 (128 rows)
    assert [row_stripes(1080, 8, r, 8)[1] for r in range(8)] == [136] * 7 + [128]
    assert _lib.lib.wcpt_row_stripes(100, 2, 0, 3, C.byref(y0), C.byref(rows)) != 0   # not a power of two
    with pytest.raises(ValueError):
        row_stripes(100, 2, 0, 6)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, out_path, rgb_only=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "wc-path-tracer_amd"), os.path.join(root, "oracle")]
    import oracle
    from wcpt import scene as wscene
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = wscene.generate("cornell")
    y0, rows = row_block(H, world, rank)
    img, _ = oracle.render_scene(s, W, H, max_bounce=4, frame=3, y0=y0, rows=rows)
    shard = torch.zeros((-(-H // world), W, 4), dtype=torch.float32)
    shard[:rows] = torch.from_numpy(img)
    frame = gather_frame(shard, H, world, rank, rgb_only=rgb_only)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rgb_only", [(2, False), (3, False), (2, True), (3, True)])
def test_gather_reassembles_frame(tmp_path, world, rgb_only):
    """Both wire formats (RGBA, and RGB with alpha restored on the presenting rank) give the 1-rank frame."""
    import oracle
    from wcpt import scene as wscene
    W, H = 48, 37
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, out, rgb_only), nprocs=world, join=True)
    full, _ = oracle.render_scene(wscene.generate("cornell"), W, H, max_bounce=4, frame=3)
    assert np.array_equal(np.load(out), full)


@pytest.mark.parametrize("height", [1, 7, 8, 135, 1080, 2160, 4099])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 8])
def test_row_block_bookkeeping_matches_across_hosts(height, n):
    """The C-ABI split (wcpt_row_block, which wcpt_group_create_screen uses for its ranks) equals the Python host's
    (wcpt.dist.row_block, which bench.py's ranks use), and the blocks tile the frame exactly: contiguous, disjoint,
    in rank order, differing by at most one row."""
    import ctypes as C
    import wcpt
    from wcpt.dist import row_block
    if height < n:
        pytest.skip("a group needs at least one row per rank")
    y0, rows = C.c_uint32(), C.c_uint32()
    nxt, sizes = 0, []
    for r in range(n):
        assert wcpt.lib.wcpt_row_block(height, n, r, C.byref(y0), C.byref(rows)) == 0
        assert (y0.value, rows.value) == row_block(height, n, r)
        assert y0.value == nxt
        nxt += rows.value
        sizes.append(rows.value)
    assert nxt == height and max(sizes) - min(sizes) <= 1
    assert wcpt.lib.wcpt_row_block(height, n, n, C.byref(y0), C.byref(rows)) == -1000
    assert wcpt.lib.wcpt_row_block(height, 0, 0, C.byref(y0), C.byref(rows)) == -1000
