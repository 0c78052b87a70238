"""N>1 path on CPU: world_size-2/3 gloo groups run the tile assignment + all_gather + un-interleave of
halogen.distributed on synthetic tiles whose values encode their pixel coordinates, and the gathered image
must equal the directly-computed one exactly.  The un-interleave is hg_comm_assemble_host, the host twin of the C-ABI
gather's device assembly (same csrc/hg_tiling.h mapping); it is also checked directly for N = 1..8 with ragged tile
shares and odd image sizes, against an independent restatement of the tiling."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from halogen import distributed as hd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pixel_value(x, y):
    return np.stack([x, y, x * 1000.0 + y, np.ones_like(x)], axis=-1).astype(np.float32)


def _local_tiles(rank, n, W, H):
    tx, ty = hd.tiles_xy(W, H)
    n_local = hd.local_tile_count(tx * ty, rank, n)
    out = np.zeros((n_local, 64, 4), np.float32)
    for lt in range(n_local):
        g = rank + lt * n
        gx, gy = g % tx, g // tx
        lane = np.arange(64)
        out[lt] = _pixel_value(gx * 8 + lane % 8, gy * 8 + lane // 8)
    return torch.from_numpy(out)


def _worker(rank, n, port, W, H, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=n)
    img = hd.gather_tiles(_local_tiles(rank, n, W, H), rank, n, W, H)
    dev = hd.gather_tiles(_local_tiles(rank, n, W, H), rank, n, W, H, on_device=True)  # bench.py's timed form
    if rank == 0:
        q.put((img, dev.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,W,H", [(2, 64, 48), (3, 70, 30)])
def test_gloo_tile_gather(n, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, W, H, q)) for r in range(n)]
    for p in procs:
        p.start()
    img, dev = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(img, _pixel_value(xx, yy))
    assert np.array_equal(dev, _pixel_value(xx, yy))  # assembled where the gather landed, through pixel_index


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("W,H", [(64, 48), (70, 30), (9, 7), (240, 8)])
def test_pixel_index_equals_host_assembly(n, W, H):
    """The device-side assembly's index map reproduces hg_comm_assemble_host on ragged shares and odd sizes."""
    tx, ty = hd.tiles_xy(W, H)
    max_local = hd.local_tile_count(tx * ty, 0, n)
    slabs = np.random.default_rng(n * 1000 + W).standard_normal((n, max_local, 64, 4)).astype(np.float32)
    want = hd.untile(slabs, n, W, H)
    idx = hd.pixel_index(n, max_local, W, H, torch.device("cpu"))
    got = torch.from_numpy(slabs).view(-1, 4).index_select(0, idx).view(H, W, 4).numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_untile_single_rank():
    W, H = 24, 16
    t = _local_tiles(0, 1, W, H)
    img = hd.untile(t.view(1, -1, 64, 4), 1, W, H)
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(img, _pixel_value(xx, yy))


def _slabs(n, W, H):
    """Every rank's local tiles as the C-ABI packs them (rank r: global tiles r, r + n, ...), padded to rank 0's
    count: the staging layout of hg_comm_gather / the all_gather of gather_tiles."""
    tx, ty = hd.tiles_xy(W, H)
    total = tx * ty
    slab_tiles = hd.local_tile_count(total, 0, n)
    slabs = np.full((n, slab_tiles, 64, 4), np.nan, np.float32)
    for r in range(n):
        tiles = _local_tiles(r, n, W, H).numpy()
        assert tiles.shape[0] == hd.local_tile_count(total, r, n)
        slabs[r, : tiles.shape[0]] = tiles
    return slabs


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("W,H", [(64, 48), (70, 30), (1, 1), (9, 17), (123, 61), (8, 200), (240, 8)])
def test_assemble_host_mapping(n, W, H):
    """hg_comm_assemble_host (the device gather's mapping, csrc/hg_tiling.h) puts every pixel where the tiling says:
    ragged shares (total tiles not a multiple of N, ranks with no tile at all when N > tiles), partial edge tiles, and
    padded slab entries never read (they hold NaN)."""
    from halogen import abi

    img = abi.assemble_host(_slabs(n, W, H), W, H, n)
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(img, _pixel_value(xx, yy)), (n, W, H)


def test_assemble_host_counts_and_errors():
    """Rank shares: rank r of n holds ceil((T - r) / n) tiles (hg_rank_tiles); slabs smaller than rank 0's share or
    with the wrong rank count are refused loudly."""
    from halogen import abi

    for total in (1, 7, 8, 9, 32400, 32401):
        for n in range(1, 9):
            counts = [hd.local_tile_count(total, r, n) for r in range(n)]
            assert sum(counts) == total and max(counts) - min(counts) <= 1 and counts == sorted(counts, reverse=True)
    slabs = _slabs(3, 70, 30)
    with pytest.raises(abi.HalogenError):
        abi.assemble_host(slabs[:, :-1], 70, 30, 3)
    with pytest.raises(ValueError):
        abi.assemble_host(slabs, 70, 30, 2)
