"""N>1 path on CPU: world_size-2/3 gloo groups run the tile assignment + all_gather + un-interleave of
halogen.distributed on synthetic tiles whose values encode their pixel coordinates, and the gathered image
must equal the directly-computed one exactly."""
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
    if rank == 0:
        q.put(img.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("n,W,H", [(2, 64, 48), (3, 70, 30)])
def test_gloo_tile_gather(n, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, W, H, q)) for r in range(n)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(img, _pixel_value(xx, yy))


def test_untile_single_rank():
    W, H = 24, 16
    t = _local_tiles(0, 1, W, H)
    img = hd.untile(t.view(1, -1, 64, 4), 1, W, H).numpy()
    yy, xx = np.mgrid[0:H, 0:W]
    assert np.array_equal(img, _pixel_value(xx, yy))
