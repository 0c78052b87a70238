"""Multi-GPU gather behind the C-ABI (hg_comm_*) on one GPU.

Two (three) contexts on device 0 play ranks 0/1 (0/1/2) of an N-rank render: each renders its interleaved 8x8
tiles with the frame-parallel split forced on (several waves per tile, colours blended in frame order, the path that
showed the round-1 zero-block observation), hg_comm_init_all joins them (contexts sharing a device take the
in-process device-copy transport; RCCL refuses two ranks on one GPU), hg_comm_gather assembles the image on the
root's device.  The merged image must be bit-equal to a 1-rank render and every pixel written (alpha == 1).
A 1-rank communicator through hg_comm_init_rank exercises the RCCL transport's set-up and assembly on this GPU."""
import numpy as np
import pytest

import cases
from halogen import abi

from test_gpu_parity import assert_bitwise, gpu_render


def _rank_ctx(packed, params, cube, rank, n, split, kernel):
    ctx = abi.Context(0)
    ctx.set_option(abi.HG_OPT_FRAME_SPLIT, split)
    ctx.set_option(abi.HG_OPT_KERNEL, kernel)
    ctx.upload_scene(packed)
    if cube is not None:
        ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    ctx.resize(W, H)
    ctx.set_tiling(rank, n)
    ctx.set_params(params)
    return ctx


@pytest.mark.gpu
@pytest.mark.parametrize("n_ranks", [2, 3])
@pytest.mark.parametrize("name,kernel", [("c1_64", abi.HG_KERNEL_MEGA_REGEN), ("dragon1_64x36", abi.HG_KERNEL_MEGA_STREAM),
                                         ("glass_64x36", abi.HG_KERNEL_AUTO)])
def test_gpu_comm_gather_equals_one_rank(gpu, name, kernel, n_ranks):
    packed, params, cube, _, acc = cases.setup(name)
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    frames = [5, 3]  # two renders, a gather after each: the second gather re-uses the staging buffers
    ctxs = [_rank_ctx(packed, params, cube, r, n_ranks, 3, kernel) for r in range(n_ranks)]
    comm = abi.Comm.all(ctxs)
    assert comm.transport == abi.HG_COMM_PEER
    try:
        done = 0
        for k, nf in enumerate(frames):
            for c in ctxs:
                c.render(nf, acc)
            done += nf
            root = k % n_ranks
            comm.gather(root)
            img = comm.readback(W, H)
            assert np.all(img[..., 3] == 1.0), f"{int((img[..., 3] != 1.0).sum())} pixels not written"
            with abi.Context(0) as one:
                one.set_option(abi.HG_OPT_FRAME_SPLIT, 1)
                ref, _ = gpu_render(packed, params, done, acc, cube, ctx=one, kernel="auto")
            assert_bitwise(img, ref, f"{name} {n_ranks} ranks after {done} frames (root {root})")
    finally:
        comm.close()
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_gpu_comm_rccl_single_rank(gpu):
    """hg_comm_unique_id + hg_comm_init_rank (the one-process-per-GPU form bench.py uses at N > 1) with one rank:
    RCCL communicator set-up, the (empty) group call and the root assembly on this GPU."""
    packed, params, cube, frames, acc = cases.setup("c1_64")
    ctx = _rank_ctx(packed, params, cube, 0, 1, 0, abi.HG_KERNEL_AUTO)
    try:
        ctx.render(frames, acc)
        comm = abi.Comm.rank(ctx, 1, abi.comm_unique_id(), 0)
        assert comm.transport == abi.HG_COMM_RCCL
        comm.gather(0)
        img = comm.readback(64, 64)
        assert_bitwise(img, ctx.readback(64, 64), "1-rank RCCL gather")
        comm.close()
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_comm_errors_are_loud(gpu):
    packed, params, cube, frames, acc = cases.setup("c1_64")
    a = _rank_ctx(packed, params, cube, 0, 2, 0, abi.HG_KERNEL_AUTO)
    b = _rank_ctx(packed, params, cube, 0, 2, 0, abi.HG_KERNEL_AUTO)  # wrong: also tiled as rank 0
    comm = abi.Comm.all([a, b])
    try:
        with pytest.raises(abi.HalogenError, match="tiled as 0/2, not 1/2"):
            comm.gather(0)
        with pytest.raises(abi.HalogenError, match="no gathered image"):
            comm.readback(64, 64)
        with pytest.raises(abi.HalogenError, match="root 5 out of range"):
            comm.gather(5)
    finally:
        comm.close()
        a.close()
        b.close()
