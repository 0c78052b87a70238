"""Multi-GPU gather behind the C-ABI (hg_comm_*) on one GPU.

Two (three) contexts on device 0 play ranks 0/1 (0/1/2) of an N-rank render: each renders its interleaved 8x8
tiles with the frame-parallel split forced on (several waves per tile, colours blended in frame order, the path that
showed the round-1 zero-block observation), hg_comm_init_all joins them (contexts sharing a device take the
in-process device-copy transport; RCCL refuses two ranks on one GPU), hg_comm_gather assembles the image on the
root's device.  The merged image must be bit-equal to a 1-rank render and every pixel written (alpha == 1).
A 1-rank communicator through hg_comm_init_rank exercises the RCCL transport's set-up, agreement and assembly on this
GPU; a 2-rank communicator whose peer never joins must fail within its deadline (SURVEY.md §5 failure detection)."""
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
        comm.synchronize()
        img = comm.readback(64, 64)
        assert_bitwise(img, ctx.readback(64, 64), "1-rank RCCL gather")
        # the agreement all-reduce sees a context not tiled for this communicator: a loud error, not a hang
        ctx.set_tiling(0, 2)
        with pytest.raises(abi.HalogenError, match="tiled as 0/2"):
            comm.gather(0)
        ctx.set_tiling(0, 1)
        ctx.render(frames, acc)
        comm.gather(0)
        assert_bitwise(comm.readback(64, 64), ctx.readback(64, 64), "1-rank RCCL gather after a refused one")
        comm.close()
    finally:
        ctx.close()


_DEAD_PEER = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from halogen import abi
ctx = abi.Context(0)
ctx.resize(64, 64)
ctx.set_tiling(0, 2)
t0 = time.time()
try:
    abi.Comm.rank(ctx, 2, abi.comm_unique_id(), 0)  # rank 1 never joins
    print("JOINED")
except abi.HalogenError as e:
    print("FAILED-LOUDLY %.1f %s" % (time.time() - t0, e), flush=True)
ctx.close()
import os
os._exit(0)  # the abandoned init's helper thread may still be blocked in RCCL: do not wait for it at exit
"""


@pytest.mark.gpu
def test_gpu_comm_dead_peer_fails_within_deadline(gpu, tmp_path):
    """A 2-rank communicator whose second rank never joins: hg_comm_init_rank (ncclCommInitRank on a helper thread,
    waited for with the deadline HALOGEN_COMM_TIMEOUT_MS) gives up at the deadline and returns HG_E_COMM with text,
    instead of blocking forever (RCCL's own non-blocking init was measured to block in the caller while a peer is
    missing).  Run in a child process so that a hang could not take the test session with it."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    pkg = str(Path(__file__).resolve().parents[1] / "halogen-pathtracer_amd")
    env = dict(os.environ, HALOGEN_COMM_TIMEOUT_MS="3000")
    r = subprocess.run([sys.executable, "-c", _DEAD_PEER, pkg], env=env, capture_output=True, text=True, timeout=100)
    out = r.stdout + r.stderr
    assert "FAILED-LOUDLY" in r.stdout, out[-2000:]
    secs = float(r.stdout.split("FAILED-LOUDLY")[1].split()[0])
    assert 2.5 <= secs < 60, out[-2000:]
    assert "did not all join within 3000 ms" in r.stdout, out[-2000:]


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


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["peer", "rccl"])
def test_gpu_comm_display_readback_pipelined(gpu, transport):
    """hg_comm_readback_begin / _end (the multi-GPU display path of the C# pass): the gathered image in every display
    format, one and two frames behind, equals the host packing of the blocking fp32 readback of the same gather."""
    packed, params, cube, _, acc = cases.setup("c1_64")
    W, H = int(params.screenParameters.x), int(params.screenParameters.y)
    n = 2 if transport == "peer" else 1
    ctxs = [_rank_ctx(packed, params, cube, r, n, 0, abi.HG_KERNEL_AUTO) for r in range(n)]
    comm = abi.Comm.all(ctxs) if transport == "peer" else abi.Comm.rank(ctxs[0], 1, abi.comm_unique_id(), 0)
    try:
        ctxs[0].set_option(abi.HG_OPT_READBACK_DEPTH, 3)
        for fmt in (abi.HG_DISPLAY_R11G11B10F, abi.HG_DISPLAY_RGBA16F, abi.HG_DISPLAY_RGBA32F):
            want, got = [], []
            pending = 0
            for _ in range(4):
                for c in ctxs:
                    c.render(1, acc)
                comm.gather(0)
                comm.readback_begin(fmt)
                pending += 1
                want.append(comm.readback(W, H))  # blocking fp32 readback of the same gather (waits for it)
                if pending == 3:
                    got.append(comm.readback_end(W, H))
                    pending -= 1
            while pending:
                got.append(comm.readback_end(W, H))
                pending -= 1
            with pytest.raises(abi.HalogenError, match="no readback outstanding"):
                comm.readback_end(W, H)
            for k, (g, w) in enumerate(zip(got, want)):
                h = abi.pack_display(w, fmt)
                gb = g.view(np.uint32) if g.dtype == np.float32 else g.view(np.uint16) if g.dtype == np.float16 else g
                hb = h.view(np.uint32) if h.dtype == np.float32 else h.view(np.uint16) if h.dtype == np.float16 else h
                assert int((gb != hb).sum()) == 0, f"format {fmt}, frame {k + 1}"
    finally:
        comm.close()
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_gpu_comm_gather_refuses_a_lost_frame(gpu):
    """A rank whose accumulation a lost render-server frame invalidated (HG_OPT_SERVER_GATE_US 0 on a 1080p C3 frame:
    its gate finds it unfinished) makes the gather fail with HG_E_FRAME_LOST (the peer transport checks every member;
    the RCCL one carries the flag in its agreement all-reduce); after a clear of that rank the gather works again and
    the image equals one context's."""
    from halogen import scenes
    from test_gpu_server import _sized
    cfg = scenes.CONFIGS["C3"]
    packed, params, cube = _sized("C3", cfg.width, cfg.height)
    W, H = cfg.width, cfg.height
    ctxs = []
    for r in range(2):
        ctx = abi.Context(0)
        ctx.set_option(abi.HG_OPT_SERVER, 2)
        ctx.set_option(abi.HG_OPT_COALESCE, 1)
        ctx.upload_scene(packed)
        if cube is not None:
            ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
        ctx.resize(W, H)
        ctx.set_tiling(r, 2)
        ctx.set_params(params)
        ctxs.append(ctx)
    comm = abi.Comm.all(ctxs)
    try:
        ctxs[0].render(1, True)
        ctxs[1].set_option(abi.HG_OPT_SERVER_GATE_US, 0)
        try:
            ctxs[1].render(1, True)
        except abi.HalogenError as e:
            assert e.rc == abi.HG_E_FRAME_LOST, e
        with pytest.raises(abi.HalogenError) as e:
            ctxs[1].synchronize()  # (the frame's gate has given up by the time the server is stopped)
        assert e.value.rc == abi.HG_E_FRAME_LOST
        with pytest.raises(abi.HalogenError) as e:
            comm.gather(0)
        assert e.value.rc == abi.HG_E_FRAME_LOST, e.value
        ctxs[1].set_option(abi.HG_OPT_SERVER_GATE_US, -1)
        ctxs[1].clear_accumulation()
        ctxs[1].set_params(params)
        ctxs[1].render(1, True)
        comm.gather(0)
        img = comm.readback(W, H)
        with abi.Context(0) as one:
            ref, _ = gpu_render(packed, params, 1, True, cube, ctx=one)
        assert_bitwise(img, ref, "gathered image after the lost rank's clear")
    finally:
        comm.close()
        for c in ctxs:
            c.close()
