#!/usr/bin/env python3
"""bench.py — the headline benchmark of BASELINE.json: Mpaths/s (+ Mrays/s) of the 1080p, 8-bounce,
871,200-triangle dragon Cornell box (config C3), on N GPUs of one node.

  python bench.py [--gpus N --steps K --warmup W] [--config C3]
  (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N; run without
  a launcher, `python bench.py --gpus N` starts that launcher itself as a child process, before anything touches a GPU,
  and relays rank 0's line and the exit status)

A STEP is one complete C3 image PER GPU: 64 progressive frames of 1 spp (the reference's unit of work is one
frame = one HalogenCompute dispatch + one accumulation blit, RP:324-347; C3 accumulates 64 of them) over the
whole 1920x1080 image, issued as one hg_render(64) call.  At N GPUs one step traces N*64 frames of the image,
its 8x8 tiles dealt round-robin to the N ranks, so per-GPU work is fixed ("scaling": "weak") and the
accumulated image is bit-identical to a 1-GPU render of N*64*K frames.  The timed region (barrier + device sync
on both sides, max over ranks) covers K steps and, for N > 1, the final RCCL gather of the tiles to rank 0.
Scene build/upload and BVH build are outside it (as in the reference meter, HalogenDebugUI.cs:37-56).

value = W*H*N*K / time (Mpaths/s); Mrays/s counts get_ray_intersection calls (device counters); primary_miss_frac
is the share of paths whose camera ray hits nothing (one-ray paths), and "framed" repeats C3 with the box opening
filling the frame (almost no such paths).
roofline: the trace kernel is bound by VALU issue and latency on a cache-resident scene, so "frac" is its VALU
issue rate (SQ_INSTS_VALU per launch from the committed rocprofv3 pass of this workload, over the launch duration
measured here with HIP events on the launch stream) against 1,024 SIMDs x 2.4 GHz / 2 cycles; the PMC-measured
DRAM-side bytes ("traffic") against 8 TB/s and SURVEY.md §8d's logical bytes (32 B per AABB test, 36 B per
triangle test, 64 B per mesh transform, 44 B per sphere test, 284 B per accepted hit, 48 B per pixel-frame)
are reported beside it.
cpu_baseline: the CPU oracle (oracle/hg_oracle.c, a scalar C restatement of the same kernel) on rank 0 at N=1,
on a stratified sample of row bands of the same workload, threads = min(16, CPUs in this process's affinity mask); the
line reports the affinity CPUs and the physical cores among them beside the thread count.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent


def gpus_requested(argv) -> int:
    """--gpus N (either form) of a command line, 1 when absent or malformed."""
    for i, a in enumerate(argv):
        try:
            if a == "--gpus" and i + 1 < len(argv):
                return int(argv[i + 1])
            if a.startswith("--gpus="):
                return int(a.split("=", 1)[1])
        except ValueError:
            return 1
    return 1


def self_launch_command(argv, n: int, port: int) -> list:
    """The launcher the driver would have used: one process per GPU (torch.distributed.run, rendezvous on 127.0.0.1),
    each running this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def self_launch(argv) -> int | None:
    """`bench.py --gpus N` (N > 1) started without a launcher (no WORLD_SIZE): start the N ranks as a child launcher and
    return its exit status (non-zero if any rank failed); rank 0 prints the one JSON line, on the inherited stdout.  Runs
    before halogen is imported, so this process never initialises a GPU (the children each open their own).  None: this
    process is a rank (or N = 1) and runs the bench itself."""
    if "WORLD_SIZE" in os.environ:
        return None
    n = gpus_requested(argv)
    if n <= 1:
        return None
    with socket.socket() as sk:  # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between the ranks' processes)
    return subprocess.run(self_launch_command(argv, n, port), env=env).returncode


if __name__ == "__main__":
    _rc = self_launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

sys.path.insert(0, str(ROOT / "halogen-pathtracer_amd"))

from halogen import abi  # noqa: E402
from halogen import render_pass as rp  # noqa: E402
from halogen import scenes  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 TB/s measured copy)
# VALU issue peak: 256 CUs x 4 SIMD-32 x 2.4 GHz, one wave64 VALU instruction per SIMD every 2 cycles
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles"), in G wave-instructions/s
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2
# Vector-memory data path (TD) floor: a wave-level load instruction holds a CU's texture-data unit for about 20 cycles
# whatever its width (tools/micro_td_width.hip, tools/sweeps/micro_td_r03.json: 16-B loads, 4 lines per wave, 20.07
# cycles, 30.6 G wave-loads/s on the GPU), so 256 CUs x 2.4 GHz / 20 cycles = 30.72 G wave-level VMEM instructions/s.
# The traversal is bound by this unit (TD busy ~0.96), DESIGN.md sections 4.5, 10.
VMEM_FLOOR_CYCLES = 20.0
VMEM_PEAK_GINST = 256 * 2.4 / VMEM_FLOOR_CYCLES
KERNEL_SYMBOL = {abi.HG_KERNEL_MEGA_STREAM: "hg_trace_stream_kernel", abi.HG_KERNEL_MEGA_REGEN: "hg_trace_regen_kernel",
                 abi.HG_KERNEL_MEGA: "hg_trace_kernel"}
METRIC = "Mpaths/s (+ Mrays/s) at 1080p, 8-bounce dragon Cornell box, 1/2/4/8 GPU"


def algorithmic_bytes(c: dict) -> float:
    return (32.0 * c["aabb_tests"] + 36.0 * c["tri_tests"] + 64.0 * c["mesh_visits"] + 44.0 * c["sphere_tests"]
            + 284.0 * c["hits"] + 48.0 * c["paths"])


def framed_measurement(ctx, packed, s, W, H, frames_per_step: int, steps: int) -> dict:
    """C3F beside the headline: the same scene, settings and image size with the camera moved in until the box
    opening fills the frame (scenes.CORNELL_FRAMED_CAMERA_POS), so nearly every path enters the box.  Warm-up launch,
    `steps` timed steps (device sync on both sides), then one counting replay step for the path statistics."""
    cfg = scenes.CONFIGS["C3F"].resized(W, H)
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), False)
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    ctx.clear_accumulation()
    ctx.set_params(params)
    for _ in range(2):  # warm-up, one launch per trace stream: each records this view's tile costs for its cost order
        ctx.render(frames_per_step, True)
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.synchronize()
    ctx.reset_counters()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.render(frames_per_step, True)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    timing = ctx.counters()  # trace-kernel launch durations (HIP events on the trace streams)
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.reset_counters()
    ctx.set_option(abi.HG_OPT_COUNTERS, 1)
    ctx.render(frames_per_step, True)
    c = ctx.counters()
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    paths = W * H * frames_per_step * steps
    kernel_symbol = KERNEL_SYMBOL.get(int(c["last_kernel"]), "?")
    mean_launch_s, span_s = launch_seconds(timing)
    # its own roofline, from the committed C3F PMC pass (profiles/pmc_traffic_C3F.json)
    roofline = roofline_of(committed_counters("C3F", W, H, frames_per_step, kernel_symbol), mean_launch_s,
                           algorithmic_bytes(c), kernel_symbol, dt / steps, span_s)
    return {"workload": cfg.name, "value": paths / dt / 1e6, "unit": "Mpaths/s", "steps": steps,
            "ms_per_step": dt * 1e3 / steps, "mrays_per_s": c["rays"] / c["paths"] * paths / dt / 1e6,
            "primary_miss_frac": c["primary_misses"] / c["paths"], "rays_per_path": c["rays"] / c["paths"],
            "tri_tests_per_path": c["tri_tests"] / c["paths"], "camera_position": list(scenes.CORNELL_FRAMED_CAMERA_POS),
            "roofline": roofline}


def fast_bvh_measurement(ctx, cfg, packed, cube, params, W, H, frames_per_step: int, steps: int, ref_img,
                         headline: float) -> dict:
    """The same workload on an SAH hierarchy (hg_build_blas_sah) instead of the reference
    builder's: NOT the contract line (the drop-in keeps BVHGenerator's tree), a second number beside it.  The kernel
    traverses any hierarchy the reference's way (tests/test_gpu_fast_bvh.py: bit-exact against the oracle on the same
    tree), so the images differ only where two triangles tie within rounding; the leg reports how many pixels of the
    timed region's final image differ from the headline's.  Same loop as the headline: warm-up, `steps` x
    hg_render(frames_per_step) from a cleared accumulator, then a counting replay step."""
    from halogen import scene as scene_mod

    prev = scene_mod.set_blas_builder("sah")
    try:
        t = time.perf_counter()
        sah = cfg.build_scene().pack()
        build_s = time.perf_counter() - t
    finally:
        scene_mod.set_blas_builder(prev)
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    ctx.upload_scene(sah)
    ctx.set_params(params)
    for _ in range(3):
        ctx.render(frames_per_step, True)
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.synchronize()
    ctx.reset_counters()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.render(frames_per_step, True)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    timing = ctx.counters()  # trace-kernel launch durations (HIP events on the trace streams)
    img = ctx.readback(W, H)
    differ = (img.view(np.uint32) != ref_img.view(np.uint32)).any(-1)
    d = np.abs(img.astype(np.float64) - ref_img.astype(np.float64))
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.reset_counters()
    ctx.set_option(abi.HG_OPT_COUNTERS, 1)
    ctx.render(frames_per_step, True)
    c = ctx.counters()
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    ctx.upload_scene(packed)  # the reference tree again for the legs after this one
    value = W * H * frames_per_step * steps / dt / 1e6
    kernel_symbol = KERNEL_SYMBOL.get(int(c["last_kernel"]), "?")
    mean_launch_s, span_s = launch_seconds(timing)
    # its own roofline, from the committed PMC pass of this workload (profiles/pmc_traffic_C3SAH.json)
    roofline = roofline_of(committed_counters("C3SAH", W, H, frames_per_step, kernel_symbol), mean_launch_s,
                           algorithmic_bytes(c), kernel_symbol, dt / steps, span_s)
    return {"workload": "C3 on an SAH BLAS (hg_build_blas_sah, max leaf 2): not the reference's hierarchy",
            "roofline": roofline,
            "value": value, "unit": "Mpaths/s", "steps": steps, "ms_per_step": dt * 1e3 / steps,
            "frac_of_headline": value / headline, "build_s": build_s, "blas_nodes": len(sah.blas),
            "pixels_differing_from_headline_image": float(differ.mean()),
            "max_abs_diff": float(d.max()), "mean_abs_diff": float(d.mean()),
            "counters_per_path": {k: c[k] / c["paths"] for k in ("rays", "tri_tests", "aabb_tests", "hits")}}


def per_frame_measurement(ctx, params, W, H, frames: int, reps: int, batched_value: float) -> dict:
    """The drop-in's operating point: the reference dispatches HalogenCompute once per frame (RP:327, RP:406) and the
    C# shim calls hg_render(ctx, 1, 1) per Execute.  The same C3 step (`frames` progressive frames from a cleared
    accumulator) is rendered as `frames` x hg_render(1) and compared bit for bit with one hg_render(frames), then timed
    (`reps` steps, the headline's K: as many frames from one clear as its timed region; device sync on both sides):
      value       the library's default: consecutive calls are held and launched HG_OPT_COALESCE (32) frames at a time;
      strict      HG_OPT_COALESCE 1: every call its own; the render server serves them once the host runs ahead
                  (HG_OPT_SERVER 1), and `strict.per_launch` times the same calls with a launch each (HG_OPT_SERVER 0);
      with_readback  hg_readback of the 33 MB image into a caller buffer after every call (which launches the held
                  frame, so this is one launch per frame too);
      with_display_readback  the C# pass's per-frame display path, hg_readback_begin/_end into the context's pinned
                  images: "sync" shows frame k before tracing k+1, "pipelined" one frame behind."""
    def fresh():
        ctx.clear_accumulation()
        ctx.set_params(params)

    ctx.set_option(abi.HG_OPT_COUNTERS, 0)  # the timed kernels (the counting replay before this leg turns them on)

    def timed(coalesce: int):
        ctx.set_option(abi.HG_OPT_COALESCE, coalesce)
        ctx.reset_counters()
        before = ctx.counters()  # (the server's counts run since hg_create: their difference is this run's)
        fresh()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for _ in range(frames):
                ctx.render(1, True)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        c = ctx.counters()
        for k in ("server_launches", "server_frames"):
            c[k] = c.get(k, 0) - before.get(k, 0)
        return dt, c

    fresh()
    ctx.render(frames, True)
    batched = ctx.readback(W, H)
    identical = {}
    for coalesce, server in ((1, 1), (32, 1), (1, 2), (1, 0)):
        ctx.set_option(abi.HG_OPT_COALESCE, coalesce)
        ctx.set_option(abi.HG_OPT_SERVER, server)
        fresh()
        for _ in range(frames):
            ctx.render(1, True)
        key = f"coalesce_{coalesce}" + {1: "", 2: "_server", 0: "_no_server"}[server]
        identical[key] = bool(np.array_equal(batched.view(np.uint32), ctx.readback(W, H).view(np.uint32)))
    ctx.set_option(abi.HG_OPT_SERVER, 1)
    paths = W * H * frames
    dt, c = timed(32)
    dt_s, c_s = timed(1)  # (the render server engages once the host runs ahead: HG_OPT_SERVER 1, the default)
    ctx.set_option(abi.HG_OPT_SERVER, 0)  # the same calls, a launch per call (round 4's pipeline), for comparison
    dt_s0, c_s0 = timed(1)
    ctx.set_option(abi.HG_OPT_SERVER, 1)
    img = np.empty((H, W, 4), np.float32)
    fresh()
    ctx.synchronize()
    t1 = time.perf_counter()
    for _ in range(frames):
        ctx.render(1, True)
        ctx.readback(W, H, img)
    dt_rb = time.perf_counter() - t1
    # display readback through the context's pinned images (hg_readback_begin_format / hg_readback_end_data), in each
    # display format: the image of this frame before the next is traced (sync), one frame behind so that frame k's copy
    # overlaps frame k+1's trace (pipelined: the C# / C++ passes' pattern), or three frames behind (depth 4)
    display = {}
    for fmt_name, fmt in abi.DISPLAY_FORMATS.items():
        res = {"bytes_per_frame": W * H * abi.DISPLAY_BPP[fmt]}
        for mode, depth, side in (("sync", 1, 0), ("pipelined", 2, 0), ("pipelined_depth4", 4, 0),
                                  ("pipelined_side", 2, 1), ("pipelined_depth4_side", 4, 1),
                                  ("pipelined_depth8_side", 8, 1), ("pipelined_depth16", 16, 0),
                                  ("sync_zero_copy", 1, 2), ("pipelined_zero_copy", 2, 2),
                                  ("pipelined_depth4_zero_copy", 4, 2)):
            fresh()
            ctx.set_option(abi.HG_OPT_READBACK_DEPTH, depth)
            ctx.set_option(abi.HG_OPT_READBACK_STREAM, side)
            ctx.synchronize()
            t1 = time.perf_counter()
            pending = 0
            for _ in range(frames):
                ctx.render(1, True)
                ctx.readback_begin(fmt)
                pending += 1
                if pending == depth:
                    ctx.readback_end(W, H, copy=False)
                    pending -= 1
            while pending:
                ctx.readback_end(W, H, copy=False)
                pending -= 1
            dt_d = time.perf_counter() - t1
            v = paths / dt_d / 1e6
            res[mode] = {"value": v, "unit": "Mpaths/s", "ms_per_frame": dt_d * 1e3 / frames,
                         "frac_of_batched": v / batched_value, "frames_behind": depth - 1,
                         "copy_stream": {0: "context", 1: "side", 2: "none (zero copy)"}[side]}
        display[fmt_name] = res
    ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 2)
    ctx.set_option(abi.HG_OPT_READBACK_STREAM, 0)
    last = ctx.readback(W, H)
    display["last_image_identical"] = bool(np.array_equal(batched.view(np.uint32), last.view(np.uint32)))
    # the images of the last run (r11g11b10f, three frames behind) equal the host packing of the fp32 image
    fresh()
    for _ in range(frames):
        ctx.render(1, True)
    ctx.readback_begin(abi.HG_DISPLAY_R11G11B10F)
    packed_img = ctx.readback_end(W, H)
    display["r11g11b10f_equals_host_packing"] = bool(np.array_equal(
        packed_img, abi.pack_display(ctx.readback(W, H), abi.HG_DISPLAY_R11G11B10F)))
    ctx.set_option(abi.HG_OPT_COALESCE, 32)
    value = paths * reps / dt / 1e6
    strict = paths * reps / dt_s / 1e6
    return {"workload": f"{frames} x hg_render(1) per step (RP:327 one call per frame)", "value": value,
            "unit": "Mpaths/s", "steps": reps, "ms_per_frame": dt * 1e3 / (reps * frames),
            "launches_per_step": c["launches"] / reps, "frac_of_batched": value / batched_value,
            "strict": {"value": strict, "ms_per_frame": dt_s * 1e3 / (reps * frames),
                       "launches_per_step": c_s["launches"] / reps, "frac_of_batched": strict / batched_value,
                       "server_launches": c_s.get("server_launches", 0), "server_frames": c_s.get("server_frames", 0),
                       "per_launch": {"value": paths * reps / dt_s0 / 1e6, "ms_per_frame": dt_s0 * 1e3 / (reps * frames),
                                      "frac_of_batched": paths * reps / dt_s0 / 1e6 / batched_value,
                                      "note": "HG_OPT_SERVER 0: every call its own launch"}},
            "with_readback": {"value": paths / dt_rb / 1e6, "unit": "Mpaths/s", "ms_per_frame": dt_rb * 1e3 / frames,
                              "readback_bytes_per_frame": W * H * 16},
            "with_display_readback": display,
            "bit_identical_to_batched": identical}


def camera_move_measurement(ctx, packed, s, cfg, W, H, frames: int, cube) -> dict:
    """The reference's moving-camera frame (VERDICT r03 missing #3).  A camera move makes Execute call
    ClearAccumulation, which sets ObjectBuffersDirty, so UpdateObjectBuffers gathers every scene array again and
    SetBufferData re-uploads it before the dispatch (RP:262-268, 279-299, 448-509); the C# drop-in keeps that call
    pattern (bindings/csharp/HalogenRenderPass.cs).  Per frame, as the drop-in issues it: hg_upload_scene (the same
    arrays), hg_set_params with the moved camera (FrameCount 1), hg_clear_accumulation, hg_render(1) and the display
    readback (R11G11B10F, one frame behind).  Reports ms per frame and the share spent inside hg_upload_scene (an
    identical upload is detected and skipped by the library), and the cost of an upload whose arrays did change (a real
    rebuild: validation, repack, copies), timed separately."""
    import ctypes as C

    from halogen.scene import PackedScene
    from halogen.unity import Transform

    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    ctx.set_option(abi.HG_OPT_READBACK_DEPTH, 2)
    base = cfg.camera()
    pos0 = tuple(base.transform.position)

    def camera_at(k: int):
        t = Transform((pos0[0] + 0.002 * k, pos0[1], pos0[2] - 0.001 * k), tuple(base.transform.rotation))
        return rp.Camera(t, base.fieldOfView, W, H)

    def frame_loop(n: int, generation: int):
        before = ctx.counters()
        up = 0.0
        pending = 0
        ctx.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            tu = time.perf_counter()
            ctx.upload_scene(packed, generation)
            up += time.perf_counter() - tu
            ctx.set_params(rp.make_params(s, camera_at(k + 1), 1, len(packed.spheres), len(packed.meshes),
                                          cube is not None))
            ctx.clear_accumulation()
            ctx.render(1, True)
            ctx.readback_begin(abi.HG_DISPLAY_R11G11B10F)
            pending += 1
            if pending == 2:
                ctx.readback_end(W, H, copy=False)
                pending -= 1
        while pending:
            ctx.readback_end(W, H, copy=False)
            pending -= 1
        dt = time.perf_counter() - t0
        after = ctx.counters()
        return dt, up, after["scene_uploads_skipped"] - before["scene_uploads_skipped"], \
            after["scene_uploads"] - before["scene_uploads"]

    # the drop-in passes' call: the geometry generation unchanged (their mesh registry did not change), so only the small
    # arrays are compared (hg_upload_scene_gen); untagged, the 78 MB of triangles and BVH entries are compared as well
    ctx.upload_scene(packed, 1)
    frame_loop(4, 1)  # warm-up
    dt, up, skipped, rebuilt = frame_loop(frames, 1)
    dt0, up0, _, _ = frame_loop(frames, 0)

    def copy(p):
        arrays = {}
        for k in ("spheres", "meshes", "materials", "triangles", "blas"):
            a = getattr(p, k)
            b = (type(a)._type_ * len(a))()
            C.memmove(b, a, C.sizeof(a))
            arrays[k] = b
        return PackedScene(**arrays)

    # a changed upload (one float of the last triangle moved, then moved back): every call rebuilds the device scene
    alt = copy(packed)
    alt.triangles[len(alt.triangles) - 1].pointA.x += 1e-3
    rebuild = []
    for k in range(4):
        t0 = time.perf_counter()
        ctx.upload_scene(alt if k % 2 == 0 else packed)  # (a new geometry: untagged)
        rebuild.append(time.perf_counter() - t0)
    # an object moved (the last mesh translated, then back): triangles and BVH as before, a partial re-upload
    moved = copy(packed)
    moved.meshes[len(moved.meshes) - 1].worldToLocal.m[12] += 0.05
    partial = []
    ctx.upload_scene(packed, 2)
    for k in range(4):
        t0 = time.perf_counter()
        ctx.upload_scene(moved if k % 2 == 0 else packed, 2)  # (triangles and BVH vouched for: generation unchanged)
        partial.append(time.perf_counter() - t0)
    ctx.upload_scene(packed)
    c = ctx.counters()
    scene_bytes = sum(C.sizeof(getattr(packed, k)) for k in ("spheres", "meshes", "materials", "triangles", "blas"))
    return {"workload": f"{frames} frames, camera moved before each: hg_upload_scene_gen (same arrays, same geometry "
                        f"generation) + hg_set_params + "
                        f"hg_clear_accumulation + hg_render(1) + R11G11B10F display one frame behind (RP:262-299)",
            "value": W * H * frames / dt / 1e6, "unit": "Mpaths/s", "ms_per_frame": dt * 1e3 / frames,
            "upload_ms_per_frame": up * 1e3 / frames, "upload_share": up / dt,
            "untagged": {"value": W * H * frames / dt0 / 1e6, "ms_per_frame": dt0 * 1e3 / frames,
                         "upload_ms_per_frame": up0 * 1e3 / frames, "upload_share": up0 / dt0,
                         "note": "hg_upload_scene without a geometry generation: every array compared byte for byte"},
            "uploads_skipped": skipped, "uploads_rebuilt": rebuilt, "scene_bytes": scene_bytes,
            "changed_upload_ms": [x * 1e3 for x in rebuild],
            "changed_upload_ms_mean": sum(rebuild) * 1e3 / len(rebuild),
            "object_moved_upload_ms": [x * 1e3 for x in partial],
            "object_moved_upload_ms_mean": sum(partial) * 1e3 / len(partial),
            "scene_uploads_partial": c["scene_uploads_partial"], "scene_uploads_vouched": c["scene_uploads_vouched"],
            "scene_uploads_total": c["scene_uploads"], "host_threads_upload": 16}


def strong_scaling_measurement(ctx, params, W, H, fps: int, steps: int, world: int, rank: int, emu: int, barrier,
                               gather_fn, coll_dev, dist, ref_img=None, coalesce: int = -1) -> dict:
    """The strong-scaling leg, beside the weak line: the FIXED image of `fps` frames per step (C3: 64),
    its 8x8 tiles dealt round-robin to the N ranks (HC:1033: pixels are independent), so the ranks share one image's work
    instead of each doing one image's worth.  Same clock as the headline (barrier + device sync on both sides, max over
    ranks) around `steps` x hg_render(fps) and the gather of the tiles to rank 0.  Reports the value, the ms per step, and
    each rank's tile count and trace time (its renders' completion on its own clock, before the gather), so load balance
    shows.  N > 1: rank 0 compares the gathered image with `ref_img` (the same frames on one context, all tiles) bit for
    bit.  --emulate-ranks N (one GPU): rank 0's share alone, and the rate N such shares would reach if equally fast."""
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)
    if coalesce >= 1:
        ctx.set_option(abi.HG_OPT_COALESCE, coalesce)
    ctx.clear_accumulation()
    ctx.set_params(params)
    for _ in range(steps):  # warm-up: the same calls (this share's launches, their buffers and cost order)
        ctx.render(fps, True)
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.reset_counters()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.render(fps, True)
    ctx.synchronize()
    t_trace = time.perf_counter() - t0
    gathered = gather_fn() if world > 1 else None
    barrier()
    dt = time.perf_counter() - t0
    c = ctx.counters()
    mine = [dt, t_trace, float(ctx.local_tile_count()), c.get("trace_busy_ms", 0.0)]
    per_rank = [mine]
    if dist is not None:
        import torch

        t = torch.tensor(mine, dtype=torch.float64, device=coll_dev)
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        per_rank = [x.tolist() for x in out]
    dt_max = max(r[0] for r in per_rank)
    n = emu or world
    paths = W * H * fps * steps if not emu else ctx.local_tile_count() * 64 * fps * steps
    res = {"scaling": "strong", "workload": f"one {W}x{H} image of {fps} frames per step, its tiles over {n} ranks",
           "n_ranks": n, "steps": steps, "value": paths / dt_max / 1e6, "unit": "Mpaths/s",
           "ms_per_step": dt_max * 1e3 / steps,
           "per_rank": [{"rank": r, "tiles": int(v[2]), "trace_ms_per_step": v[1] * 1e3 / steps,
                         "total_ms_per_step": v[0] * 1e3 / steps, "trace_busy_ms": v[3]} for r, v in enumerate(per_rank)],
           "trace_balance": min(v[1] for v in per_rank) / max(v[1] for v in per_rank),
           # a share holds consecutive calls until its launch fills the GPU (HG_OPT_COALESCE's share window)
           "launches": int(c.get("launches", 0))}
    if emu:
        res["emulated"] = f"rank 0's share of {n} on one GPU: value is that share's rate; x{n} if every share ran alike"
        res["value_if_balanced"] = res["value"] * n
    if rank == 0 and world > 1 and gathered is not None and ref_img is not None:
        g = gathered if isinstance(gathered, np.ndarray) else gathered.cpu().numpy()
        res["gathered_bit_identical_to_one_context"] = bool(np.array_equal(g.view(np.uint32), ref_img.view(np.uint32)))
    return res


def compact_summary(result: dict) -> dict:
    """The operating points in a few hundred bytes, the last key of the line (the driver keeps the line's last 8 KB):
    the headline, the per-frame points as fractions of it, the camera-move frame, the framed and SAH views, the strong
    leg and the roofline fraction."""
    def r(x, nd=3):
        return None if x is None else round(float(x), nd)

    pf = result.get("per_frame") or {}
    strict = pf.get("strict") or {}
    disp = (pf.get("with_display_readback") or {}).get("r11g11b10f") or {}
    cam = result.get("camera_move") or {}
    strong = result.get("strong_scaling") or {}
    roof = result.get("roofline") or {}
    behind = {"at_once": "sync", "one_behind": "pipelined", "three_behind": "pipelined_depth4",
              "seven_behind": "pipelined_depth8_side", "fifteen_behind": "pipelined_depth16"}
    return {
        "value": r(result.get("value"), 1),
        "primary_miss_frac": r(result.get("primary_miss_frac")),
        "roofline_frac": r(roof.get("frac")),
        "per_frame": {
            "coalesced": {"frac_of_batched": r(pf.get("frac_of_batched"))},
            "strict": {"value": r(strict.get("value"), 1), "frac_of_batched": r(strict.get("frac_of_batched")),
                       "server_launches": strict.get("server_launches")},
            "per_launch": {"frac_of_batched": r((strict.get("per_launch") or {}).get("frac_of_batched"))},
            "display_r11g11b10f": {k: r((disp.get(m) or {}).get("frac_of_batched")) for k, m in behind.items()},
        } if pf else None,
        "camera_move": {"value": r(cam.get("value"), 1), "frac_of_batched": r(cam.get("value") / result["value"])
                        if cam.get("value") else None, "upload_share": r(cam.get("upload_share"), 4)} if cam else None,
        "framed": r((result.get("framed") or {}).get("value"), 1),
        "fast_bvh": r((result.get("fast_bvh") or {}).get("value"), 1),
        "strong": {"n_ranks": strong.get("n_ranks"), "value": r(strong.get("value"), 1),
                   "per_gpu_frac_of_weak": r(strong.get("per_gpu_frac_of_weak"))} if strong else None,
    }


def split_detail(result: dict, path: str) -> None:
    """The per-format display tables go to `path` (JSON), the line keeps the reference's display format
    (R11G11B10F) and the bit-identity checks."""
    pf = result.get("per_frame")
    if not pf or not pf.get("with_display_readback"):
        return
    full = pf["with_display_readback"]
    pf["with_display_readback"] = {k: v for k, v in full.items() if k not in ("rgba32f", "rgba16f")}
    pf["with_display_readback"]["other_formats"] = path
    try:
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        Path(path).write_text(json.dumps({"with_display_readback": full, "config": result.get("config")}, indent=1))
    except OSError as e:
        pf["with_display_readback"]["other_formats"] = f"not written: {e}"


def committed_counters(config: str, W: int, H: int, frames_per_launch: int, kernel_symbol: str) -> dict:
    """The committed PMC figures of this workload's production kernel (tools/summarize_profile.py):
    profiles/pmc_traffic_<config>.json, or profiles/pmc_traffic.json (the headline config's), when they match the
    config, image size, frames per launch and the counter-free instantiation of the kernel that ran."""
    for name in (f"pmc_traffic_{config}.json", "pmc_traffic.json"):
        f = ROOT / "profiles" / name
        if not f.exists():
            continue
        try:
            t = json.loads(f.read_text())
        except Exception:
            continue
        if (t.get("config") == config and t.get("width") == W and t.get("height") == H
                and t.get("frames_per_launch") == frames_per_launch
                and str(t.get("kernel", "")).startswith(kernel_symbol + "<false")):  # counter-free build
            return t
    return {}


def library_sha256() -> str:
    import hashlib

    return hashlib.sha256(abi.LIB_PATH.read_bytes()).hexdigest()


def launch_seconds(timing: dict) -> tuple:
    """(device time per trace launch, mean of the launches' own event spans).  Consecutive launches run on two trace
    streams and overlap, so each launch's span also counts the time it shared the GPU with its neighbour; the union of
    the spans (hg_counters.trace_busy_ms) per launch is the kernel's device time per launch, the roofline's divisor.
    rocprofv3's kernel trace gives both (tools/summarize_profile.py: avg_ms_timed_union, avg_ms_timed)."""
    n = max(timing.get("trace_launches", 0), 1)
    busy = timing.get("trace_busy_ms", 0.0) or timing.get("trace_ms", 0.0)
    return busy / n / 1e3, timing.get("trace_ms", 0.0) / n / 1e3


def roofline_of(pmc: dict, mean_launch_s: float, logical_per_launch, kernel_symbol: str, step_s: float = 0.0,
                events_launch_s: float = 0.0) -> dict:
    """The dominant kernel against the unit that binds it.  The trace kernel works on a cache-resident scene (C3: 90 MB,
    inside the 256 MiB Infinity Cache) and is bound by the vector-memory data path (the texture-data unit busy ~96 % of
    the launch): `achieved` is its wave-level vector-memory instruction rate ((SQ_INSTS_VMEM_RD + SQ_INSTS_VMEM_WR) per
    launch from the committed rocprofv3 pass of this workload and build, over the launch time measured live with HIP
    events) against the per-CU instruction floor of that unit (VMEM_PEAK_GINST); td_busy / td_stalled_on_l1 sit beside
    it.  The VALU issue rate is the secondary figure (`valu`: SQ_INSTS_VALU against 1,024 SIMDs x 2.4 GHz / 2 cycles).
    HBM stays beside both: the PMC-measured DRAM-side bytes (traffic) against 8 TB/s, and the section 8(d) logical bytes."""
    ok = mean_launch_s > 0
    valu = pmc.get("valu_insts_per_launch")
    valu_achieved = valu / mean_launch_s / 1e9 if valu and ok else None
    valu_frac = valu_achieved / VALU_PEAK_GINST if valu_achieved else None
    lane = pmc.get("valu_lane_util")
    vmem = pmc.get("vmem_insts_per_launch")
    vmem_achieved = vmem / mean_launch_s / 1e9 if vmem and ok else None
    vmem_frac = vmem_achieved / VMEM_PEAK_GINST if vmem_achieved else None
    busy = pmc.get("vmem_unit_busy") or {}
    traffic = pmc.get("hbm_bytes_per_launch")
    lib_sha = library_sha256()
    valu_obj = {"achieved": valu_achieved, "peak": VALU_PEAK_GINST, "unit": "Ginst/s", "frac": valu_frac,
                "insts_per_launch": valu,
                "unit_note": "wave64 VALU instructions issued per second (peak = 1024 SIMDs x 2.4 GHz / 2 cycles)",
                "lane_util": lane, "useful_lane_frac": valu_frac * lane if valu_frac and lane else None,
                "frac_per_launch_span": valu / events_launch_s / 1e9 / VALU_PEAK_GINST if valu and events_launch_s
                else None,
                "frac_per_step_period": valu / step_s / 1e9 / VALU_PEAK_GINST if valu and step_s else None}
    vmem_obj = {"achieved": vmem_achieved, "peak": VMEM_PEAK_GINST, "unit": "Ginst/s", "frac": vmem_frac,
                "insts_per_launch": vmem, "rd_per_launch": pmc.get("vmem_rd_insts_per_launch"),
                "wr_per_launch": pmc.get("vmem_wr_insts_per_launch"),
                "floor_cycles_per_inst": VMEM_FLOOR_CYCLES,
                "unit_note": "wave-level vector-memory instructions per second against the texture-data unit's "
                             "per-instruction floor (256 CUs x 2.4 GHz / 20 cycles, tools/micro_td_width.hip)",
                "td_busy": busy.get("td_busy"), "td_stalled_on_l1": busy.get("td_stalled_on_l1"),
                "ta_busy": busy.get("ta_busy"),
                "frac_per_step_period": vmem / step_s / 1e9 / VMEM_PEAK_GINST if vmem and step_s else None}
    bound_vmem = vmem_achieved is not None
    top = vmem_obj if bound_vmem else valu_obj
    return {"bound": "vmem" if bound_vmem else "valu", "achieved": top["achieved"], "peak": top["peak"],
            "unit": top["unit"], "unit_note": top["unit_note"], "frac": top["frac"],
            "vmem": vmem_obj, "valu": valu_obj,
            "lane_util": lane, "wait_any_frac": pmc.get("wait_any_frac"), "l2_hit_rate": pmc.get("l2_hit_rate"),
            "vmem_unit_busy": pmc.get("vmem_unit_busy"),
            "traffic": traffic,
            "traffic_gbs": traffic / mean_launch_s / 1e9 if traffic and ok else None,
            "traffic_frac": traffic / mean_launch_s / 1e9 / HBM_PEAK_GBS if traffic and ok else None,
            "hbm_peak_gbs": HBM_PEAK_GBS,
            "hbm_target_note": "north_star's >= 50 % of the HBM roofline during traversal does not apply: the scene "
                               "is cache-resident (L1/L2/Infinity Cache serve the BVH), so traffic_frac is the DRAM-side "
                               "share, not a bound; the traversal is bound by the vector-memory data path, whose "
                               "instruction rate `frac` prices (DRAM-side traffic and VALU issue beside it; DESIGN.md "
                               "sections 4.5, 10)",
            "write_bytes_per_launch": pmc.get("write_bytes_per_launch"),
            "logical_bytes_per_launch": logical_per_launch,
            "logical_gbs": logical_per_launch / mean_launch_s / 1e9 if logical_per_launch and ok else None,
            "mean_launch_ms": mean_launch_s * 1e3, "kernel": kernel_symbol,
            "launch_ms_basis": "union of the timed launches' HIP-event spans on both trace streams / launches",
            "mean_launch_span_ms": events_launch_s * 1e3 if events_launch_s else None,
            # launches of consecutive steps overlap (two trace streams): the step period is the throughput's clock
            "step_period_ms": step_s * 1e3 if step_s else None,
            "counters_from": pmc.get("summary"),
            "counters_library_matches": (pmc.get("library_sha256") == lib_sha) if pmc.get("library_sha256") else None}


def host_cpus() -> dict:
    """The CPUs this process may run on (sched_getaffinity), the physical cores among them (distinct (package, core)
    pairs from sysfs topology), and the machine's logical CPU count (os.cpu_count: on the GPU box the whole machine,
    many times this process's share)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores = set()
    for cpu in aff:
        t = Path(f"/sys/devices/system/cpu/cpu{cpu}/topology")
        try:
            cores.add((t.joinpath("physical_package_id").read_text().strip(), t.joinpath("core_id").read_text().strip()))
        except OSError:
            cores.add(("?", str(cpu)))
    return {"affinity_cpus": len(aff), "physical_cores_in_affinity": len(cores), "machine_logical_cpus": os.cpu_count()}


def cpu_baseline(packed, params, cube, width, height, seconds, threads):
    """Oracle on stratified 2-row bands of frame 1 until `seconds` of wall time are used.  The plain oracle build: its
    traversal holds no diagnostics (those live in the stats build, oracle/Makefile)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import hg_oracle  # test-infra import, cpu_baseline leg only

    hg_oracle.lib()
    assert hg_oracle.lib().hgo_stats_build() == 0
    n_bands = 27
    order = [int(b) for b in np.linspace(0, height - 2, n_bands).astype(int)]
    paths = 0
    frames = 0
    t0 = time.perf_counter()
    acc = np.zeros((height, width, 4), np.float32)
    while True:  # whole passes over the 27 bands, frame 1, 2, ... until the time budget is used
        frames += 1
        params.frameCount = frames
        for y in order:
            hg_oracle.render(packed, params, 1, True, acc=acc, cubemap=cube,
                             pix_range=(y * width, (y + 2) * width), threads=threads)
            paths += 2 * width
        if time.perf_counter() - t0 > seconds:
            break
    params.frameCount = 1
    dt = time.perf_counter() - t0
    host = host_cpus()
    return {"value": paths / dt / 1e6, "unit": "Mpaths/s", "cores": threads, "threads": threads, **host,
            "kind": "port",
            "sample": f"{n_bands} stratified 2-row bands x {width} px (every ~{height // n_bands} rows) x {frames} "
                      f"frames = {paths} paths in {dt:.1f} s; scalar C oracle (oracle/hg_oracle.c, plain build), "
                      f"{threads} threads on {host['affinity_cpus']} allowed CPUs "
                      f"({host['physical_cores_in_affinity']} physical cores)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)  # both trace streams sort a cost order before the timed launches
    ap.add_argument("--config", default="C3", choices=sorted(scenes.CONFIGS))
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-framed", action="store_true", help="skip the C3F (box opening fills the frame) measurement")
    ap.add_argument("--no-per-frame", action="store_true", help="skip the one-dispatch-per-frame leg")
    ap.add_argument("--per-frame-only", action="store_true",
                    help="profiling aid: only the per-frame leg's timed part (no headline line)")
    ap.add_argument("--launch-frames", type=int, default=1, help="--per-frame-only: frames per hg_render call")
    ap.add_argument("--coalesce", type=int, default=1, help="--per-frame-only: HG_OPT_COALESCE (1: every call launches)")
    ap.add_argument("--display", choices=["none", "sync", "pipelined"], default="none",
                    help="--per-frame-only: the display readback (hg_readback_begin/_end) after every call, as the "
                         "per_frame leg's with_display_readback")
    ap.add_argument("--display-format", default="rgba32f", choices=sorted(abi.DISPLAY_FORMATS),
                    help="--per-frame-only with --display: the display format")
    ap.add_argument("--readback-depth", type=int, default=2, help="--per-frame-only, --display pipelined: readbacks "
                    "in flight (HG_OPT_READBACK_DEPTH)")
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--kernel", default="auto", choices=["auto", "mega", "regen", "stream"])
    ap.add_argument("--frames-per-step", type=int, default=64,
                    help="progressive 1-spp frames per step per GPU-equivalent (64 = one C3 image)")
    ap.add_argument("--no-counters", action="store_true")
    ap.add_argument("--save-image", default="")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + HALOGEN_BENCH_DEVICE=0: rehearse the N-rank path on one GPU (CPU collectives)")
    ap.add_argument("--gather", default="abi", choices=["abi", "torch"],
                    help="N > 1: the timed tile gather through the C-ABI (default: hg_comm, RCCL send/recv on the "
                         "contexts' streams + device assembly, the drop-in's own path) or through torch.distributed "
                         "(all_gather_into_tensor, assembled on rank 0's device through hg_comm_assemble_host's index)")
    ap.add_argument("--no-abi-check", action="store_true",
                    help="N > 1: skip the untimed cross-check gather (the other transport of --gather), compared bit for "
                         "bit with the timed gather and timed on its own (an hg_comm failure is reported in the line, "
                         "never hangs: every hg_comm wait has a deadline)")
    ap.add_argument("--frame-split", type=int, default=-1, help="HG_OPT_FRAME_SPLIT (0 auto, 1 off, k); -1: default")
    ap.add_argument("--tile-order", type=int, default=-1, help="HG_OPT_TILE_ORDER (0 off, 1 on); -1: default")
    ap.add_argument("--wave-units", type=int, default=-1, help="HG_OPT_WAVE_UNITS (0 auto, k tiles per wave); -1: default")
    ap.add_argument("--lane-pick", type=int, default=-1, help="HG_OPT_LANE_PICK (0 in turn, 1 first idle); -1: default")
    ap.add_argument("--readback-stream", type=int, default=0, help="--per-frame-only: HG_OPT_READBACK_STREAM (1 side)")
    ap.add_argument("--server", type=int, default=-1, help="HG_OPT_SERVER (1: the render server for calls of few frames, "
                    "the default; 0: every call launches); -1: default")
    ap.add_argument("--bvh", default="reference", choices=["reference", "sah"],
                    help="BLAS builder of the timed scene: the reference's (the drop-in's parity path, the contract line) "
                         "or hg_build_blas_sah (NOT the reference's hierarchy; A/B and the fast_bvh leg)")
    ap.add_argument("--sah-leaf", type=int, default=2, help="--bvh sah: largest leaf the SAH build makes by size alone")
    ap.add_argument("--no-fast-bvh", action="store_true", help="skip the fast_bvh leg (C3 on an SAH BLAS)")
    ap.add_argument("--queue-fill", type=int, default=-1, help="HG_OPT_QUEUE_FILL (0 off, k rounds); -1: default")
    ap.add_argument("--server-ahead", type=int, default=-1, help="HG_OPT_SERVER_AHEAD (frames traced ahead); -1: default")
    ap.add_argument("--server-idle-us", type=int, default=-1, help="HG_OPT_SERVER_IDLE_US; -1: default")
    ap.add_argument("--descent-t", type=int, default=-2, help="HG_OPT_DESCENT_T (-1 auto, 0..64); -2: default")
    ap.add_argument("--no-strong", action="store_true", help="N > 1 / --emulate-ranks: skip the strong-scaling leg")
    ap.add_argument("--strong-coalesce", type=int, default=-1,
                    help="the strong leg's HG_OPT_COALESCE (frames held for one launch); -1: the library's default")
    ap.add_argument("--dist-probe", action="store_true",
                    help="launcher check, no GPU: every rank joins the process group, all-reduces its rank, rank 0 prints "
                         "one JSON line (tests/test_bench_launch.py)")
    ap.add_argument("--detail-out", default="gpurun_out/bench_detail.json",
                    help="the per-format display tables and other bulky legs (the line keeps a compact summary)")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="1-GPU rehearsal of one rank's share at N ranks (tiles t %% N == 0, N*fps frames); "
                         "reports that rank's own Mpaths/s, not a contract line")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    emu = args.emulate_ranks if world == 1 and args.emulate_ranks > 1 else 0
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = int(os.environ.get("HALOGEN_BENCH_DEVICE", local_rank))  # rehearsal: every rank on one GPU
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit(f"--gpus {args.gpus}: run bench.py as a script (it starts its {args.gpus} ranks itself) "
                             f"or under torch.distributed.run with {args.gpus} processes")
    dist = None
    if args.dist_probe:  # the launcher's check (no GPU, gloo): the ranks join, agree, and rank 0 prints one line
        import torch
        import torch.distributed as dist_mod

        if world > 1:
            dist_mod.init_process_group("gloo")
        if os.environ.get("HALOGEN_BENCH_PROBE_FAIL_RANK") == str(rank):  # (the test of a failing rank's exit status)
            raise SystemExit(3)
        t = torch.tensor([float(rank)])
        if world > 1:
            dist_mod.all_reduce(t)
        if rank == 0:
            print(json.dumps({"dist_probe": True, "world": world, "rank_sum": int(t.item()),
                              "local_ranks_device": device}), flush=True)
        if world > 1:
            dist_mod.barrier()
            dist_mod.destroy_process_group()
        return
    if world > 1:
        import torch
        import torch.distributed as dist_mod

        dist = dist_mod
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    coll_dev = f"cuda:{device}" if args.dist_backend == "nccl" else "cpu"

    cfg = scenes.CONFIGS[args.config]
    if args.width and args.height:
        cfg = cfg.resized(args.width, args.height)
    settings = scenes.settings_for(cfg)
    s = rp.clamp_settings(settings)
    t_setup = time.perf_counter()
    from halogen import scene as scene_mod

    scene_mod.SAH_MAX_LEAF = args.sah_leaf
    scene_mod.set_blas_builder(args.bvh)
    packed = cfg.build_scene().pack()
    scene_mod.set_blas_builder("reference")
    cube = settings.environmentCubemap if s["UseEnvironmentCubemap"] else None
    W, H = cfg.width, cfg.height
    params = rp.make_params(s, cfg.camera(), 1, len(packed.spheres), len(packed.meshes), cube is not None)

    ctx = abi.Context(device)
    ctx.set_option(abi.HG_OPT_KERNEL, {"auto": abi.HG_KERNEL_AUTO, "mega": abi.HG_KERNEL_MEGA,
                                       "regen": abi.HG_KERNEL_MEGA_REGEN, "stream": abi.HG_KERNEL_MEGA_STREAM}[args.kernel])
    # HIP events around every trace-kernel launch, on the trace stream it runs on (hg_counters.trace_ms): the roofline's
    # launch duration.  (kernel_ms spans a launch from its trace's start to its blend's end; consecutive launches
    # overlap on the two trace streams, so those spans overlap too.)
    ctx.set_option(abi.HG_OPT_TIMING, 1)
    if args.block:
        ctx.set_option(abi.HG_OPT_BLOCK, args.block)
    if args.frame_split >= 0:
        ctx.set_option(abi.HG_OPT_FRAME_SPLIT, args.frame_split)
    if args.tile_order >= 0:
        ctx.set_option(abi.HG_OPT_TILE_ORDER, args.tile_order)
    if args.wave_units >= 0:
        ctx.set_option(abi.HG_OPT_WAVE_UNITS, args.wave_units)
    if args.lane_pick >= 0:
        ctx.set_option(abi.HG_OPT_LANE_PICK, args.lane_pick)
    if args.server >= 0:
        ctx.set_option(abi.HG_OPT_SERVER, args.server)
    if args.descent_t >= -1:
        ctx.set_option(abi.HG_OPT_DESCENT_T, args.descent_t)
    if args.queue_fill >= 0:
        ctx.set_option(abi.HG_OPT_QUEUE_FILL, args.queue_fill)
    if args.server_ahead >= 0:
        ctx.set_option(abi.HG_OPT_SERVER_AHEAD, args.server_ahead)
    if args.server_idle_us >= 0:
        ctx.set_option(abi.HG_OPT_SERVER_IDLE_US, args.server_idle_us)
    ctx.set_option(abi.HG_OPT_COUNTERS, 0)  # timed region: production kernel (counts come from the replay below)
    ctx.upload_scene(packed)
    if cube is not None:
        ctx.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
    ctx.resize(W, H)
    ctx.set_tiling(rank, emu or world)
    ctx.set_params(params)
    comm = None
    gather_mode = args.gather

    os.environ.setdefault("HALOGEN_COMM_TIMEOUT_MS", "30000")  # hg_comm's deadline for a missing or failed peer

    def join_comm():  # hg_comm over RCCL: rank 0 makes the id, every rank joins (bounded by the comm deadline)
        box = [abi.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return abi.Comm.rank(ctx, world, box[0], rank)

    comm_init_error = None
    if dist is not None and gather_mode == "abi":
        # Every rank joins; if any rank's join fails (bounded by the comm deadline), all of them agree to time the torch
        # gather instead and the line says why (`gather_init_error`), so a broken hg_comm never costs the measurement.
        try:
            comm = join_comm()
        except abi.HalogenError as e:
            comm_init_error = f"rank {rank}: {str(e)[:300]}"
        import torch

        bad = torch.tensor([1 if comm_init_error else 0], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if int(bad.item()):
            errs = [None] * world
            dist.all_gather_object(errs, comm_init_error)
            comm_init_error = "; ".join(e for e in errs if e) or "a peer failed to join"
            if comm is not None:
                comm.close()
                comm = None
            gather_mode = "torch"
    setup_s = time.perf_counter() - t_setup

    frames_per_step = (emu or world) * args.frames_per_step  # per-GPU work fixed: image frame-equivalents per GPU
    if args.per_frame_only:  # profiling aid (tools/profile.sh): one warm-up step of the same launches, then steps x frames x hg_render(1)
        ctx.set_option(abi.HG_OPT_COALESCE, args.coalesce)
        ctx.set_option(abi.HG_OPT_COUNTERS, 0)  # (the per-frame legs run the production kernels)
        depth = 1 if args.display == "sync" else args.readback_depth
        ctx.set_option(abi.HG_OPT_READBACK_DEPTH, depth)
        ctx.set_option(abi.HG_OPT_READBACK_STREAM, args.readback_stream)
        fmt = abi.DISPLAY_FORMATS[args.display_format]
        for _ in range(frames_per_step // args.launch_frames):  # warm-up step of the timed launches (their buffers)
            ctx.render(args.launch_frames, True)
        ctx.clear_accumulation()
        ctx.set_params(params)
        ctx.reset_counters()
        ctx.synchronize()
        t0 = time.perf_counter()
        pending = 0
        host = {"render": 0.0, "begin": 0.0, "end": 0.0}  # host time inside each call (the end includes its wait)
        pc = time.perf_counter
        n_calls = args.steps * frames_per_step // args.launch_frames
        for _ in range(n_calls):
            a = pc()
            ctx.render(args.launch_frames, True)
            b = pc()
            host["render"] += b - a
            if args.display != "none":
                ctx.readback_begin(fmt)
                e = pc()
                host["begin"] += e - b
                pending += 1
                if pending == depth:
                    ctx.readback_end(W, H, copy=False)
                    host["end"] += pc() - e
                    pending -= 1
        while pending:
            ctx.readback_end(W, H, copy=False)
            pending -= 1
        ctx.synchronize()
        dt = time.perf_counter() - t0
        c = ctx.counters()
        print(json.dumps({"per_frame_only": True, "value": W * H * frames_per_step * args.steps / dt / 1e6,
                          "unit": "Mpaths/s", "launches": c["launches"], "ms_per_step": dt * 1e3 / args.steps,
                          "server_launches": c["server_launches"], "server_frames": c["server_frames"],
                          "server_ahead": c["server_ahead"],
                          "device_ms_per_frame": c["kernel_ms"] / max(c["launches"], 1),
                          "host_ms_per_call": {k: v * 1e3 / n_calls for k, v in host.items()}}), flush=True)
        ctx.close()
        return
    for _ in range(args.warmup):
        ctx.render(frames_per_step, True)
    ctx.synchronize()
    # timed region renders frames 1 .. K*N from a cleared accumulator (the C3 image at K=64, N=1)
    ctx.clear_accumulation()
    ctx.set_params(params)
    ctx.reset_counters()

    def barrier():
        ctx.synchronize()
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    gather_error = None
    for attempt in range(2):
        local = None
        if dist is not None and comm is None:  # the torch gather's staging tensor and rank 0's pixel index, untimed
            import torch

            from halogen import distributed as hd

            local = torch.empty((ctx.local_tile_count(), 64, 4), dtype=torch.float32, device=f"cuda:{device}")
            if rank == 0:
                tx, ty = hd.tiles_xy(W, H)
                hd.pixel_index(world, hd.local_tile_count(tx * ty, 0, world), W, H, torch.device(coll_dev))
        if attempt:  # the rerun after a failed hg_comm gather starts from a cleared accumulator again
            ctx.clear_accumulation()
            ctx.set_params(params)
            ctx.reset_counters()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.render(frames_per_step, True)
        gathered = None
        failed = None
        if comm is not None:
            try:
                comm.gather(0)  # enqueued on the context stream after the renders
                comm.synchronize()  # bounded wait (deadline + RCCL async errors) before the barrier's unbounded one
            except abi.HalogenError as e:
                failed = f"rank {rank}: {str(e)[:300]}"
        elif dist is not None:
            ctx.copy_tiles_device(local.data_ptr(), local.numel() * 4)
            # assembled on rank 0's device (as the N=1 image stays in the accumulator); to the host after the clock
            gathered = hd.gather_tiles(local.to(coll_dev), rank, world, W, H, on_device=True)
        barrier()
        dt = time.perf_counter() - t0
        if comm is not None:
            # after the clock: if any rank's hg_comm gather failed, every rank reruns the timed region with the torch
            # gather and the line says why (`gather_error`), so a broken transport never costs the measurement
            import torch

            bad = torch.tensor([1 if failed else 0], dtype=torch.int32, device=coll_dev)
            dist.all_reduce(bad, op=dist.ReduceOp.MAX)
            if int(bad.item()) and attempt == 0:
                errs = [None] * world
                dist.all_gather_object(errs, failed)
                gather_error = "; ".join(e for e in errs if e) or "a peer's gather failed"
                try:
                    comm.close()
                except abi.HalogenError:
                    pass
                comm = None
                gather_mode = "torch"
                continue
        break
    if comm is not None and rank == 0:
        gathered = comm.readback(W, H)
    elif gathered is not None:
        gathered = gathered.cpu().numpy()

    abi_check = None
    gather_ms = {}
    if dist is not None and not args.no_abi_check and comm_init_error is None and gather_error is None:
        import torch

        from halogen import distributed as hd

        def time_gather(fn):  # one gather alone, barrier + device sync on both sides, max over ranks (ms)
            barrier()
            t = time.perf_counter()
            out = fn()
            barrier()
            v = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            return out, float(v.item()) * 1e3

        def torch_gather():
            loc = torch.empty((ctx.local_tile_count(), 64, 4), dtype=torch.float32, device=f"cuda:{device}")
            ctx.copy_tiles_device(loc.data_ptr(), loc.numel() * 4)
            return hd.gather_tiles(loc.to(coll_dev), rank, world, W, H, on_device=True)

        def abi_gather(cm):
            cm.gather(0)
            cm.synchronize()
            return None

        # untimed cross-check: the other transport gathers the same accumulators; both gathers are also timed alone
        try:
            if comm is not None:  # timed: hg_comm; check: torch
                _, gather_ms["abi"] = time_gather(lambda: abi_gather(comm))
                timg, gather_ms["torch"] = time_gather(torch_gather)
                same = bool(np.array_equal(timg.cpu().numpy().view(np.uint32), np.asarray(gathered).view(np.uint32))) \
                    if rank == 0 else None
                abi_check = {"ok": True, "checked_with": "torch all_gather_into_tensor", "bit_identical_to_timed_gather": same}
            elif args.dist_backend == "nccl":  # timed: torch; check: hg_comm
                _, gather_ms["torch"] = time_gather(torch_gather)
                with join_comm() as c2:
                    _, gather_ms["abi"] = time_gather(lambda: abi_gather(c2))
                    same = None
                    if rank == 0:
                        img2 = c2.readback(W, H)
                        same = bool(np.array_equal(img2.view(np.uint32), np.asarray(gathered).view(np.uint32)))
                    abi_check = {"ok": True, "checked_with": f"hg_comm (transport {c2.transport})",
                                 "bit_identical_to_timed_gather": same}
        except abi.HalogenError as e:
            abi_check = {"ok": False, "error": str(e)[:400]}

    timing = ctx.counters()  # kernel_ms / launches of the timed launches
    kernel_symbol = KERNEL_SYMBOL.get(int(timing["last_kernel"]), "?")  # the variant HG_KERNEL_AUTO resolved to
    replay_identical = None
    timed_img = ctx.readback(W, H) if world == 1 and (not args.no_counters or args.save_image) else None
    if not args.no_counters:
        # Counting replay, untimed: the same K steps from the same cleared state with the device counters on give
        # the exact traversal counts of the timed launches (the render is deterministic — checked on the image).
        ctx.clear_accumulation()
        ctx.set_params(params)
        ctx.reset_counters()
        ctx.set_option(abi.HG_OPT_COUNTERS, 1)
        for _ in range(args.steps):
            ctx.render(frames_per_step, True)
        ctx.synchronize()
        if timed_img is not None:
            replay_identical = bool(np.array_equal(timed_img.view(np.uint32), ctx.readback(W, H).view(np.uint32)))
    cnt = ctx.counters()
    for k in ("kernel_ms", "launches", "trace_ms", "trace_launches", "trace_busy_ms"):
        cnt[k] = timing[k]
    if dist is not None:
        import torch

        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        keys = ["paths", "rays", "tri_tests", "aabb_tests", "mesh_visits", "sphere_tests", "hits", "primary_misses"]
        v = torch.tensor([float(cnt[k]) for k in keys], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(v)
        totals = dict(zip(keys, (int(x) for x in v.tolist())))
    else:
        totals = cnt

    strong = None
    if (dist is not None or emu) and not args.no_strong:
        def strong_gather():
            if comm is not None:
                comm.gather(0)
                comm.synchronize()
                return comm.readback(W, H) if rank == 0 else None
            import torch

            from halogen import distributed as hd

            loc = torch.empty((ctx.local_tile_count(), 64, 4), dtype=torch.float32, device=f"cuda:{device}")
            ctx.copy_tiles_device(loc.data_ptr(), loc.numel() * 4)
            return hd.gather_tiles(loc.to(coll_dev), rank, world, W, H, on_device=True)

        ref_img = None
        if rank == 0 and dist is not None:  # the same frames on one context, all tiles (untimed)
            with abi.Context(device) as one:
                one.upload_scene(packed)
                if cube is not None:
                    one.upload_cubemap(cube.face_size, cube.n_mips, cube.texels)
                one.resize(W, H)
                one.set_params(params)
                for _ in range(args.steps):
                    one.render(args.frames_per_step, True)
                ref_img = one.readback(W, H)
        strong = strong_scaling_measurement(ctx, params, W, H, args.frames_per_step, args.steps, world, rank, emu,
                                            barrier, strong_gather, coll_dev, dist, ref_img, args.strong_coalesce)

    total_paths = W * H * frames_per_step * args.steps
    if emu:  # this GPU traced only its 1/N share of the tiles
        total_paths = ctx.local_tile_count() * 64 * frames_per_step * args.steps
    result = None
    if rank == 0:
        launches = max(cnt["launches"], 1)
        # the trace kernel's own launch duration (events on its stream; what rocprofv3 --stats averages)
        if cnt.get("trace_launches"):
            mean_launch_s, span_s = launch_seconds(cnt)
        else:
            mean_launch_s, span_s = cnt["kernel_ms"] / launches / 1e3, 0.0
        counters_ok = not args.no_counters and cnt["paths"] > 0
        # §8(d)'s byte model: LOGICAL bytes per launch (every node / triangle / record read the algorithm makes,
        # whether L1/L2/Infinity Cache or HBM serves it) — a work measure, not a bound on this cache-resident kernel
        logical_per_launch = algorithmic_bytes(cnt) / launches if counters_ok else None
        pmc = committed_counters(args.config, W, H, frames_per_step, kernel_symbol)
        roofline = roofline_of(pmc, mean_launch_s, logical_per_launch, kernel_symbol,
                               dt / max(args.steps, 1) if launches == args.steps else 0.0, span_s)
        result = {
            "metric": METRIC,
            "value": total_paths / dt / 1e6,
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (scene rebuilt from the reference's scene constants; Dragon_8k.fbx subdivided 10x)",
            "config": {"workload": cfg.name, "width": W, "height": H, "frames_per_step": frames_per_step,
                       "spp_total": frames_per_step * args.steps, "max_bounces": s["MaxBounces"],
                       "triangles": len(packed.triangles), "blas_nodes": len(packed.blas),
                       "parallelism": f"tiles{world}"},
            "mrays_per_s": totals["rays"] / dt / 1e6 if counters_ok else None,
            "roofline": roofline,
            "counters_per_path": {k: totals[k] / max(totals["paths"], 1) for k in
                                  ("rays", "tri_tests", "aabb_tests", "hits")} if counters_ok else None,
            # share of the paths whose camera ray hits nothing (from C3's camera ~54 % leave through the open front
            # as one ray): Mpaths/s counts them as paths, Mrays/s counts their single ray
            "primary_miss_frac": totals["primary_misses"] / max(totals["paths"], 1) if counters_ok else None,
            "counting_replay_bit_identical": replay_identical,
            "simd_utilisation": {"descent": cnt["aabb_tests"] / 2 / max(64 * cnt["node_rounds"], 1),
                                 "leaf": cnt["tri_tests"] / max(64 * cnt["tri_rounds"], 1),
                                 "shading": (cnt["rays"] / (64 * cnt["shade_rounds"])) if cnt.get("shade_rounds")
                                 else None} if counters_ok else None,
            # wave-clock split of the counting replay (regenerating / streaming megakernels)
            "phase_split": {"traversal": cnt["trace_cycles"] / (cnt["trace_cycles"] + cnt["shade_cycles"]),
                            "shading": cnt["shade_cycles"] / (cnt["trace_cycles"] + cnt["shade_cycles"])}
            if counters_ok and cnt.get("trace_cycles", 0) + cnt.get("shade_cycles", 0) > 0 else None,
            # analysis builds (HG_PHASE_DETAIL=1): the shading phase split further, as fractions of all wave cycles
            "shading_detail": dict(zip(("hit_resolve", "material_bsdf", "path_end_camera", "next_ray_setup"),
                                       (x / (cnt["trace_cycles"] + cnt["shade_cycles"]) for x in cnt["shade_detail"])))
            if counters_ok and any(cnt.get("shade_detail", [])) else None,
            "emulated_ranks": emu or None,
            # N > 1: the same image's work split over the ranks (strong scaling), beside the weak line above
            "strong_scaling": strong,
            # N > 1: every pixel of the gathered image was written by some rank (alpha of a blended pixel is ~1)
            "gather_complete": bool((gathered[..., 3] > 0.5).all().item()) if gathered is not None else None,
            "gather": (gather_mode + (f" (hg_comm transport {comm.transport})" if comm is not None else
                                      " (all_gather_into_tensor, assembled on rank 0's device through "
                                      "hg_comm_assemble_host's pixel index)"))
            if dist is not None else None,
            "abi_gather_check": abi_check,
            "gather_init_error": comm_init_error,
            "gather_error": gather_error,
            # each gather alone (after the timed region; max over ranks): the one `gather` names is inside `value`
            "gather_ms": gather_ms or None,
            "setup_s": setup_s,
            "kernel_ms": {"pipeline_total": cnt["kernel_ms"], "pipelines": cnt["launches"],
                          "trace_total": cnt["trace_ms"], "trace_busy": cnt.get("trace_busy_ms"),
                          "trace_launches": cnt["trace_launches"]},
            "cpu_baseline": None,
        }
        if args.save_image:
            img = (gathered if isinstance(gathered, np.ndarray) else gathered.cpu().numpy()) if gathered is not None \
                else timed_img
            np.save(args.save_image, img)
        if world == 1 and not emu and not args.no_per_frame:
            result["per_frame"] = per_frame_measurement(ctx, params, W, H, frames_per_step, max(2, args.steps),
                                                        result["value"])
        if world == 1 and not emu and not args.no_per_frame:
            result["camera_move"] = camera_move_measurement(ctx, packed, s, cfg, W, H, 32, cube)
        if world == 1 and not emu and args.config == "C3" and not args.no_counters and not args.no_framed:
            result["framed"] = framed_measurement(ctx, packed, s, W, H, frames_per_step, max(2, args.steps // 4))
        if (world == 1 and not emu and args.config == "C3" and args.bvh == "reference" and not args.no_fast_bvh
                and timed_img is not None):
            result["fast_bvh"] = fast_bvh_measurement(ctx, cfg, packed, cube, params, W, H, frames_per_step, args.steps,
                                                      timed_img, result["value"])
        if world == 1 and not args.no_cpu_baseline:
            # the box's CPU share is 16 (OMP_NUM_THREADS there); never more threads than CPUs this process may use
            threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                                 else (os.cpu_count() or 1)))
            result["cpu_baseline"] = cpu_baseline(packed, params, cube, W, H, args.cpu_seconds, threads)
        if strong and strong.get("value"):
            # the strong leg's rate per GPU against this line's weak rate per GPU (N ranks: both totals over N GPUs;
            # --emulate-ranks: both rank 0's share on its one GPU, so the ratio is the same quantity)
            strong["per_gpu_frac_of_weak"] = strong["value"] / result["value"]
        split_detail(result, args.detail_out)
        result["summary"] = compact_summary(result)
        print(json.dumps(result), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
