"""Multi-GPU framebuffer tiling (not in the reference, which is single-GPU).

Pixels are independent: a pixel's value depends only on the scene, the uniforms, its GLOBAL index and
FrameCount (HalgoenCompute.compute:1033).  So the image's 8x8 tiles are dealt round-robin to ranks
(tile t -> rank t % N, which balances the centre-heavy dragon), every rank traces and accumulates all
frames of its own tiles, and the only collective is one gather of the packed accumulated tiles at the end.

This module is the torch.distributed form of that gather (backend "nccl" = RCCL over xGMI on ROCm, "gloo" in the CPU
tests and the one-GPU rehearsal): one all_gather_into_tensor of every rank's tiles, then the image is assembled on
the host by hg_comm_assemble_host, the host twin of the C-ABI gather's device assembly (hg_comm_gather), which reads
pixels through the same tile -> rank / slot / pixel mapping (csrc/hg_tiling.h).  The gathered image is bit-identical
to a 1-GPU render (tests/test_gpu_parity.py, tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import abi

TILE = 8


def tiles_xy(width: int, height: int) -> tuple[int, int]:
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def local_tile_count(total_tiles: int, rank: int, n_ranks: int) -> int:
    return max(0, (total_tiles - rank + n_ranks - 1) // n_ranks)


_PIXEL_INDEX: dict = {}


def pixel_index(n_ranks: int, max_local: int, width: int, height: int, device) -> torch.Tensor:
    """For every pixel of the (height, width) image, its float4 slot in the gathered (n_ranks, max_local, 64) tiles:
    hg_comm_assemble_host's mapping (csrc/hg_tiling.h, the device gather's), evaluated once on the slot numbers
    themselves (exact in float32 below 2^24 slots) and cached per shape and device."""
    key = (n_ranks, max_local, width, height, str(device))
    if key not in _PIXEL_INDEX:
        n = n_ranks * max_local * 64
        if n >= 1 << 24:
            raise ValueError(f"{n} tile slots: beyond the float32-exact index map")
        slots = np.repeat(np.arange(n, dtype=np.float32).reshape(n_ranks, max_local, 64, 1), 4, axis=3)
        img = abi.assemble_host(slots, width, height, n_ranks)
        _PIXEL_INDEX[key] = torch.from_numpy(img[..., 0].astype(np.int64).reshape(-1)).to(device)
    return _PIXEL_INDEX[key]


def gather_tiles(local: torch.Tensor, rank: int, n_ranks: int, width: int, height: int,
                 on_device: bool = False):
    """local: (n_local_tiles, 64, 4) float32 tiles of this rank (hg_copy_tiles_device layout).
    Returns the (height, width, 4) image on rank 0 (None elsewhere).  One all_gather_into_tensor of
    max-local-tiles x 1 KiB per rank (ranks hold ceil/floor shares, padded to the max).  on_device: the image is
    assembled where the gather landed (one index_select through pixel_index) and returned as a tensor there, as the
    C-ABI gather leaves it on the root GPU; else on the host (hg_comm_assemble_host)."""
    tx, ty = tiles_xy(width, height)
    total = tx * ty
    max_local = local_tile_count(total, 0, n_ranks)
    buf = torch.zeros((max_local, 64, 4), dtype=torch.float32, device=local.device)
    buf[: local.shape[0]] = local
    out = torch.empty((n_ranks * max_local, 64, 4), dtype=torch.float32, device=local.device)
    dist.all_gather_into_tensor(out, buf)
    if rank != 0:
        return None
    if on_device:
        idx = pixel_index(n_ranks, max_local, width, height, out.device)
        return out.view(-1, 4).index_select(0, idx).view(height, width, 4)
    return untile(out.view(n_ranks, max_local, 64, 4), n_ranks, width, height)


def untile(per_rank, n_ranks: int, width: int, height: int) -> np.ndarray:
    """(n_ranks, max_local, 64, 4) slabs -> (height, width, 4): global tile g lives at rank g % N, slot g // N
    (hg_comm_assemble_host, the mapping of the device gather)."""
    slabs = per_rank.cpu().numpy() if isinstance(per_rank, torch.Tensor) else np.asarray(per_rank)
    return abi.assemble_host(slabs, width, height, n_ranks)
