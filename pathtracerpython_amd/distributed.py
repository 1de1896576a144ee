"""Multi-GPU rendering: image rows sharded across ranks, one gather to rank 0.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).  The
reference's only parallelism is a process pool over rays (main.py:197-231);
every (pixel, sample) is independent under the keyed RNG, so ranks need no
exchange until the end.  Rank r renders the rows iy with iy % world == r
(interleaved bands: neighbouring rows cost about the same, so every rank gets
an even share of cheap escape rows and expensive box rows), then a single
gather of the fixed-size row tiles to rank 0 assembles the framebuffer.

The partition and assembly are pure functions so the CPU test suite can run
them over gloo with world_size 2 (tests/test_distributed.py).
"""
import numpy as np


def rank_band(height, rank, world):
    """pt_render_params row selection of `rank`: (row_begin, row_end,
    row_step, row_phase)."""
    return 0, height, world, rank


def band_rows_of(height, rank, world):
    """iy values rank renders, in framebuffer (top-first) order."""
    return list(range(rank, height, world))[::-1]


def max_band_rows(height, world):
    return (height + world - 1) // world


def assemble(tiles, height):
    """tiles[r]: (max_rows, W, 3) array, the first len(band_rows_of(r)) rows
    valid (top-first).  Returns the (H, W, 3) framebuffer."""
    world = len(tiles)
    W = tiles[0].shape[1]
    fb = np.zeros((height, W, 3), dtype=tiles[0].dtype)
    for r, tile in enumerate(tiles):
        rows = band_rows_of(height, r, world)
        for j, iy in enumerate(rows):
            fb[height - 1 - iy] = tile[j]
    return fb


def gather_tiles(tile, group=None):
    """Gather equal-shape tiles (torch tensors) to rank 0; returns the list on
    rank 0 and None elsewhere.  With the nccl backend this is one RCCL gather
    over xGMI."""
    import torch.distributed as dist
    import torch
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if world == 1:
        return [tile]
    bufs = [torch.empty_like(tile) for _ in range(world)] if rank == 0 else None
    dist.gather(tile, gather_list=bufs, dst=0, group=group)
    return bufs


def deinterleave(gathered, out):
    """Frame from the gathered row tiles of an interleaved split whose height
    is a multiple of the world size, as one tensor copy (on the tiles'
    device): gathered (world, rows, W, 3), tile r row j (top-first) = image
    row iy = r + world*(rows-1-j) = frame row world*j + (world-1-r).  out:
    (world*rows, W, 3)."""
    world, rows = gathered.shape[0], gathered.shape[1]
    out.view(rows, world, *gathered.shape[2:]).copy_(gathered.flip(0).permute(1, 0, 2, 3))
    return out


def assemble_bands_device(gathered, out, stream=None):
    """The frame from the gathered row tiles of an interleaved split, on the
    GPU (pt_assemble_bands_device, one HBM-bound kernel; any height, also
    ragged bands): gathered (world, max_rows, W, 3) float32/float64 device
    tensor, out (H, W, 3) of the same dtype.  Asynchronous on `stream` (a
    hipStream_t handle; default: torch's current stream)."""
    import ctypes as C
    import torch
    from . import _native
    from ._abi import PT_FLAG_OUT_F64
    if gathered.dtype != out.dtype or gathered.dtype not in (torch.float32, torch.float64):
        raise ValueError("gathered and out must both be float32 or both float64")
    if not (gathered.is_contiguous() and out.is_contiguous()):
        raise ValueError("gathered and out must be contiguous")
    world, max_rows, W = gathered.shape[0], gathered.shape[1], gathered.shape[2]
    H = out.shape[0]
    if out.shape[1:] != (W, 3) or gathered.shape[3] != 3:
        raise ValueError("shapes must be (world, max_rows, W, 3) and (H, W, 3)")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    flags = PT_FLAG_OUT_F64 if gathered.dtype == torch.float64 else 0
    _native.check(_native.lib().pt_assemble_bands_device(
        C.c_void_p(gathered.data_ptr()), world, max_rows, W, H, flags, C.c_void_p(out.data_ptr()),
        C.c_void_p(stream)), "pt_assemble_bands_device")
    return out


def render_distributed(renderer, width, height, spp=1, bounces=1, seed=None, rr=False,
                       rr_depth=3, group=None, return_tiles=False):
    """Render `height` rows interleaved over the ranks of `group` on each
    rank's current CUDA/HIP device; returns the framebuffer (float32 numpy) on
    rank 0 and None on the other ranks."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rb, re, step, phase = rank_band(height, rank, world)
    p = renderer.params(width, height, spp, bounces, seed, rr, rr_depth, row_begin=rb,
                        row_end=re, row_step=step, row_phase=phase)
    rows = max_band_rows(height, world)
    tile = torch.zeros((rows, width, 3), dtype=torch.float32, device="cuda")
    renderer.render_device(p, tile.data_ptr(), torch.cuda.current_stream().cuda_stream)
    tiles = gather_tiles(tile, group) if world > 1 else [tile]
    if rank != 0:
        return None
    host = [t.cpu().numpy() for t in tiles]
    if return_tiles:
        return host
    return assemble(host, height)
