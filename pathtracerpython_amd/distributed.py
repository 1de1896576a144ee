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

Two ways to make the frame:
  * device frame: each rank renders its band into a device tile, ONE gather
    of the tiles to rank 0 (RCCL over xGMI with the nccl backend) and a
    device assembly kernel put the frame in rank 0's HBM (gather_tiles,
    assemble_bands_device) — for consumers on the GPU (the device image
    finalisation, a PNG);
  * host frame (HostFrame): the ranks of one node share a frame in
    page-locked host memory (a /dev/shm mapping) and each GPU's render
    writes its band straight into its rows, over its own PCIe link while the
    kernel runs; a per-rank flag written after the render on its stream tells
    rank 0 the frame is complete.  No gather and no separate device-to-host
    copy: this is the frame SURVEY.md §8(d)'s metric asks for (kernel + D2H:
    the framebuffer in host memory), at N GPUs as at one.
"""
import ctypes as C
import mmap
import os
import secrets

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
                       rr_depth=3, group=None, return_tiles=False, transport="device"):
    """Render `height` rows interleaved over the ranks of `group` on each
    rank's current CUDA/HIP device; returns the framebuffer (float32 numpy) on
    rank 0 and None on the other ranks.
    transport "device": each band into a device tile, one gather to rank 0
    (RCCL with the nccl backend); "host": every band straight into one shared
    page-locked host frame (HostFrame; the ranks of one node)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rb, re, step, phase = rank_band(height, rank, world)
    p = renderer.params(width, height, spp, bounces, seed, rr, rr_depth, row_begin=rb,
                        row_end=re, row_step=step, row_phase=phase)
    if transport == "host":
        if return_tiles:
            raise ValueError("return_tiles needs the device transport")
        from ._native import NativeError
        name = [HostFrame.new_name() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(name, src=0, group=group)

        def agree(err):
            """Every rank learns the first rank's error (or None) before any
            rank renders or waits, so no rank is left in a barrier or rank 0
            spinning on a flag that never comes."""
            if world == 1:
                return err
            errs = [None] * world
            dist.all_gather_object(errs, err, group=group)
            return next((e for e in errs if e), None)

        def attempt(fn):
            try:
                return fn(), None
            except Exception as e:   # noqa: BLE001 (re-raised on every rank)
                return None, f"rank {rank}: {type(e).__name__}: {e}"
        hf, err = (attempt(lambda: HostFrame(height, width, world, rank, name[0], create=True))
                   if rank == 0 else (None, None))
        if world > 1:
            # rank 0's file exists (or its error is known) before the others open it
            first = agree(err)
            if first is None and rank != 0:
                hf, err = attempt(lambda: HostFrame(height, width, world, rank, name[0]))
            err = first or agree(err)
        try:
            if err:
                raise NativeError(f"host frame: {err}")
            _, err = attempt(lambda: hf.render(renderer, p, 0, torch.cuda.current_stream().cuda_stream))
            err = agree(err)
            if err:
                raise NativeError(f"host frame render: {err}")
            fb = hf.wait(0).copy() if rank == 0 else None
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier(group=group)
        finally:
            if hf is not None:
                hf.close()
        return fb
    if transport != "device":
        raise ValueError(f"transport must be 'device' or 'host', not {transport!r}")
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


class HostFrame:
    """A (height, width, 3) framebuffer ring in page-locked host memory shared
    by the `world` rank processes of one node (/dev/shm/<name>), which each
    GPU renders its interleaved band into directly (include/pt_capi.h: host
    frames).  `slots` frames rotate so a rank can render step s + 1 while
    rank 0 still reads step s; a rank waits before reusing a slot until rank 0
    has released the step that last used it.

    Layout: a 4096-B header — ready[r] (the last step + 1 rank r's band of
    which is in the frame; written by the GPU, pt_signal) at byte 64 r,
    released[slot] (the last step + 1 rank 0 is done with in that slot) at
    byte 2048 + 64 slot — then the slots' frames.

    Rank 0 creates the file (create=True) and hands its name to the others;
    close() unmaps it and rank 0 removes it."""

    HEADER = 4096
    READY, RELEASED = 0, 2048

    def __init__(self, height, width, world, rank, name, slots=2, dtype=np.float32, create=False,
                 map_device=True):
        """map_device=False: the shared memory and its flags only, no HIP
        mapping (no render(); the CPU tests of the protocol use it)."""
        from . import _native
        if world > 32 or slots > 32:
            raise ValueError("at most 32 ranks and 32 slots")
        self.H, self.W, self.world, self.rank, self.slots = height, width, world, rank, slots
        self.dtype = np.dtype(dtype)
        self.frame_bytes = height * width * 3 * self.dtype.itemsize
        self.bytes = self.HEADER + slots * self.frame_bytes
        self.path = os.path.join("/dev/shm", name)
        self.owner = create
        if create:   # a tmpfs too small for the frame would SIGBUS on first touch
            st = os.statvfs("/dev/shm")
            if st.f_bavail * st.f_frsize < self.bytes:
                raise OSError(f"/dev/shm has {st.f_bavail * st.f_frsize} B free, the host frame "
                              f"needs {self.bytes} B")
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, self.bytes)
            self._mm = mmap.mmap(fd, self.bytes, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        except BaseException:
            if create:   # no half-made frame left in /dev/shm
                os.unlink(self.path)
            raise
        finally:
            os.close(fd)
        self._cbuf = C.c_char.from_buffer(self._mm)
        self.host = C.addressof(self._cbuf)
        self._lib = _native.lib()
        self.dev = None
        self._rendered = False
        if map_device:
            dev = C.c_void_p()
            rc = self._lib.pt_host_map(C.c_void_p(self.host), self.bytes, C.byref(dev))
            if rc != 0:
                err = _native.last_error()
                self.close()
                raise _native.NativeError(f"pt_host_map failed ({rc}): {err}")
            self.dev = dev.value
        self.u64 = np.frombuffer(self._mm, dtype=np.uint64, count=self.HEADER // 8)
        self._iy_top = max(iy for iy in range(rank, height, world)) if rank < height else None
        self.band_rows = list(range(rank, height, world))[::-1]   # iy, top row first

    @staticmethod
    def new_name():
        return f"pt_frame_{os.getpid()}_{secrets.token_hex(4)}"

    def frame(self, step):
        """The frame of `step` (numpy view of the shared memory)."""
        off = self.HEADER + (step % self.slots) * self.frame_bytes
        return np.frombuffer(self._mm, dtype=self.dtype, count=self.H * self.W * 3,
                             offset=off).reshape(self.H, self.W, 3)

    def band_target(self, step):
        """(device address, out_row_stride) of this rank's band in the frame of
        `step`: its top row (iy_top, image row H-1-iy_top), every world-th row."""
        if self._iy_top is None or self.dev is None:
            return None, 0
        off = self.HEADER + (step % self.slots) * self.frame_bytes + \
            (self.H - 1 - self._iy_top) * self.W * 3 * self.dtype.itemsize
        return self.dev + off, self.world * self.W * 3

    def render(self, renderer, p, step, stream, timeout_s=300.0, events=None):
        """Enqueue this rank's band of `step` on `stream` (asynchronous): wait
        (host) until the slot is released, render into the frame, then the
        ready flag.  p: this rank's band params (row_step = world,
        row_phase = rank, out_row_stride 0).  events: optional (start, end)
        torch.cuda.Events recorded around the render launch."""
        from . import _native
        from ._abi import with_flags
        need = step - self.slots + 1
        if need > 0:
            slot = step % self.slots
            _native.check(self._lib.pt_wait_flags(
                C.c_void_p(self.host + self.RELEASED + 64 * slot), 1, 8, need, timeout_s),
                "pt_wait_flags (slot release)")
        if self.dev is None:
            raise ValueError("HostFrame opened with map_device=False: no device renders")
        ptr, stride = self.band_target(step)
        if events:
            events[0].record()
        if ptr is not None:
            renderer.render_device(with_flags(p, out_row_stride=stride), ptr, stream)
        if events:
            events[1].record()
        self._rendered = True
        _native.check(self._lib.pt_signal(C.c_void_p(self.dev + self.READY + 64 * self.rank),
                                          step + 1, C.c_void_p(stream or 0)), "pt_signal")

    def wait(self, step, timeout_s=300.0):
        """Host: until every rank's band of `step` is in the frame."""
        from . import _native
        _native.check(self._lib.pt_wait_flags(C.c_void_p(self.host + self.READY), self.world, 8,
                                              step + 1, timeout_s), "pt_wait_flags (frame ready)")
        return self.frame(step)

    def release(self, step):
        """Rank 0: done with the frame of `step` (its slot may be reused)."""
        self.u64[(self.RELEASED + 64 * (step % self.slots)) // 8] = step + 1

    def close(self):
        if getattr(self, "_mm", None) is None:
            return
        from . import _native
        if self.dev is not None:
            if self._rendered:
                # renders into the frame may still be running (an error
                # between render() and wait()): unmap only after they finish
                import torch
                torch.cuda.synchronize()
            self.dev = None
            _native.check(self._lib.pt_host_unmap(C.c_void_p(self.host)), "pt_host_unmap")
        self.u64 = None
        del self._cbuf
        try:
            self._mm.close()
        except BufferError:   # a caller still holds a frame() view: unmapped with it
            pass
        self._mm = None
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass

    def discard(self):
        """On the way out of a process that cannot close() cleanly (renders
        may still be writing): remove the shared file (rank 0), nothing else."""
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
