"""Experiment (round 4): where the framebuffer's trip to host memory costs.

K2 frame (512^2 x 64 spp x 4 bounces) and one rank's band of the 8-way
interleaved split, on one MI355X:
  device   : render into HBM (the bench's round-3 timed step)
  d2h      : render into HBM + the PCIe copy to pinned host memory
  hostframe: render straight into a page-locked /dev/shm frame (HostFrame),
             pt_signal + pt_wait_flags per step, the next step enqueued
             before waiting for this one
For the band also the strided 2-D copy of the band into its frame rows.
Prints one JSON line per case (median ms per step / per launch) and checks
every host-frame result bitwise against the device render.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.distributed import HostFrame  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402
from pathtracerpython_amd._abi import with_flags  # noqa: E402

W = H = 512
SPP, B, SEED = 64, 4, 9
N = int(os.environ.get("EXP_STEPS", "40"))


def timed(fn, n, stream):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def kernel_ms(r, p, ptr, stream, n=20):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        r.render_device(p, ptr, stream)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    scene_reader.VERBOSE = False
    sc = scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl"))
    r = Renderer(sc)
    st = torch.cuda.current_stream()
    s = st.cuda_stream
    for world, phase in ((1, 0), (8, 0)):
        p = r.params(W, H, SPP, B, SEED, row_step=world, row_phase=phase)
        rows = r.band_rows(p)
        tile = torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda")
        host = torch.empty((rows, W, 3), dtype=torch.float32).pin_memory()
        out = {"case": f"N={world} band (phase {phase})", "rows": rows}
        out["kernel_device_ms"] = kernel_ms(r, p, tile.data_ptr(), s)
        out["step_device_ms"] = timed(lambda i: r.render_device(p, tile.data_ptr(), s), N, st)
        ref = tile.cpu().numpy().copy()

        def d2h(i):
            r.render_device(p, tile.data_ptr(), s)
            host.copy_(tile, non_blocking=True)
        out["step_d2h_ms"] = timed(d2h, N, st)
        t = []
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            host.copy_(tile, non_blocking=True)
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e3)
        out["d2h_alone_ms"] = float(np.median(t))
        with HostFrame(H, W, world, phase, HostFrame.new_name(), create=True) as hf:
            ptr, stride = hf.band_target(0)
            pk = with_flags(p, out_row_stride=stride)
            out["kernel_hostframe_ms"] = kernel_ms(r, pk, ptr, s)
            # strided copy of the device band into its frame rows
            import ctypes as C
            hip = C.CDLL("libamdhip64.so")
            t = []
            for _ in range(20):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rc = hip.hipMemcpy2DAsync(C.c_void_p(hf.host + (ptr - hf.dev)), C.c_size_t(stride * 4),
                                          C.c_void_p(tile.data_ptr()), C.c_size_t(W * 12),
                                          C.c_size_t(W * 12), C.c_size_t(rows), 2, C.c_void_p(s))
                assert rc == 0
                torch.cuda.synchronize()
                t.append((time.perf_counter() - t0) * 1e3)
            out["band_copy2d_ms"] = float(np.median(t))
            if world == 1:
                # the pipelined host-frame loop (enqueue s + 1, wait s, release s)
                def loop(n):
                    hf.render(r, p, 0, s)
                    for i in range(n):
                        if i + 1 < n:
                            hf.render(r, p, i + 1, s)
                        hf.wait(i)
                        hf.release(i)
                loop(3)
                torch.cuda.synchronize()
                # (the ring restarts: flags only grow, so keep counting)
                base = 3
                hf.render(r, p, base, s)
                t0 = time.perf_counter()
                for i in range(base, base + N):
                    if i + 1 < base + N:
                        hf.render(r, p, i + 1, s)
                    hf.wait(i)
                    hf.release(i)
                out["step_hostframe_ms"] = (time.perf_counter() - t0) / N * 1e3
                torch.cuda.synchronize()
                got = hf.frame(base + N - 1).copy()
                out["hostframe_bitwise"] = bool(np.array_equal(got, ref))
                del got
            else:
                got = hf.frame(0)[H - 1 - max(range(phase, H, world))::world].copy()
                out["hostframe_bitwise"] = bool(np.array_equal(got, ref))
        print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
