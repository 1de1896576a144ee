"""Dev tool: what one GPU's share of an N-GPU strong-scaling K2 step costs
(DESIGN.md §8), the framebuffer's trip to host memory included (SURVEY.md
§8(d): kernel + D2H).  For the built library (or PT_HIP_LIB), at N = 1/2/4/8
and for one rank's interleaved row band (row_step N, phases 0 and N-1),
median of the last half of `launches`:
  band_kernel_ms       the band rendered into a device tile (HIP events)
  host_kernel_ms       the band rendered straight into its rows of a
                       page-locked host frame (distributed.HostFrame)
  host_step_ms         bench.py's host-frame step as this rank runs it: the
                       band into the frame + pt_signal, the next step queued
                       before waiting (pt_wait_flags) for this one's flag —
                       wall time per step over `launches` steps
Then the fixed legs of the device-frame transport on this GPU: the device
assembly of gathered tiles and the PCIe copy of the 3 MB frame.  The RCCL
gather itself needs N GPUs (two ranks on one device are refused).
Prints one JSON object per line.
Usage: prof_scaling.py [launches] [N...]"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from pathtracerpython_amd import _native, scene_reader  # noqa: E402
from pathtracerpython_amd.distributed import HostFrame, deinterleave  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402

scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
Ns = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
lib = os.path.basename(os.environ.get("PT_HIP_LIB", "libpt_hip.so"))
torch.cuda.set_device(0)
W = H = 512
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
tile = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()


def kernel_ms(p, ptr):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        r.render_device(p, ptr, s.cuda_stream)
        b.record()
    torch.cuda.synchronize()
    return statistics.median([a.elapsed_time(b) for a, b in ev][n // 2:])


for N in Ns:
    for phase in sorted({0, N - 1}):
        p = r.params(W, H, 64, 4, 9, row_begin=0, row_end=H, row_step=N, row_phase=phase)
        rec = {"lib": lib, "N": N, "phase": phase}
        rec["band_kernel_ms"] = round(kernel_ms(p, tile.data_ptr()), 4)
        with HostFrame(H, W, N, phase, HostFrame.new_name(), create=True) as hf:
            ptr, stride = hf.band_target(0)
            rec["host_kernel_ms"] = round(kernel_ms(r.params(W, H, 64, 4, 9, row_step=N, row_phase=phase,
                                                             out_row_stride=stride), ptr), 4)
            own = C.c_void_p(hf.host + hf.READY + 64 * phase)

            def wait(step):
                _native.check(_native.lib().pt_wait_flags(own, 1, 8, step + 1, 60.0), "pt_wait_flags")
                hf.release(step)

            def loop(first, k):
                hf.render(r, p, first, s.cuda_stream)
                for i in range(first, first + k):
                    if i + 1 < first + k:
                        hf.render(r, p, i + 1, s.cuda_stream)
                    wait(i)
            loop(0, 5)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loop(5, n)
            rec["host_step_ms"] = round((time.perf_counter() - t0) / n * 1e3, 4)
            torch.cuda.synchronize()
        rec["x_N"] = round(rec["host_step_ms"] * N, 4)
        print(json.dumps(rec), flush=True)


def ev_time(fn, reps=50):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


if lib == "libpt_hip.so":
    from pathtracerpython_amd.distributed import assemble_bands_device
    for N in (2, 4, 8):
        g = torch.rand((N, H // N, W, 3), device="cuda")
        f = torch.empty((H, W, 3), device="cuda")
        print(json.dumps({"leg": "deinterleave_torch", "N": N,
                          "ms": round(ev_time(lambda: deinterleave(g, f)), 4)}), flush=True)
        print(json.dumps({"leg": "assemble_bands_device", "N": N,
                          "ms": round(ev_time(lambda: assemble_bands_device(g, f)), 4)}), flush=True)
    host = torch.empty((H, W, 3), dtype=torch.float32).pin_memory()
    print(json.dumps({"leg": "d2h_pinned_3MB", "ms": round(ev_time(lambda: host.copy_(tile, non_blocking=True)), 4)}),
          flush=True)
    dst = torch.empty_like(tile)
    print(json.dumps({"leg": "d2d_copy_3MB", "ms": round(ev_time(lambda: dst.copy_(tile)), 4)}), flush=True)
