"""Dev tool: what one GPU's share of an N-GPU strong-scaling K2 step costs
(DESIGN.md §8).  For the built library (or PT_HIP_LIB): the kernel time of one
rank's interleaved row band (row_step N, phases 0 and N-1) at N = 1/2/4/8,
median of the last half of `launches`; then the fixed per-step legs on this
GPU: the device assembly of the gathered tiles (bench.py's step: the native
pt_assemble_bands_device, and torch's strided copy for comparison) and,
for reference, the PCIe D2H of the frame (outside bench.py's timed step).
Prints one JSON object per line.
Usage: prof_scaling.py [launches] [N...]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.distributed import deinterleave  # noqa: E402
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
for N in Ns:
    for phase in sorted({0, N - 1}):
        p = r.params(W, H, 64, 4, 9, row_begin=0, row_end=H, row_step=N, row_phase=phase)
        ms = []
        for i in range(n):
            r.render_device(p, tile.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            ms.append(r.last_kernel_ms())
        med = statistics.median(ms[n // 2:])
        print(json.dumps({"lib": lib, "N": N, "phase": phase, "band_kernel_ms": round(med, 4),
                          "x_N": round(med * N, 4), "min": round(min(ms), 4)}), flush=True)


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
