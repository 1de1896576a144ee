"""Dev tool: where a K2 render's wave time goes, from a library built with
-DPT_PHASE_CLOCKS (pt_path.h phase clocks; instrumented, so ~10% slower than
the shipped kernel — use the fractions, not the absolute times).
Usage: PT_HIP_LIB=.../phase.so python3 phase_clocks.py [launches] [row_step]
Prints one JSON line: wave-cycles per phase summed over waves, and fractions."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from pathtracerpython_amd import _native, scene_reader  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402

scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
lib = _native.lib()
fn = lib.pt_debug_phase_clocks
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
clk = (C.c_ulonglong * 8)()
p = r.params(512, 512, 64, 4, 9, row_step=step, row_phase=0)
tile = torch.zeros((r.band_rows(p), 512, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
r.render_device(p, tile.data_ptr(), s.cuda_stream)   # warm-up
torch.cuda.synchronize()
fn(clk, 1)
ms = []
for _ in range(n):
    r.render_device(p, tile.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ms.append(r.last_kernel_ms())
fn(clk, 1)
names = ["setup_rng_lights_bounce", "uniform_unit_pass", "bvh_and_light_units", "colour_next_hit_regen",
         "iterations", "primary_ray", "lane_total", "lane_iterations"]
v = {k: clk[i] / n for i, k in enumerate(names)}
names = names[:7]
loop = sum(v[k] for k in names[:4])
out = {"row_step": step, "kernel_ms": ms, "per_launch": v,
       "fraction_of_lane_total": {k: round(v[k] / v["lane_total"], 4) for k in names[:4] + ["primary_ray"]},
       "fraction_of_bounce_loop": {k: round(v[k] / loop, 4) for k in names[:4]},
       # lanes active in the wave's bounce-loop iterations (the rest: lanes
       # out of samples, waiting for the wave's longest lane)
       "tail_lane_utilisation": round(v["lane_iterations"] / (64 * v["iterations"]), 4)}
print(json.dumps(out), flush=True)
