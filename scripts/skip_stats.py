"""Dev tool: how often the K2 render's uniform-unit pass skips work at wave
level, from a library built with -DPT_SKIPSTAT (pt_path.h PT_SKIP_EV; counts
once per wave and event, so the instrumented kernel is slow — use the ratios).
Usage: PT_HIP_LIB=.../skipstat.so python3 skip_stats.py [launches]
Prints one JSON line."""
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
lib = _native.lib()
fn = lib.pt_debug_skip_stats
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
v = (C.c_ulonglong * 16)()
p = r.params(512, 512, 64, 4, 9)
tile = torch.zeros((512, 512, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
fn(v, 1)
for _ in range(n):
    r.render_device(p, tile.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
fn(v, 1)
names = ["unit_iters", "shadow_part_old", "shadow_part_lcull", "ray0_plane", "ray1_plane", "ray2_plane",
         "ray0_nm_skip", "ray1_nm_skip", "ray2_nm_skip", "closest_part", "closest_skip",
         "lanes_unit_iters", "lanes_off_lcull", "lanes_ray0_out", "lanes_ray1_out", "lanes_ray2_out"]
d = {k: v[i] / n for i, k in enumerate(names)}
out = {"per_launch_wave_events": d,
       "shadow_part_kept_by_lcull": round(d["shadow_part_lcull"] / max(1, d["shadow_part_old"]), 4),
       "ray_nm_skip_frac": [round(d["ray%d_nm_skip" % k] / max(1, d["ray%d_plane" % k]), 4) for k in range(3)],
       "closest_skip_frac": round(d["closest_skip"] / max(1, d["closest_part"]), 4),
       # lane level: the share of (lane, unit) pairs a lane alone could skip
       "lane_off_lcull_frac": round(d["lanes_off_lcull"] / max(1, d["lanes_unit_iters"]), 4),
       # (lane, ray, unit) tests certainly out of range or already occluded (rays 0, 1),
       # over the lanes of the waves that ran the ray's plane part
       "lane_ray_out_per_unit_iter_lane": [round(d["lanes_ray%d_out" % k] / max(1, d["lanes_unit_iters"]), 4)
                                           for k in range(3)]}
print(json.dumps(out), flush=True)
