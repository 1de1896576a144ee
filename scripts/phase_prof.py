"""Per-phase cycle shares of the K2 lane loop from an s_memtime-instrumented
build (scripts/prof_phase.so, dev tool): bounce sampling, shadow setup, the
fused unit loop, closest finish + bookkeeping."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PT_HIP_LIB"] = os.path.join(ROOT, "scripts", "prof_phase.so")
os.environ["PT_DEV_OLD_LIB"] = "1"
sys.path.insert(0, ROOT)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
p = r.params(512, 512, 64, 4, 9)
fb, st = r.render_params(p, stats=True)
fb, st = r.render_params(p, stats=True)
names = ("bounce sampling (RNG block 3, bounce())", "shadow setup (3 RNG blocks, light points)",
         "fused unit loop (3 shadow + closest, + light units)", "closest finish, colour, regeneration")
v = [st["closest_tests"], st["shadow_tests"], st["ray_bounces"], st["shading_points"]]
tot = sum(v)
for n, x in zip(names, v):
    print("%-55s %6.1f%%" % (n, 100.0 * x / tot))
print("kernel ms %.3f (instrumented)" % r.last_kernel_ms())
