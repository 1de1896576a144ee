"""Profiling driver: a few K2 launches (512x512, 64 spp, 4 bounces) of the
render kernel, for rocprofv3 counter passes (dev tool)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
f64 = "--f64" in sys.argv
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
lanes = int(sys.argv[sys.argv.index("--lanes") + 1]) if "--lanes" in sys.argv else 0
p = r.params(512, 512, 64, 4, 9, force_f64=f64, lanes_per_pixel=lanes)
tile = torch.zeros((512, 512, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
ms = []
for i in range(n):
    r.render_device(p, tile.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ms.append(r.last_kernel_ms())
import statistics
med = statistics.median(ms[len(ms) // 2:])
print("kernel ms", [round(x, 4) for x in ms], "median(last half) %.4f" % med,
      "Mpath/s %.1f" % (512 * 512 * 64 / med / 1e3))
import hashlib
print("fb sha", hashlib.sha256(tile.cpu().numpy().tobytes()).hexdigest()[:16])
