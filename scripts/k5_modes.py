"""K5 (100k-triangle synthetic mesh): time the wavefront and the single-kernel
renders of the same image and check they are bitwise equal (dev tool).
Usage: k5_modes.py [W] [spp] [bounces]"""
import os, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
from pathtracerpython_amd.synth import write_k5_scene

W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
SPP = int(sys.argv[2]) if len(sys.argv) > 2 else 64
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4
scene_reader.VERBOSE = False
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=W)))
s = torch.cuda.current_stream()
res = {}
for mega in (False, True):
    p = r.params(W, W, SPP, B, 9, megakernel=mega)
    out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
    ms = []
    for i in range(3):
        t0 = time.perf_counter()
        r.render_device(p, out.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        ms.append((r.last_kernel_ms(), (time.perf_counter() - t0) * 1e3))
    best = min(ms)
    res[mega] = out.cpu().numpy()
    print("%-12s K5 %dx%d %d spp %d b: device ms %.1f (wall %.1f)  %.2f Mpath/s" % (
        "single" if mega else "wavefront", W, W, SPP, B, best[0], best[1],
        W * W * SPP / best[0] / 1e3), flush=True)
print("bitwise equal:", np.array_equal(res[False], res[True]), flush=True)
