"""Time K2 (512^2 x 64 spp x 4 b) with alternative builds of libpt_hip.so and
split factors (dev tool).  Usage: variant_sweep.py lib1.so [lib2.so ...]"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, numpy as np
sys.path.insert(0, %r)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer, to_list_order
scene_reader.VERBOSE = False
r = Renderer(scene_reader.Scene(os.path.join(%r, "scenes/cornell/cornellroom.sdl")))
p = r.params(512, 512, 64, 4, 9)
tile = torch.zeros((512, 512, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
ms = []
for i in range(6):
    r.render_device(p, tile.data_ptr(), s.cuda_stream); torch.cuda.synchronize(); ms.append(r.last_kernel_ms())
ref = r.render(64, 64, 2, 4, 9, out_f64=True, force_f64=True)
got = r.render(64, 64, 2, 4, 9, out_f64=True)
print("%%-40s split=%%s  kernel_ms min %%.3f med %%.3f  Mpath/s %%.1f  exact=%%s" %% (os.path.basename(os.environ["PT_HIP_LIB"]), os.environ.get("PT_SPLIT", "auto"), min(ms[1:]), sorted(ms[1:])[2], 512*512*64/min(ms[1:])/1e3, np.array_equal(ref, got)), flush=True)
''' % (ROOT, ROOT)
splits = os.environ.get("SPLITS", "auto").split(",")
for lib in sys.argv[1:]:
    for sp in splits:
        env = dict(os.environ, PT_HIP_LIB=os.path.abspath(lib), PT_DEV_OLD_LIB="1")
        if sp != "auto":
            env["PT_SPLIT"] = sp
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=300)
        if r.returncode:
            print("FAILED", lib, sp, r.returncode, flush=True)
            sys.exit(r.returncode)
