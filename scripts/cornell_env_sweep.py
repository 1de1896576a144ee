"""Time a Cornell box render under different environment settings (dev tool).
Usage: cornell_env_sweep.py W SPP BOUNCES RR VAR v1 v2 ...   e.g. 1024 1024 8 1 PT_SPLIT 2 4 8"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, SPP, B, RR, VAR = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
CHILD = r'''
import os, sys
sys.path.insert(0, %r)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
r = Renderer(scene_reader.Scene(os.path.join(%r, "scenes", "cornell", "cornellroom.sdl")))
W, SPP, B, RR = %d, %d, %d, %d
p = r.params(W, W, SPP, B, 9, rr=bool(RR))
out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
ms = []
for i in range(3):
    r.render_device(p, out.data_ptr(), s); torch.cuda.synchronize(); ms.append(r.last_kernel_ms())
print("%%s=%%-6s Cornell %%dx%%d %%d spp %%d b rr=%%d: ms %%.2f  %%.1f Mpath/s" %% (%r, os.environ.get(%r), W, W, SPP, B, RR, min(ms), W * W * SPP / min(ms) / 1e3), flush=True)
''' % (ROOT, ROOT, W, SPP, B, RR, VAR, VAR)
for v in sys.argv[6:]:
    r = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, **{VAR: v}), timeout=600)
    if r.returncode:
        print("FAILED", v, r.returncode, flush=True)
        sys.exit(r.returncode)
