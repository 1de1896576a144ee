"""Time the K5 wavefront render under different environment settings (dev
tool).  Usage: k5_env_sweep.py W SPP VAR v1 v2 ...   e.g. PT_WF_THR_SHADOW 8 16 24"""
import os, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pathtracerpython_amd.synth import write_k5_scene
W, SPP, VAR = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
sdl = write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=W)
CHILD = r'''
import os, sys
sys.path.insert(0, %r)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
r = Renderer(scene_reader.Scene(%r))
W, SPP = %d, %d
p = r.params(W, W, SPP, 4, 9)
out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
ms = []
for i in range(3):
    r.render_device(p, out.data_ptr(), s); torch.cuda.synchronize(); ms.append(r.last_kernel_ms())
print("%%s=%%-6s K5 %%dx%%d %%d spp: ms %%.1f  %%.2f Mpath/s" %% (%r, os.environ.get(%r), W, W, SPP, min(ms), W * W * SPP / min(ms) / 1e3), flush=True)
''' % (ROOT, sdl, W, SPP, VAR, VAR)
for v in sys.argv[4:]:
    r = subprocess.run([sys.executable, "-c", CHILD], env=dict(os.environ, **{VAR: v}), timeout=600)
    if r.returncode:
        print("FAILED", v, r.returncode, flush=True)
        sys.exit(r.returncode)
