"""Time the K5 wavefront render with several library builds (dev tool).
Usage: k5_lib_sweep.py W SPP lib1.so [lib2.so ...]"""
import os, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pathtracerpython_amd.synth import write_k5_scene
W, SPP = int(sys.argv[1]), int(sys.argv[2])
sdl = write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=W)
CHILD = r'''
import os, sys
sys.path.insert(0, %r)
import numpy as np, torch
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
a = out.cpu().numpy().copy()
p2 = r.params(64, 64, 2, 4, 9); ref = r.render(64, 64, 2, 4, 9, out_f64=True, megakernel=True)
got = r.render(64, 64, 2, 4, 9, out_f64=True)
print("%%-16s K5 %%dx%%d %%d spp: ms %%.1f  %%.2f Mpath/s  wf==single(64^2): %%s" %% (os.path.basename(os.environ["PT_HIP_LIB"]), W, W, SPP, min(ms), W * W * SPP / min(ms) / 1e3, np.array_equal(ref, got)), flush=True)
''' % (ROOT, sdl, W, SPP)
for lib in sys.argv[3:]:
    env = dict(os.environ, PT_HIP_LIB=os.path.abspath(lib), PT_DEV_OLD_LIB="1")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=600)
    if r.returncode:
        print("FAILED", lib, r.returncode, flush=True)
        sys.exit(r.returncode)
