"""Dev check for variant builds: the K5 scene (100k triangles) at 160^2 x 4
spp x 4 bounces through the wavefront kernels must equal the single kernel
bit for bit (prints OK / MISMATCH)."""
import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
from pathtracerpython_amd.synth import write_k5_scene
scene_reader.VERBOSE = False
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=160)))
wf = r.render(160, 160, 4, 4, 9, out_f64=True)
mk = r.render(160, 160, 4, 4, 9, out_f64=True, megakernel=True)
print("k5 parity", "OK" if np.array_equal(wf, mk) else "MISMATCH %g" % np.abs(wf - mk).max())
