"""Dev tool: K2 kernel time of the full frame and of one interleaved row band
(row_step N, phase 0: one rank's share of an N-GPU strong-scaling render).
Usage: prof_band.py [launches] [N...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import statistics
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
Ns = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
tile = torch.zeros((512, 512, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
for N in Ns:
    p = r.params(512, 512, 64, 4, 9, row_begin=0, row_end=512, row_step=N, row_phase=0)
    ms = []
    for i in range(n):
        r.render_device(p, tile.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        ms.append(r.last_kernel_ms())
    med = statistics.median(ms[n // 2:])
    print("N=%d band kernel ms median %.3f (x N = %.3f)" % (N, med, med * N), flush=True)
