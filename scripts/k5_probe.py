"""K5 (100k-triangle synthetic mesh) probe on one GPU (dev tool): writes the
scene, renders a small image with the hybrid and the forced-f64 kernels,
checks them bitwise and against the CPU oracle on a pixel subset, and
prints the kernel time.  Usage: k5_probe.py [W] [spp] [bounces] [n_tris]"""
import os, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
from pathtracerpython_amd.synth import write_k5_scene
from oracle import oracle

W = int(sys.argv[1]) if len(sys.argv) > 1 else 64
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4
n = int(sys.argv[4]) if len(sys.argv) > 4 else 100_000
scene_reader.VERBOSE = False
d = tempfile.mkdtemp()
t0 = time.time()
sc = scene_reader.Scene(write_k5_scene(d, n_tris=n, size=W))
r = Renderer(sc)
print("scene %d tris, ingest+upload %.2f s" % (r.packed.n_tri, time.time() - t0), flush=True)
fb = r.render(W, W, spp, B, 9, out_f64=True)
t = r.last_kernel_ms()
fb = r.render(W, W, spp, B, 9, out_f64=True)
print("hybrid kernel %.2f ms  (%.3f Mpath/s)" % (r.last_kernel_ms(), W * W * spp / r.last_kernel_ms() / 1e3), flush=True)
f64 = r.render(W, W, spp, B, 9, out_f64=True, force_f64=True)
print("forced-f64 kernel %.2f ms  bitwise equal: %s" % (r.last_kernel_ms(), np.array_equal(fb, f64)), flush=True)
rows = [0, W // 3, W - 1]
pix = np.array([ix * W + iy for iy in rows for ix in range(0, W, 4)], dtype=np.int64)
t0 = time.time()
cols, _ = oracle.render(r.packed, W, W, spp, B, 9, pixels=pix, threads=16)
got = np.array([fb[W - 1 - (k % W), k // W] for k in pix])
print("oracle %d pixels (%.1f s): max |diff| %.3g" % (len(pix), time.time() - t0, np.abs(got - cols).max()), flush=True)

if len(sys.argv) > 5:   # timing at a bigger size: k5_probe.py W spp B n TW TSPP
    TW, TS = int(sys.argv[5]), int(sys.argv[6])
    p = r.params(TW, TW, TS, B, 9)
    out = torch.zeros((TW, TW, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    r.render_device(p, out.data_ptr(), st)
    torch.cuda.synchronize()
    r.render_device(p, out.data_ptr(), st)
    torch.cuda.synchronize()
    ms = r.last_kernel_ms()
    print("K5 timing %dx%d %d spp %d b: %.1f ms  %.2f Mpath/s" % (TW, TW, TS, B, ms, TW * TW * TS / ms / 1e3), flush=True)
