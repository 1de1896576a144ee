"""Profiling driver: a few K5 launches (100k-triangle synthetic mesh, BVH
instantiation of k_render) for rocprofv3 counter passes (dev tool).
Usage: prof_k5.py [launches] [W] [spp]"""
import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
from pathtracerpython_amd.synth import write_k5_scene
scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
W = int(sys.argv[2]) if len(sys.argv) > 2 else 512
SPP = int(sys.argv[3]) if len(sys.argv) > 3 else 16
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=W)))
p = r.params(W, W, SPP, 4, 9)
out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
ms = []
for i in range(n):
    r.render_device(p, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ms.append(r.last_kernel_ms())
print("kernel ms", ms, "Mpath/s %.2f" % (W * W * SPP / min(ms) / 1e3))
import hashlib
print("fb sha", hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16])
if "--times" in sys.argv:   # each kernel's own time (the walks one after the other)
    from pathtracerpython_amd._abi import PT_FLAG_KERNEL_TIMES, with_flags
    _, kt = r.render_params(with_flags(p, PT_FLAG_KERNEL_TIMES), stats=True)
    print("own ms per render: shade %.1f shadow %.1f closest %.1f sort %.1f (launches %d / %d / %d / %d)" % (
        kt["shade_ms"], kt["shadow_ms"], kt["closest_ms"], kt["sort_ms"], kt["shade_launches"],
        kt["shadow_launches"], kt["closest_launches"], kt["sort_launches"]))
if "--counts" in sys.argv:   # the walks' work (PT_FLAG_WALK_COUNT launch)
    from pathtracerpython_amd._abi import PT_FLAG_WALK_COUNT, with_flags
    _, wc = r.render_params(with_flags(p, PT_FLAG_WALK_COUNT), stats=True)
    for k in ("shadow", "closest"):
        q = max(1, wc[k + "_queries"])
        print("%s walks: queries %d, node visits %d (%.2f per query), leaf units %d (%.2f per query)" % (
            k, wc[k + "_queries"], wc[k + "_node_visits"], wc[k + "_node_visits"] / q,
            wc[k + "_leaf_units"], wc[k + "_leaf_units"] / q))
