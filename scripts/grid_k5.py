"""Dev tool: the K5 shadow walks through the grid vs the BVH.
1. parity: K5 (100k triangles) at 160^2 x 4 spp x 4 bounces, grid wavefront ==
   tree wavefront == single kernel, bit for bit;
2. timing: the bench render (1024^2 x 256 spp unless argv gives W SPP) with
   per-kernel HIP-event times, grid and tree, and the walks' work counts.
Prints JSON lines."""
import json, os, sys, tempfile, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from pathtracerpython_amd import scene_reader
from pathtracerpython_amd.render import Renderer
from pathtracerpython_amd.synth import write_k5_scene
scene_reader.VERBOSE = False
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
SPP = int(sys.argv[2]) if len(sys.argv) > 2 else 256
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(), n_tris=100_000, seed=0, size=160)))
g = r.render(160, 160, 4, 4, 9, out_f64=True)
t = r.render_params(r.params(160, 160, 4, 4, 9, out_f64=True, tree_walk=True))
m = r.render(160, 160, 4, 4, 9, out_f64=True, megakernel=True)
print(json.dumps({"parity_grid_eq_tree": bool(np.array_equal(g, t)), "parity_grid_eq_single": bool(np.array_equal(g, m)),
                  "max_diff": float(np.abs(g - m).max())}), flush=True)
if not np.array_equal(g, m):
    sys.exit(1)
out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
for tree in (False, True):
    p = r.params(W, W, SPP, 4, 9, tree_walk=tree)
    r.render_device(p, out.data_ptr(), s.cuda_stream)   # warm-up
    torch.cuda.synchronize()
    ms = []
    for _ in range(2):
        r.render_device(p, out.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        ms.append(r.last_kernel_ms())
    _, st = r.render_params(r.params(W, W, SPP, 4, 9, tree_walk=tree, kernel_times=True), stats=True)
    _, wc = r.render_params(r.params(W, W, SPP, 4, 9, tree_walk=tree, walk_count=True), stats=True)
    keys = ("shade_ms", "shadow_ms", "closest_ms", "shadow_queries", "shadow_node_visits", "shadow_leaf_units")
    d = {k: (st.get(k) if k.endswith("_ms") else wc.get(k)) for k in keys}
    print(json.dumps({"walk": "tree" if tree else "grid", "render_ms": ms, "Mpath_s": round(W * W * SPP / min(ms) / 1e3, 2),
                      **d}), flush=True)
