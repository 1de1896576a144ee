"""Experiment (round 4): what would shrinking the K5 walks'
working set under an XCD's 4 MiB L2 buy?  The K5 recipe (synth.py) at
25k / 50k / 100k / 200k triangles (BVH nodes + leaf records ~96 B per
triangle: 2.4 / 4.8 / 9.6 / 19.2 MB), 512^2 x 64 spp x 4 bounces, one
PT_FLAG_KERNEL_TIMES render (the walks serialised: own times) and one
PT_FLAG_WALK_COUNT render each.  Prints per size the walks' own ms, node
visits and leaf units, and the time per node visit (ns, whole chip) — if the
walk's cost per visit does not drop once the tree fits in L2, compacting the
records toward 4 MiB cannot pay more than that difference.
Run under rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum for the L2 hit rates.
Usage: exp_k5_working_set.py [sizes...]"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402
from pathtracerpython_amd.synth import write_k5_scene  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [25_000, 50_000, 100_000, 200_000]
scene_reader.VERBOSE = False
torch.cuda.set_device(0)
W, SPP = 512, 64
for n in sizes:
    r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(prefix="k5ws_"), n_tris=n, seed=0,
                                                   size=W)))
    r.render(W, W, SPP, 4, 9)   # warm-up (allocations)
    _, kt = r.render_params(r.params(W, W, SPP, 4, 9, kernel_times=True), stats=True)
    _, wc = r.render_params(r.params(W, W, SPP, 4, 9, walk_count=True), stats=True)
    rec = {"n_tris": n}
    for kind in ("shadow", "closest"):
        ms = kt[f"{kind}_ms"]
        v, u, q = wc[f"{kind}_node_visits"], wc[f"{kind}_leaf_units"], wc[f"{kind}_queries"]
        rec[kind] = {"ms": round(ms, 2), "queries": q, "visits_per_query": round(v / max(1, q), 2),
                     "units_per_query": round(u / max(1, q), 2),
                     "ns_per_visit": round(ms * 1e6 / max(1, v), 5),
                     "ns_per_visit_plus_unit": round(ms * 1e6 / max(1, v + u), 5)}
    rec["shade_ms"] = round(kt["shade_ms"], 2)
    print(json.dumps(rec), flush=True)
    r.close()
