"""Dev experiment: node visits per query of 4- and 8-wide BVH walks on the K5
scene (wide_bvh_count.cpp, host only).
Usage: wide_bvh_count.py [size] [spp] [n_tris] [order: 0 nearest-first, 1 nearest then node order]"""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd._abi import make_params  # noqa: E402
from pathtracerpython_amd.pack import pack_scene  # noqa: E402
from pathtracerpython_amd.synth import write_k5_scene  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 32
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ntri = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000
order = int(sys.argv[4]) if len(sys.argv) > 4 else 0   # 1: nearest child first, the rest in node order
so = os.path.join(tempfile.gettempdir(), "wide_bvh_count.so")
# WX_FLAGS: extra compiler flags (builder variants, e.g. -DPT_BVH_BINS=64)
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-w", "-o", so,
                os.path.join(HERE, "wide_bvh_count.cpp")] + os.environ.get("WX_FLAGS", "").split(), check=True)
lib = C.CDLL(so)
scene_reader.VERBOSE = False
with tempfile.TemporaryDirectory() as d:
    pk = pack_scene(scene_reader.Scene(write_k5_scene(d, n_tris=ntri, seed=0, size=size)))
    p = make_params(size, size, spp, 4, 9, 0)
    out = (C.c_int64 * 36)()
    rc = lib.wx_count(C.byref(pk.desc), C.byref(p), out, C.c_int(order))
    assert rc == 0, rc
o = list(out)
names = ["queries", "visits", "boxes", "leaves", "units", "mismatches", "maxstack"]
res = {"size": size, "spp": spp, "n_tris": ntri, "order": order}
for w, N in enumerate((4, 8)):
    for j, kind in enumerate(("shadow", "closest")):
        v = dict(zip(names, o[w * 14 + j * 7: w * 14 + j * 7 + 7]))
        v["visits_per_query"] = round(v["visits"] / max(v["queries"], 1), 2)
        v["boxes_per_query"] = round(v["boxes"] / max(v["queries"], 1), 2)
        v["units_per_query"] = round(v["units"] / max(v["queries"], 1), 2)
        res[f"{kind}_{N}wide_exact_boxes"] = v
ws = o[28:36]
res["shipped_qnode"] = {"shadow_visits_per_query": round(ws[1] / max(ws[0], 1), 2),
                        "shadow_units_per_query": round(ws[3] / max(ws[0], 1), 2),
                        "closest_visits_per_query": round(ws[5] / max(ws[4], 1), 2),
                        "closest_units_per_query": round(ws[7] / max(ws[4], 1), 2)}
print(json.dumps(res, indent=1))
