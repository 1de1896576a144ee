"""Dev experiment: one-ray shadow walk node visits, top-down (shipped order)
vs bottom-up from the origin triangle's leaf (bottomup_count.cpp, host only).
Usage: bottomup_count.py [size] [spp] [n_tris]"""
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
so = os.path.join(tempfile.gettempdir(), "bottomup_count.so")
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-w", "-o", so,
                os.path.join(HERE, "bottomup_count.cpp")] + os.environ.get("WX_FLAGS", "").split(), check=True)
lib = C.CDLL(so)
scene_reader.VERBOSE = False
with tempfile.TemporaryDirectory() as d:
    pk = pack_scene(scene_reader.Scene(write_k5_scene(d, n_tris=ntri, seed=0, size=size)))
    p = make_params(size, size, spp, 4, 9, 0)
    out = (C.c_int64 * 12)()
    rc = lib.bu_count(C.byref(pk.desc), C.byref(p), out)
    assert rc == 0, rc
o = list(out)
res = {"size": size, "spp": spp, "n_tris": ntri}
for j, kind in enumerate(("top_down", "bottom_up")):
    rays, visits, units, mism, occ, occv = o[6 * j: 6 * j + 6]
    res[kind] = {"rays": rays, "visits_per_ray": round(visits / rays, 2), "units_per_ray": round(units / rays, 2),
                 "mismatches": mism, "occluded": occ, "visits_per_occluded_ray": round(occv / max(occ, 1), 2),
                 "visits_per_open_ray": round((visits - occv) / max(rays - occ, 1), 2)}
print(json.dumps(res, indent=1))
