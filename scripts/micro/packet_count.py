"""Dev experiment: wave-coherent (packet) shadow walks over the sorted shadow
list vs the shipped one-ray walks, on the K5 scene (packet_count.cpp, host
only).
Usage: packet_count.py [size] [spp] [split] [steps] [order: 0 nearest lane, 1 first lane] [n_tris]"""
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
from pathtracerpython_amd.pack import pack_scene  # noqa: E402
from pathtracerpython_amd.synth import write_k5_scene  # noqa: E402

a = [int(x) for x in sys.argv[1:]]
size, spp, split, steps, order, ntri = (a + [64, 64, 16, 4, 0, 100_000][len(a):])[:6]
so = os.path.join(tempfile.gettempdir(), "packet_count.so")
subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-w", "-o", so,
                os.path.join(HERE, "packet_count.cpp")], check=True)
lib = C.CDLL(so)
scene_reader.VERBOSE = False
with tempfile.TemporaryDirectory() as d:
    pk = pack_scene(scene_reader.Scene(write_k5_scene(d, n_tris=ntri, seed=0, size=size)))
    out = (C.c_int64 * 10)()
    rc = lib.pk_count(C.byref(pk.desc), size, spp, split, 4, steps, order, 64, out)
    assert rc == 0, rc
names = ["rays", "lane_visits", "lane_units", "waves", "wave_visits", "wave_units", "active_at_visit",
         "active_at_unit", "mismatches", "max_stack"]
o = dict(zip(names, list(out)))
res = {"size": size, "spp": spp, "split": split, "steps": steps, "order": order, "n_tris": ntri, **o}
res["lane_visits_per_ray"] = round(o["lane_visits"] / max(1, o["rays"]), 2)
res["lane_units_per_ray"] = round(o["lane_units"] / max(1, o["rays"]), 2)
res["wave_visits_per_wave"] = round(o["wave_visits"] / max(1, o["waves"]), 2)
res["wave_units_per_wave"] = round(o["wave_units"] / max(1, o["waves"]), 2)
res["lanes_active_per_visit"] = round(o["active_at_visit"] / max(1, o["wave_visits"]), 2)
res["lanes_active_per_unit"] = round(o["active_at_unit"] / max(1, o["wave_units"]), 2)
# node visits a wave issues: packet = its union; one-ray walks = lane visits over
# the lanes a visit keeps busy (measured VALU lane utilisation of k_wf_shadow: 0.749)
res["one_ray_wave_visits_per_wave"] = round(o["lane_visits"] / 64 / 0.749 / max(1, o["waves"]) * 1.0, 2)
print(json.dumps(res, indent=1))
