"""Stamp a summarize_pmc.py result as profiles/traffic_<config>.json (dev tool):
the HBM bytes per launch bench.py reports as `roofline.traffic`, with the
kernel-source hash bench.py checks (a stale file is reported as stale, and
tests/test_profiles.py fails on it).  An optional second summary (the K5
closest walks) is recorded as `closest_hbm_bytes_per_launch`.
Usage: stamp_traffic.py pmc.json out.json median|mean "source text" [closest_pmc.json]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pathtracerpython_amd import build  # noqa: E402

src, dst, stat, text = sys.argv[1:5]
key = "hbm_bytes_per_launch_mean" if stat == "mean" else "hbm_bytes_per_launch"
d = json.load(open(src))
# the stamp is the id of the library that was measured (which _native.lib()
# only loads when it is the hash of the sources on disk)
sha = build.embedded_build_id(build.OUT)
assert sha == build.source_sha(), (sha, build.source_sha())
t = {"hbm_bytes_per_launch": d[key], "statistic": "mean" if stat == "mean" else "median",
     "source_sha": sha, "source": text, "dispatches": d.get("dispatches")}
if len(sys.argv) > 5:
    c = json.load(open(sys.argv[5]))
    t["closest_hbm_bytes_per_launch"] = c[key]
    t["closest_dispatches"] = c.get("dispatches")
json.dump(t, open(dst, "w"), indent=1)
print(json.dumps(t))
