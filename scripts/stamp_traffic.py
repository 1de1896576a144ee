"""Stamp a summarize_pmc.py result as profiles/traffic_<config>.json (dev tool):
the HBM bytes per launch bench.py reports as `roofline.traffic`, with the
kernel-source hash bench.py checks (a stale file is reported as stale).
Usage: stamp_traffic.py pmc.json out.json median|mean "source text"
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

src, dst, stat, text = sys.argv[1:5]
d = json.load(open(src))
key = "hbm_bytes_per_launch_mean" if stat == "mean" else "hbm_bytes_per_launch"
t = {"hbm_bytes_per_launch": d[key], "source_sha": bench.source_sha(), "source": text}
json.dump(t, open(dst, "w"), indent=1)
print(json.dumps(t))
