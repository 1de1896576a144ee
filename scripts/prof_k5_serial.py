"""Profiling driver (dev tool): the full K5 render (1024x1024, 256 spp, 4
bounces) as bench.py's k5 roofline times it — a PT_FLAG_KERNEL_TIMES launch,
whose two walks of a step run one after the other on one stream, so
`rocprofv3 --kernel-trace --stats` gives each walk kernel's own duration
(profiles/rNN_k5_kernel_stats_serial.csv).  Prints the HIP-event times the
launch reports next to them.
Usage: prof_k5_serial.py [renders]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
scene_reader.VERBOSE = False
torch.cuda.set_device(0)
r = Renderer(scene_reader.Scene(write_k5_scene(tempfile.mkdtemp(prefix="k5_"), n_tris=100_000, seed=0,
                                               size=1024)))
for i in range(n):
    _, kt = r.render_params(r.params(1024, 1024, 256, 4, 9, kernel_times=True), stats=True)
    print(json.dumps({k: v for k, v in kt.items() if k.endswith(("_ms", "_launches"))}), flush=True)
r.close()
