"""Dev tool: K2 renders back to back on one stream vs alternating over two
streams (double-buffered frames), so that one launch's drain can overlap the
next launch's start.  Prints ms per render for each, median of `reps` runs of
`n` renders.  Usage: prof_overlap.py [n] [reps]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402

scene_reader.VERBOSE = False
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
torch.cuda.set_device(0)
W = H = 512
sc = scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl"))
rs = [Renderer(sc), Renderer(sc)]   # one handle per stream (a handle orders its launches)
p = rs[0].params(W, H, 64, 4, 9)
fbs = [torch.zeros((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run(k_streams):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for i in range(n):
        j = i % k_streams
        rs[j].render_device(p, fbs[j].data_ptr(), streams[j].cuda_stream)
    for s in streams:
        cur.wait_stream(s)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for k in (1, 2, 1, 2):   # warm-up pass included
    run(k)
res = {}
for k in (1, 2):
    res[k] = statistics.median(run(k) for _ in range(reps))
print(json.dumps({"ms_per_render_one_stream": round(res[1], 4), "ms_per_render_two_streams": round(res[2], 4),
                  "n": n, "reps": reps}), flush=True)
