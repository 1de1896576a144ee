"""Per-wave start/end clocks of one K2 launch (dev tool; needs a library built
with the wave-time instrumentation, passed as PT_HIP_LIB with).
Prints the occupancy profile: how long the launch runs below full occupancy
at its start and end.  Usage: wave_times.py [W] [spp] [waves in the launch]."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pathtracerpython_amd import scene_reader, _native
from pathtracerpython_amd.render import Renderer
scene_reader.VERBOSE = False
W, SPP = int(sys.argv[1]) if len(sys.argv) > 1 else 512, int(sys.argv[2]) if len(sys.argv) > 2 else 64
r = Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl")))
p = r.params(W, W, SPP, 4, 9)
out = torch.zeros((W, W, 3), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    r.render_device(p, out.data_ptr(), s)
torch.cuda.synchronize()
lib = _native.lib()
nw = min(int(sys.argv[3]) if len(sys.argv) > 3 else W * W * 8 // 64, 1 << 20)
buf = np.zeros(2 * nw, dtype=np.uint64)
assert lib.pt_dev_wave_times(buf.ctypes.data_as(C.c_void_p), C.c_size_t(2 * nw)) == 0
st, en = buf[0::2].astype(np.int64), buf[1::2].astype(np.int64)
t0 = st.min()
st, en = (st - t0) / 100.0, (en - t0) / 100.0   # 100 MHz -> microseconds
span = en.max()
dur = en - st
print(f"waves {nw}  span {span:.0f} us  kernel_ms {r.last_kernel_ms():.3f}  wave dur mean {dur.mean():.0f} "
      f"p50 {np.median(dur):.0f} p99 {np.percentile(dur, 99):.0f} max {dur.max():.0f} us")
grid = np.linspace(0, span, 201)
act = np.array([((st <= t) & (en > t)).sum() for t in grid])
full = np.percentile(act, 50)
print("active waves (every 5% of the span):", act[::10].tolist())
below = grid[act < 0.9 * full]
tail = span - below[below > span / 2].min() if (below > span / 2).any() else 0.0
head = below[below < span / 2].max() if (below < span / 2).any() else 0.0
print(f"median active {full:.0f}; below 90%: first {head:.0f} us, last {tail:.0f} us; "
      f"idle wave-time fraction {1 - act.mean() / full:.3f}")
