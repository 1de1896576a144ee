"""Time the device image finalisation (pt_image_u8_device) on a 4096^2
framebuffer, f32 and f64 (dev tool).  Prints GB/s against the algorithmic
bytes: two reads of the framebuffer (min/max pass, normalise pass) + the
uint8 write."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pathtracerpython_amd.render import image_u8_device
N = 4096
s = torch.cuda.current_stream()
for dt, f64 in ((torch.float32, False), (torch.float64, True)):
    fb = torch.rand((N, N, 3), dtype=dt, device="cuda")
    out = torch.empty((N, N, 3), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        image_u8_device(fb.data_ptr(), N, N, f64, out.data_ptr(), s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record(s)
    for _ in range(reps):
        image_u8_device(fb.data_ptr(), N, N, f64, out.data_ptr(), s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = 2 * fb.numel() * fb.element_size() + out.numel()
    print("%s %dx%d: %.3f ms  %.0f GB/s algorithmic (%.1f%% of 8 TB/s)" % (
        dt, N, N, ms, nbytes / ms / 1e6, nbytes / ms / 1e6 / 8000 * 100))
