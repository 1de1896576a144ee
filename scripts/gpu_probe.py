"""Quick GPU probe: golden parity, hybrid == f64, first timing (dev tool)."""
import glob, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pathtracerpython_amd.scene_reader as sr
sr.VERBOSE = False
from pathtracerpython_amd.render import Renderer, to_list_order

sc = sr.Scene(os.path.join(ROOT, 'scenes/cornell/cornellroom.sdl'))
r = Renderer(sc)
for f in sorted(glob.glob(os.path.join(ROOT, 'tests/golden/render_*.npz'))):
    g = np.load(f)
    W, H, spp, B, seed = [int(g[k]) for k in ('width', 'height', 'spp', 'bounces', 'seed')]
    fb, st = r.render(W, H, spp, B, seed, stats=True)
    err = np.abs(to_list_order(fb).astype(np.float64) - g['colors']).max()
    print(os.path.basename(f), 'linf', err, st, flush=True)
for (W, H, spp, B) in [(64, 64, 4, 4), (128, 128, 2, 6)]:
    a = r.render(W, H, spp, B, 9)
    b = r.render(W, H, spp, B, 9, force_f64=True)
    print('hybrid==f64', W, H, spp, B, np.array_equal(a, b), np.abs(a - b).max(), flush=True)
for f64 in (False, True):
    p = r.params(512, 512, 64, 4, 9, force_f64=f64)
    r.render_params(p)
    t = time.time(); fb = r.render_params(p); dt = time.time() - t
    ms = r.last_kernel_ms()
    print('K2 f64' if f64 else 'K2 hybrid', 'wall %.2f ms kernel %.2f ms -> %.3f Gpaths/s' % (dt * 1e3, ms, 512 * 512 * 64 / ms / 1e6), flush=True)
p = r.params(512, 512, 64, 4, 9, count=True)
fb, st = r.render_params(p, stats=True)
print('K2 stats', st, 'tests/path', (st['closest_tests'] + st['shadow_tests']) / (512 * 512 * 64))
