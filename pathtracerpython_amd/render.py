"""Host API of the MI355X path tracer: `render(scene, width, height, spp) ->
framebuffer`, plus batched drop-ins for the reference's two Pool callables.

The reference's render is the body of main() (main.py:165-293): for `-r` spp
and `-b` bounces it traces every pixel of the SDL `size` and averages the
samples (main.py:274-280).  Here that whole loop is one call into the HIP
library (libpt_hip.so, include/pt_capi.h).  The RNG is the keyed Philox
stream documented in tests/golden/philox_ref.py; the key defaults to the SDL
`seed` (which the reference parses, scene_reader.py:169-170, but ignores).

Framebuffers are float32, image orientation: fb[H-1-iy, ix] is the averaged
radiance of the reference's pixel k = ix*H + iy (utils.py:64-69), before
make_image's min-max normalisation.
"""
import ctypes as C
import numbers

import numpy as np

from . import _native
from ._abi import (PT_FLAG_COUNT, PT_FLAG_FORCE_F64, PT_FLAG_KERNEL_TIMES, PT_FLAG_MEGAKERNEL,
                   PT_FLAG_OUT_F64, PT_FLAG_RR, PT_FLAG_WALK_COUNT, PtStats, band_rows, make_params)
from .pack import pack_scene

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class Renderer:
    """A scene uploaded to a HIP device (one `pt_scene` handle): the current
    device, or `device`."""

    def __init__(self, scene, device=None, packed=None):
        self.scene = scene
        self.packed = packed if packed is not None else pack_scene(scene)
        self._lib = _native.lib()
        h = C.c_void_p()
        if device is None:
            _native.check(self._lib.pt_scene_create(C.byref(self.packed.desc), C.byref(h)),
                          "pt_scene_create")
        else:
            _native.check(self._lib.pt_scene_create_on(C.byref(self.packed.desc), int(device),
                                                       C.byref(h)), "pt_scene_create_on")
        self._h = h
        self.device = device

    # ------------------------------------------------------------ render --
    def params(self, width=None, height=None, spp=1, bounces=1, seed=None, rr=False,
               rr_depth=3, force_f64=False, count=False, out_f64=False, row_begin=0,
               row_end=None, row_step=1, row_phase=0, sample_begin=0, megakernel=False,
               walk_count=False, kernel_times=False, out_row_stride=0, lanes_per_pixel=0):
        """megakernel=True: scenes with a BVH render with the single kernel
        instead of the wavefront kernels (the same framebuffer, bit for bit).
        walk_count / kernel_times (wavefront renders): the walks' work counts /
        per-kernel HIP-event times in the stats.  out_row_stride: elements
        between output rows (0: packed).  lanes_per_pixel: 0 lets the
        library choose per launch; a fixed power of two makes any band split
        bit-identical (include/pt_capi.h)."""
        width = int(self.scene.width if width is None else width)
        height = int(self.scene.height if height is None else height)
        seed = self.scene.seed if seed is None else seed
        seed = 0 if seed is None else int(seed)
        flags = (PT_FLAG_RR if rr else 0) | (PT_FLAG_FORCE_F64 if force_f64 else 0) | \
            (PT_FLAG_COUNT if count else 0) | (PT_FLAG_OUT_F64 if out_f64 else 0) | \
            (PT_FLAG_MEGAKERNEL if megakernel else 0) | \
            (PT_FLAG_WALK_COUNT if walk_count else 0) | (PT_FLAG_KERNEL_TIMES if kernel_times else 0)
        return make_params(width, height, spp, bounces, seed, flags, rr_depth, row_begin,
                           row_end, row_step, row_phase, sample_begin, out_row_stride,
                           lanes_per_pixel)

    def band_rows(self, p):
        n = C.c_int32(0)
        _native.check(self._lib.pt_band_rows(C.byref(p), C.byref(n)), "pt_band_rows")
        return n.value

    def render_params(self, p, stats=False):
        rows = self.band_rows(p)
        dt = np.float64 if p.flags & PT_FLAG_OUT_F64 else np.float32
        if p.out_row_stride:
            raise ValueError("render_params returns a packed band: use out_row_stride 0")
        out = np.zeros((rows, p.width, 3), dtype=dt)
        st = PtStats()
        _native.check(self._lib.pt_render(self._h, C.byref(p), C.c_void_p(out.ctypes.data),
                                          C.byref(st)), "pt_render")
        wide = bool(p.flags & (PT_FLAG_WALK_COUNT | PT_FLAG_KERNEL_TIMES))
        return (out, st.as_dict(all_fields=wide)) if stats else out

    def render(self, width=None, height=None, spp=1, bounces=1, seed=None, rr=False,
               rr_depth=3, force_f64=False, stats=False, out_f64=False, megakernel=False,
               **band):
        """Framebuffer (rows, W, 3), float32 (float64 with out_f64); rows = H
        for a full render.  stats=True also returns the work counters."""
        p = self.params(width, height, spp, bounces, seed, rr, rr_depth, force_f64,
                        count=stats, out_f64=out_f64, megakernel=megakernel, **band)
        return self.render_params(p, stats=stats)

    def render_device(self, p, out_ptr, stream=None):
        """Asynchronous render into a device buffer (e.g. a torch tensor's
        data_ptr()) on a HIP stream handle (int) — used by the multi-GPU path."""
        _native.check(self._lib.pt_render_device(self._h, C.byref(p), C.c_void_p(out_ptr),
                                                 C.c_void_p(stream or 0), None),
                      "pt_render_device")

    def render_image(self, width=None, height=None, spp=1, bounces=1, seed=None, rr=False,
                     rr_depth=3, return_fb=False):
        """make_image's uint8 array (H, W, 3) of a full render, finalised on
        the device (pt_image_u8_device) from the float64 framebuffer; with
        return_fb also that framebuffer.  Square images are exactly what
        make_image (utils.py:150-161) returns for the same colours."""
        import torch
        p = self.params(width, height, spp, bounces, seed, rr, rr_depth, out_f64=True)
        W, H = p.width, p.height
        fb = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
        img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        self.render_device(p, fb.data_ptr(), s)
        image_u8_device(fb.data_ptr(), W, H, True, img.data_ptr(), s)
        img = img.cpu().numpy()
        return (img, fb.cpu().numpy()) if return_fb else img

    def last_kernel_ms(self):
        ms = C.c_float(0)
        _native.check(self._lib.pt_last_kernel_ms(self._h, C.byref(ms)), "pt_last_kernel_ms")
        return ms.value

    # ------------------------------------------- batched Pool callables --
    def intersect_objects(self, rays):
        """Batched intersect_objects (main.py:83-122).  rays: (n, 6) origin,
        direction.  Returns (tri (n,) int32, -1 = None; P (n, 3) f64).  The
        reference's isItLight is tri >= packed.n_obj_tri."""
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        n = rays.shape[0]
        tri = np.zeros(n, dtype=np.int32)
        P = np.zeros((n, 3), dtype=np.float64)
        _native.check(self._lib.pt_intersect_objects(self._h, rays.ctypes.data_as(_dp), n,
                                                     tri.ctypes.data_as(_ip),
                                                     P.ctypes.data_as(_dp)),
                      "pt_intersect_objects")
        return tri, P

    def compute_color(self, obj, point, normal, u):
        """Batched compute_color (main.py:142-145) with the 12 light-sampling
        uniforms of each point given explicitly (slots 0..11)."""
        obj = np.ascontiguousarray(obj, dtype=np.int32).reshape(-1)
        point = np.ascontiguousarray(point, dtype=np.float64).reshape(-1, 3)
        normal = np.ascontiguousarray(normal, dtype=np.float64).reshape(-1, 3)
        u = np.ascontiguousarray(u, dtype=np.float64).reshape(-1, 12)
        n = obj.shape[0]
        if not (point.shape[0] == normal.shape[0] == u.shape[0] == n):
            raise ValueError("obj/point/normal/u must have the same length")
        out = np.zeros((n, 3), dtype=np.float64)
        _native.check(self._lib.pt_compute_color(self._h, obj.ctypes.data_as(_ip),
                                                 point.ctypes.data_as(_dp),
                                                 normal.ctypes.data_as(_dp),
                                                 u.ctypes.data_as(_dp), n,
                                                 out.ctypes.data_as(_dp)),
                      "pt_compute_color")
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pt_scene_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render(scene, width=None, height=None, spp=1, bounces=1, seed=None, rr=False, rr_depth=3,
           devices=1):
    """main.py's render as a function: framebuffer (H, W, 3) float32.
    devices: GPUs of this process — a count (devices 0..n-1) or a list of
    device ids; more than one renders interleaved row bands concurrently
    (MultiRenderer, pt_render_multi)."""
    count = isinstance(devices, numbers.Integral)
    ids = list(range(int(devices))) if count else [int(d) for d in devices]
    if not ids:
        raise ValueError("devices: need at least one")
    if len(ids) == 1 and count:
        with Renderer(scene) as r:
            return r.render(width, height, spp, bounces, seed, rr, rr_depth)
    with MultiRenderer(scene, ids) as m:
        return m.render(width, height, spp, bounces, seed, rr, rr_depth)


class MultiRenderer:
    """One scene on several GPUs of this process (pt_render_multi): the rows
    are dealt out interleaved, every device renders its band concurrently and
    each band is copied straight into its rows of the host framebuffer.
    Bit-identical to Renderer.render on one device when both are given the
    same lanes_per_pixel; with the default 0 each band's launch picks its own
    lanes per pixel and the values agree to ~1e-15 relative (the sum order
    of a pixel's samples follows its lane count).  (The multi-process path is
    distributed.py.)"""

    def __init__(self, scene, devices):
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ValueError("need at least one device")
        first = Renderer(scene, device=self.devices[0])
        self.renderers = [first] + [Renderer(scene, device=d, packed=first.packed)
                                    for d in self.devices[1:]]
        self.packed = first.packed

    def render(self, width=None, height=None, spp=1, bounces=1, seed=None, rr=False,
               rr_depth=3, stats=False, out_f64=False, row_begin=0, row_end=None,
               lanes_per_pixel=0):
        r0 = self.renderers[0]
        p = r0.params(width, height, spp, bounces, seed, rr, rr_depth, count=stats,
                      out_f64=out_f64, row_begin=row_begin, row_end=row_end,
                      lanes_per_pixel=lanes_per_pixel)
        rows = r0.band_rows(p)
        out = np.zeros((rows, p.width, 3), dtype=np.float64 if out_f64 else np.float32)
        hs = (C.c_void_p * len(self.renderers))(*[r._h.value for r in self.renderers])
        st = PtStats()
        _native.check(r0._lib.pt_render_multi(hs, len(self.renderers), C.byref(p),
                                              C.c_void_p(out.ctypes.data), C.byref(st)),
                      "pt_render_multi")
        return (out, st.as_dict()) if stats else out

    def close(self):
        for r in self.renderers:
            r.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def image_u8_device(fb_ptr, width, height, f64, out_ptr, stream=None):
    """Device image finalisation (make_image, utils.py:150-161) of a full
    framebuffer at fb_ptr (f32, or f64) into height*width*3 uint8 at out_ptr,
    asynchronous on a HIP stream handle."""
    lib = _native.lib()
    _native.check(lib.pt_image_u8_device(C.c_void_p(fb_ptr), int(width), int(height),
                                         PT_FLAG_OUT_F64 if f64 else 0, C.c_void_p(out_ptr),
                                         C.c_void_p(stream or 0)), "pt_image_u8_device")


def image_u8(fb):
    """make_image's normalisation of a host framebuffer (H, W, 3) float32 or
    float64, computed on the GPU: global min-max, x255, uint8 truncation."""
    fb = np.asarray(fb)
    if fb.dtype not in (np.float32, np.float64):
        fb = fb.astype(np.float64)
    fb = np.ascontiguousarray(fb)
    H, W = fb.shape[:2]
    out = np.zeros((H, W, 3), dtype=np.uint8)
    _native.check(_native.lib().pt_image_u8(C.c_void_p(fb.ctypes.data), W, H,
                                            PT_FLAG_OUT_F64 if fb.dtype == np.float64 else 0,
                                            C.c_void_p(out.ctypes.data)), "pt_image_u8")
    return out


def to_list_order(fb):
    """Framebuffer (H, W, 3) -> (W*H, 3) in the reference's list order
    k = ix*H + iy (the order of `colored_intersections`, main.py:177-183)."""
    fb = np.asarray(fb)
    H, W = fb.shape[:2]
    return fb[::-1].transpose(1, 0, 2).reshape(W * H, 3)


def from_list_order(colors, width, height):
    """Inverse of to_list_order."""
    c = np.asarray(colors).reshape(width, height, 3)
    return c.transpose(1, 0, 2)[::-1]


def band_row_indices(height, row_begin=0, row_end=None, row_step=1, row_phase=0):
    """iy of each framebuffer row of a band render, top row first."""
    return band_rows(height, row_begin, row_end, row_step, row_phase)[::-1]
