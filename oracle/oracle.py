"""ctypes wrapper of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the checker; never by the product package.  See pt_oracle.c's header.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(HERE, "pt_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        build()
    from pathtracerpython_amd._abi import PtRenderParams, PtSceneDesc, PtStats
    lib = C.CDLL(LIB)
    lib.oracle_render.argtypes = [C.POINTER(PtSceneDesc), C.POINTER(PtRenderParams),
                                  C.POINTER(C.c_int64), C.c_int64, C.c_int, _dp,
                                  C.POINTER(PtStats)]
    lib.oracle_render.restype = C.c_int
    lib.oracle_intersect.argtypes = [_dp, _dp, _dp, _dp]
    lib.oracle_intersect.restype = C.c_int
    lib.oracle_intersect_objects.argtypes = [C.POINTER(PtSceneDesc), _dp, C.c_int64, _ip, _dp]
    lib.oracle_compute_color.argtypes = [C.POINTER(PtSceneDesc), _ip, _dp, _dp, _dp,
                                         C.c_int64, _dp]
    lib.oracle_rotate.argtypes = [_dp, _dp, _dp]
    lib.oracle_rotate.restype = None
    lib.oracle_pick_light.argtypes = [C.POINTER(PtSceneDesc), C.c_double]
    lib.oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_uint32)]
    lib.oracle_philox.restype = None
    _lib = lib
    return lib


def _d(a):
    return a.ctypes.data_as(_dp)


def host_threads():
    """Host threads this process may use: the CPUs it is pinned to, capped by
    OMP_NUM_THREADS when set (the GPU box sets it to the CPU share of one
    GPU; os.cpu_count() there shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, 256))


def render(packed, width, height, spp, bounces, seed, flags=0, rr_depth=3,
           pixels=None, threads=None, sample_begin=0):
    """Averaged colours (n, 3) f64 for reference list indices `pixels`
    (default: all, k = ix*H + iy) and the work counters."""
    from pathtracerpython_amd._abi import PtStats, make_params
    lib = load()
    if pixels is None:
        pixels = np.arange(width * height, dtype=np.int64)
    pixels = np.ascontiguousarray(pixels, dtype=np.int64)
    out = np.zeros((len(pixels), 3), dtype=np.float64)
    p = make_params(width, height, spp, bounces, seed, flags, rr_depth,
                    sample_begin=sample_begin)
    st = PtStats()
    nt = threads or host_threads()
    rc = lib.oracle_render(C.byref(packed.desc), C.byref(p),
                           pixels.ctypes.data_as(C.POINTER(C.c_int64)),
                           len(pixels), nt, _d(out), C.byref(st))
    if rc:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return out, st.as_dict()


def intersect(tri, o, d):
    lib = load()
    tri = np.ascontiguousarray(tri, dtype=np.float64).reshape(9)
    o = np.ascontiguousarray(o, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.float64)
    P = np.zeros(3)
    h = lib.oracle_intersect(_d(tri), _d(o), _d(d), _d(P))
    return bool(h), P


def intersect_objects(packed, rays):
    lib = load()
    rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
    n = rays.shape[0]
    tri = np.zeros(n, dtype=np.int32)
    P = np.zeros((n, 3))
    lib.oracle_intersect_objects(C.byref(packed.desc), _d(rays), n,
                                 tri.ctypes.data_as(_ip), _d(P))
    return tri, P


def compute_color(packed, obj, point, normal, u):
    lib = load()
    obj = np.ascontiguousarray(obj, dtype=np.int32)
    point = np.ascontiguousarray(point, dtype=np.float64).reshape(-1, 3)
    normal = np.ascontiguousarray(normal, dtype=np.float64).reshape(-1, 3)
    u = np.ascontiguousarray(u, dtype=np.float64).reshape(-1, 12)
    out = np.zeros((len(obj), 3))
    lib.oracle_compute_color(C.byref(packed.desc), obj.ctypes.data_as(_ip), _d(point),
                             _d(normal), _d(u), len(obj), _d(out))
    return out


def rotate(n, v):
    lib = load()
    n = np.ascontiguousarray(n, dtype=np.float64)
    v = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(3)
    lib.oracle_rotate(_d(n), _d(v), _d(out))
    return out


def pick_light(packed, u):
    return load().oracle_pick_light(C.byref(packed.desc), float(u))


def philox(ctr, key):
    lib = load()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.oracle_philox(c, k, o)
    return tuple(o)
