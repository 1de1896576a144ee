"""ctypes mirror of include/pt_capi.h (structs, flags, error codes)."""
import ctypes as C

PT_API_VERSION = 7

PT_OK = 0
PT_EINVAL = -1
PT_EHIP = -2
PT_ENOMEM = -3
PT_ENODEV = -4
PT_EUNSUPPORTED = -5
PT_ETIMEOUT = -6

PT_FLAG_RR = 1 << 0
PT_FLAG_FORCE_F64 = 1 << 1
PT_FLAG_COUNT = 1 << 2
PT_FLAG_OUT_F64 = 1 << 3
PT_FLAG_MEGAKERNEL = 1 << 4
PT_FLAG_WALK_COUNT = 1 << 5
PT_FLAG_KERNEL_TIMES = 1 << 6
# bit 7: reserved (v4's PT_FLAG_TREE_WALK, retired in v5)

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class PtSceneDesc(C.Structure):
    _fields_ = [
        ("n_tri", C.c_int32), ("n_obj_tri", C.c_int32), ("n_obj", C.c_int32),
        ("reserved", C.c_int32),
        ("tri_v", _dp), ("tri_n", _dp), ("tri_area", _dp), ("tri_obj", _ip),
        ("mat", _dp),
        ("eye", C.c_double * 3), ("ortho", C.c_double * 4),
        ("ambient", C.c_double), ("light_rgb", C.c_double * 3),
    ]


class PtRenderParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
        ("bounces", C.c_int32), ("seed", C.c_uint64), ("flags", C.c_uint32),
        ("rr_depth", C.c_int32), ("row_begin", C.c_int32),
        ("row_end", C.c_int32), ("row_step", C.c_int32),
        ("row_phase", C.c_int32), ("sample_begin", C.c_int32),
        ("out_row_stride", C.c_int32), ("lanes_per_pixel", C.c_int32),
        ("reserved", C.c_int32),
    ]


class PtMesh(C.Structure):
    """pt_mesh (include/pt_capi.h): a mesh read by pt_obj_load."""
    _fields_ = [("n_vert", C.c_int64), ("n_tri", C.c_int64), ("n_skip", C.c_int64),
                ("vert", C.POINTER(C.c_double)), ("face", C.POINTER(C.c_int64)),
                ("tri_v", C.POINTER(C.c_double)), ("tri_n", C.POINTER(C.c_double)),
                ("tri_area", C.POINTER(C.c_double)), ("skip_off", C.POINTER(C.c_int64)),
                ("skip_len", C.POINTER(C.c_int64))]


class PtStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "closest_tests", "shadow_tests", "ray_bounces", "shading_points",
        "light_hits", "escapes", "f64_fallbacks", "f64_rescans",
        "shadow_queries", "shadow_node_visits", "shadow_leaf_units",
        "closest_queries", "closest_node_visits", "closest_leaf_units")] + \
        [(n, C.c_double) for n in ("shade_ms", "shadow_ms", "closest_ms")] + \
        [(n, C.c_uint64) for n in ("shade_launches", "shadow_launches", "closest_launches")] + \
        [("sort_ms", C.c_double), ("sort_launches", C.c_uint64)]

    COUNTERS = ("closest_tests", "shadow_tests", "ray_bounces", "shading_points",
                "light_hits", "escapes", "f64_fallbacks", "f64_rescans")

    def as_dict(self, all_fields=False):
        """The reference-semantics counters (PT_FLAG_COUNT); all_fields adds
        the wavefront walk counts and per-kernel times."""
        names = [n for n, _ in self._fields_] if all_fields else self.COUNTERS
        return {n: (float if n.endswith("_ms") else int)(getattr(self, n)) for n in names}


def make_params(width, height, spp, bounces, seed, flags=0, rr_depth=3,
                row_begin=0, row_end=None, row_step=1, row_phase=0,
                sample_begin=0, out_row_stride=0, lanes_per_pixel=0):
    p = PtRenderParams()
    p.width, p.height, p.spp, p.bounces = int(width), int(height), int(spp), int(bounces)
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.flags = int(flags)
    p.rr_depth = int(rr_depth)
    p.row_begin = int(row_begin)
    p.row_end = int(height if row_end is None else row_end)
    p.row_step = int(row_step)
    p.row_phase = int(row_phase)
    p.sample_begin = int(sample_begin)
    p.out_row_stride = int(out_row_stride)
    p.lanes_per_pixel = int(lanes_per_pixel)
    return p


def with_flags(p, add=0, **fields):
    """A copy of params p with flag bits `add` set and any fields replaced."""
    q = PtRenderParams()
    C.pointer(q)[0] = p
    q.flags = p.flags | int(add)
    for k, v in fields.items():
        setattr(q, k, int(v))
    return q


def band_rows(height, row_begin=0, row_end=None, row_step=1, row_phase=0):
    """Python twin of pt_band_rows: the iy values a launch renders, in order."""
    row_end = height if row_end is None else row_end
    return [iy for iy in range(row_begin, row_end) if iy % row_step == row_phase]
