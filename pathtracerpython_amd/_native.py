"""ctypes binding of libpt_hip.so (include/pt_capi.h).

The HIP library is the only implementation of the hot path: there is no CPU
fallback.  If the library is missing or no gfx950 device is visible, calls
raise `NativeError` — loudly, never silently.
"""
import ctypes as C
import os

from ._abi import PtMesh, PtRenderParams, PtSceneDesc, PtStats  # noqa: F401 (PtMesh re-exported)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PT_HIP_LIB", os.path.join(HERE, "_lib", "libpt_hip.so"))

_lib = None


class NativeError(RuntimeError):
    pass


def _bind(lib):
    vp = C.c_void_p
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int32)
    sig = {
        "pt_api_version": ([], C.c_int),
        "pt_last_error": ([], C.c_char_p),
        "pt_build_id": ([], C.c_char_p),
        "pt_test_fault_inject": ([C.c_int32], C.c_int),
        "pt_device_count": ([ip], C.c_int),
        "pt_scene_create": ([C.POINTER(PtSceneDesc), C.POINTER(vp)], C.c_int),
        "pt_scene_create_on": ([C.POINTER(PtSceneDesc), C.c_int32, C.POINTER(vp)], C.c_int),
        "pt_render_multi": ([C.POINTER(vp), C.c_int32, C.POINTER(PtRenderParams), vp,
                             C.POINTER(PtStats)], C.c_int),
        "pt_scene_destroy": ([vp], None),
        "pt_band_rows": ([C.POINTER(PtRenderParams), ip], C.c_int),
        "pt_render_device": ([vp, C.POINTER(PtRenderParams), vp, vp, C.POINTER(PtStats)], C.c_int),
        "pt_render": ([vp, C.POINTER(PtRenderParams), vp, C.POINTER(PtStats)], C.c_int),
        "pt_last_kernel_ms": ([vp, C.POINTER(C.c_float)], C.c_int),
        "pt_intersect_objects": ([vp, dp, C.c_int64, ip, dp], C.c_int),
        "pt_compute_color": ([vp, ip, dp, dp, dp, C.c_int64, dp], C.c_int),
        "pt_image_u8_device": ([vp, C.c_int32, C.c_int32, C.c_uint32, vp, vp], C.c_int),
        "pt_image_u8": ([vp, C.c_int32, C.c_int32, C.c_uint32, vp], C.c_int),
        "pt_assemble_bands_device": ([vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_uint32,
                                      vp, vp], C.c_int),
        "pt_host_map": ([vp, C.c_uint64, C.POINTER(vp)], C.c_int),
        "pt_host_unmap": ([vp], C.c_int),
        "pt_signal": ([vp, C.c_uint64, vp], C.c_int),
        "pt_wait_flags": ([vp, C.c_int32, C.c_int32, C.c_uint64, C.c_double], C.c_int),
        "pt_obj_load": ([C.c_char_p, C.POINTER(C.POINTER(PtMesh))], C.c_int),
        "pt_mesh_free": ([C.POINTER(PtMesh)], None),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


EXPORTS = ("pt_api_version", "pt_last_error", "pt_build_id", "pt_test_fault_inject",
           "pt_device_count", "pt_scene_create",
           "pt_scene_create_on", "pt_render_multi", "pt_scene_destroy", "pt_band_rows",
           "pt_render_device", "pt_render", "pt_last_kernel_ms", "pt_intersect_objects", "pt_compute_color",
           "pt_image_u8_device", "pt_image_u8", "pt_assemble_bands_device", "pt_host_map",
           "pt_host_unmap", "pt_signal", "pt_wait_flags", "pt_obj_load", "pt_mesh_free")


def lib():
    """Load libpt_hip.so once.  torch (if present) is imported first so the
    library binds to the same HIP runtime instance torch uses."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} not found: build it with `python __graft_entry__.py build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        import torch  # noqa: F401  (shares libamdhip64 with torch)
    except Exception:
        pass
    raw = C.CDLL(LIB_PATH)
    from ._abi import PT_API_VERSION
    if not hasattr(raw, "pt_build_id") or raw.pt_api_version() != PT_API_VERSION:
        raise NativeError(f"{LIB_PATH} has C-ABI version {raw.pt_api_version()}, this binding "
                          f"needs {PT_API_VERSION}: rebuild it (python __graft_entry__.py build)")
    lib_ = _bind(raw)
    got = lib_.pt_build_id().decode("ascii", "replace")
    want = source_sha()
    # a library built from other sources than those on disk is refused, so a
    # measurement never carries the wrong sources' name (build.py); dev
    # variants built from patched sources opt out explicitly and are still
    # named by their own id (bench.py reports build_id())
    if got != want and os.environ.get("PT_ALLOW_FOREIGN_BUILD") != "1":
        raise NativeError(f"{LIB_PATH} was built from sources {got}, the sources on disk are {want}: "
                          "rebuild it (python __graft_entry__.py build)")
    _lib = lib_
    return _lib


def source_sha():
    from .build import source_sha as sha
    return sha()


def build_id():
    """The loaded library's PT_BUILD_ID (the content hash of its sources)."""
    return lib().pt_build_id().decode("ascii", "replace")


def last_error():
    msg = lib().pt_last_error()
    return msg.decode() if msg else ""


def check(rc, what):
    if rc != 0:
        raise NativeError(f"{what} failed ({rc}): {last_error()}")


def device_count():
    n = C.c_int32(0)
    check(lib().pt_device_count(C.byref(n)), "pt_device_count")
    return n.value
