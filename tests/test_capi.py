"""C-ABI of libpt_hip.so: loads without a GPU, exports every entry point
include/pt_capi.h declares, validates arguments, and fails loudly (no CPU
fallback) when no gfx950 device is present."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from pathtracerpython_amd import _native
from pathtracerpython_amd._abi import PtRenderParams, PtSceneDesc, PtStats, band_rows, make_params

HEADER = os.path.join(ROOT, "include", "pt_capi.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_api():
    assert set(declared_functions()) == set(_native.EXPORTS)


def test_library_exports_every_symbol():
    lib = _native.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_abi_struct_layout(hostcheck):
    """The ctypes mirror (_abi.py) against the C++ compiler's layout of
    include/pt_capi.h (tests/hostcheck)."""
    out = (C.c_int64 * 8)()
    hostcheck.hc_abi_layout(out)
    assert list(out) == [C.sizeof(PtSceneDesc), C.sizeof(PtRenderParams), C.sizeof(PtStats),
                         PtStats.shadow_queries.offset, PtStats.shade_ms.offset,
                         PtStats.closest_launches.offset, PtSceneDesc.light_rgb.offset,
                         PtRenderParams.sample_begin.offset]
    assert C.sizeof(PtStats) == 14 * 8 + 3 * 8 + 3 * 8 + 2 * 8


def test_api_version():
    from pathtracerpython_amd._abi import PT_API_VERSION
    assert _native.lib().pt_api_version() == PT_API_VERSION == 7


@pytest.mark.parametrize("H,step,phase,b,e", [(10, 1, 0, 0, 10), (10, 3, 1, 0, 10),
                                              (10, 4, 3, 0, 10), (7, 2, 0, 3, 6),
                                              (5, 8, 6, 0, 5), (9, 1, 0, 9, 9)])
def test_band_rows_matches_python(H, step, phase, b, e):
    p = make_params(4, H, 1, 1, 0, row_begin=b, row_end=e, row_step=step, row_phase=phase)
    n = C.c_int32(-1)
    assert _native.lib().pt_band_rows(C.byref(p), C.byref(n)) == 0
    assert n.value == len(band_rows(H, b, e, step, phase))


def test_band_rows_rejects_bad_step():
    p = make_params(4, 4, 1, 1, 0, row_step=2, row_phase=2)
    n = C.c_int32()
    assert _native.lib().pt_band_rows(C.byref(p), C.byref(n)) == -1
    assert "row_step" in _native.last_error()


def test_scene_create_validates(packed):
    lib = _native.lib()
    h = C.c_void_p()
    assert lib.pt_scene_create(None, C.byref(h)) != 0
    bad = PtSceneDesc()
    C.memmove(C.byref(bad), C.byref(packed.desc), C.sizeof(PtSceneDesc))
    bad.n_obj_tri = bad.n_tri   # light without triangles
    rc = lib.pt_scene_create(C.byref(bad), C.byref(h))
    assert rc in (-1, -4)   # EINVAL, or ENODEV first when no GPU is visible


def test_no_gpu_fails_loudly(packed):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from pathtracerpython_amd.render import Renderer
    with pytest.raises(_native.NativeError, match="no HIP device|gfx950"):
        Renderer(_load_cornell())


def _load_cornell():
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl"))


def test_missing_library_is_an_error(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_native.NativeError, match="no CPU fallback"):
        _native.lib()


def test_list_order_roundtrip():
    from pathtracerpython_amd.render import from_list_order, to_list_order
    W, H = 5, 3
    cols = np.arange(W * H * 3, dtype=np.float64).reshape(W * H, 3)
    fb = from_list_order(cols, W, H)
    # k = ix*H + iy sits at fb[H-1-iy, ix]
    for k in range(W * H):
        ix, iy = divmod(k, H)
        assert np.array_equal(fb[H - 1 - iy, ix], cols[k])
    assert np.array_equal(to_list_order(fb), cols)


def test_image_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from pathtracerpython_amd.render import image_u8
    with pytest.raises(_native.NativeError, match="no HIP device"):
        image_u8(np.zeros((2, 2, 3)))


def test_wait_flags_on_host():
    """pt_wait_flags is host code (no GPU): all flags at or above the value
    returns at once; a flag that never arrives times out with PT_ETIMEOUT."""
    from pathtracerpython_amd._abi import PT_ETIMEOUT
    lib = _native.lib()
    f = np.zeros(16, dtype=np.uint64)
    f[::4] = [3, 7, 3, 9]
    ptr = C.c_void_p(f.ctypes.data)
    assert lib.pt_wait_flags(ptr, 4, 4, 3, 1.0) == 0
    assert lib.pt_wait_flags(ptr, 0, 4, 99, 0.0) == 0
    assert lib.pt_wait_flags(ptr, 4, 4, 4, 0.05) == PT_ETIMEOUT
    assert "flag 0" in _native.last_error()
    assert lib.pt_wait_flags(ptr, 4, 0, 1, 0.05) == -1


def test_render_params_validation_without_gpu():
    """Flag bit 7 (v4's PT_FLAG_TREE_WALK) is retired, lanes_per_pixel must be
    a power of two <= min(64, spp), out_row_stride 0 or >= width*3: rejected
    by pt_render before any device is touched."""
    lib = _native.lib()
    out = np.zeros((4, 4, 3), dtype=np.float32)
    for kw in (dict(flags=1 << 7), dict(lanes_per_pixel=3), dict(lanes_per_pixel=16),
               dict(out_row_stride=11)):
        p = make_params(4, 4, 8, 1, 0, **{k: v for k, v in kw.items() if k == "flags"})
        for k, v in kw.items():
            setattr(p, k, v)
        assert lib.pt_render(None, C.byref(p), C.c_void_p(out.ctypes.data), None) == -1
        assert "null scene" not in _native.last_error()


def test_host_map_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    buf = np.zeros(4096, dtype=np.uint8)
    dev = C.c_void_p()
    assert _native.lib().pt_host_map(C.c_void_p(buf.ctypes.data), buf.nbytes, C.byref(dev)) == -4


def test_build_id_is_the_sources_hash():
    """the library carries the content hash of the sources it
    was built from (pt_build_id, compiled in by build.py), which is the hash
    of the sources on disk, and build.py reads the same id from the file."""
    from pathtracerpython_amd import build
    sha = build.source_sha()
    assert _native.build_id() == sha
    assert build.embedded_build_id(_native.LIB_PATH) == sha
    assert not build._stale()


def test_library_with_another_build_id_is_refused(tmp_path):
    """A library stamped with another sha (here: a copy whose embedded id is
    rewritten) is refused by _native.lib(), in a fresh process."""
    import subprocess
    import sys
    from pathtracerpython_amd import build
    data = open(_native.LIB_PATH, "rb").read()
    i = data.find(build.MARKER)
    assert i >= 0 and data.find(build.MARKER, i + 1) < 0
    j = i + len(build.MARKER)
    other = "0123456789abcdef" if data[j:j + 16] != b"0123456789abcdef" else "fedcba9876543210"
    bad = tmp_path / "libpt_hip.so"
    bad.write_bytes(data[:j] + other.encode() + data[j + 16:])
    assert build.embedded_build_id(str(bad)) == other
    code = ("from pathtracerpython_amd import _native\n"
            "try:\n    _native.lib()\nexcept _native.NativeError as e:\n    print('REFUSED', e)\n"
            "else:\n    print('LOADED', _native.build_id())\n")
    env = dict(os.environ, PT_HIP_LIB=str(bad))
    env.pop("PT_ALLOW_FOREIGN_BUILD", None)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120).stdout
    assert "REFUSED" in out and f"built from sources {other}" in out, out
    # dev variants opt out explicitly, and are then named by their own id
    env["PT_ALLOW_FOREIGN_BUILD"] = "1"
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120).stdout
    assert f"LOADED {other}" in out, out


def test_build_is_stale_when_a_source_changes(tmp_path):
    """Staleness is the content hash, not file times: a touched but unchanged
    source is not stale, an edited copy of the sources is."""
    import shutil
    from pathtracerpython_amd import build
    os.utime(os.path.join(build.CSRC, "pt_core.h"))
    assert not build._stale()
    csrc = tmp_path / "csrc"
    shutil.copytree(build.CSRC, csrc)
    assert build.source_sha(str(csrc)) == build.source_sha()
    with open(csrc / "pt_core.h", "a") as f:
        f.write("\n// edit\n")
    assert build.source_sha(str(csrc)) != build.source_sha()
    assert build._stale(csrc=str(csrc))


def test_build_id_covers_the_compile_recipe():
    """The K2 kernel's and the shade step's units are compiled under their own
    scheduler flag (build.UNITS): the same sources under another recipe are
    another binary, so they carry another id."""
    from pathtracerpython_amd import build
    assert set(build.UNITS) == {"pt_k2.hip", "pt_shade.hip"}
    for u in build.UNITS:
        assert os.path.exists(os.path.join(build.CSRC, u))
    assert build.source_sha(units={}) != build.source_sha()
    assert build.source_sha(flags=build.FLAGS + ["-O2"]) != build.source_sha()


def test_variant_builds_carry_their_own_id():
    """a build with -D switches is named by the sources AND its
    switches, so it never passes for the default build (the binding loads it
    only with PT_ALLOW_FOREIGN_BUILD=1)."""
    from pathtracerpython_amd import build
    sha = build.source_sha()
    assert build.variant_id(sha, ()) == sha
    v = build.variant_id(sha, ("PT_MMERGE=0",))
    assert v != sha and len(v) == 16
    assert build.variant_id(sha, ("A=1", "B=2")) == build.variant_id(sha, ("B=2", "A=1"))
    assert build.variant_id(sha, ("A=1",)) != build.variant_id(sha, ("A=2",))
