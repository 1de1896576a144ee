"""Shared fixtures.  `gpu`-marked tests need an MI355X (run on the GPU box with
`pytest -m gpu`); everything else runs on CPU in the build container."""
import ctypes as C
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
CORNELL = os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libpt_hip.so")


@pytest.fixture(scope="session")
def cornell():
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(CORNELL)


@pytest.fixture(scope="session")
def packed(cornell):
    from pathtracerpython_amd.pack import pack_scene
    return pack_scene(cornell)


def golden_renders():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "render_*.npz"))):
        g = np.load(f)
        out.append((os.path.basename(f), {k: g[k] for k in g.files}))
    return out


@pytest.fixture(scope="session")
def kat():
    g = np.load(os.path.join(GOLDEN, "kat_cornell.npz"))
    return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def mesh_golden(tmp_path_factory):
    """The edge-case mesh scene (BVH-sized: duplicates, a fan, triangles in
    the back wall's plane; tests/golden/mesh_scene.py) and the reference's
    render of it (gen_golden.py mesh): (scene, golden dict)."""
    sys.path.insert(0, GOLDEN)
    import mesh_scene as ms
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    d = tmp_path_factory.mktemp("mesh_golden")
    sc = scene_reader.Scene(ms.write_mesh_scene(str(d), os.path.dirname(CORNELL)))
    g = np.load(os.path.join(GOLDEN, ms.NAME))
    return sc, {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def k5mini_golden(tmp_path_factory):
    """The K5 scene generator at 1,000 triangles (synth.write_k5_scene, the
    BASELINE config-5 distribution) and the reference's render of it
    (gen_golden.py k5mini): (scene, golden dict)."""
    from pathtracerpython_amd import scene_reader
    from pathtracerpython_amd.synth import write_k5_scene
    scene_reader.VERBOSE = False
    g = np.load(os.path.join(GOLDEN, "k5mini_render_8x8_s2_b3_seed9.npz"))
    g = {k: g[k] for k in g.files}
    d = tmp_path_factory.mktemp("k5mini_golden")
    sc = scene_reader.Scene(write_k5_scene(str(d), n_tris=int(g["n_tris"]), seed=0,
                                           size=int(g["width"])))
    return sc, g


def scene_goldens():
    """The reference's renders of the test scenes below (gen_golden.py
    scenes): [(name, writer, golden dict)]."""
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*_scene_*_render_*.npz"))):
        g = np.load(f)
        name = os.path.basename(f)
        out.append((name, name.split("_render_")[0].rsplit("_", 1)[0], {k: g[k] for k in g.files}))
    return out


def scene_golden_ids():
    return [n for n, _, _ in scene_goldens()]


def scene_of_golden(tmp_path, writer, g):
    return globals()[writer](tmp_path, int(g["scene_seed"]))


@pytest.fixture(scope="session")
def hostcheck():
    """Host build of the kernel's per-lane code (tests/hostcheck)."""
    d = os.path.join(ROOT, "tests", "hostcheck")
    subprocess.run(["make", "-s", "-C", d], check=True)
    lib = C.CDLL(os.path.join(d, "build", "libhostcheck.so"))
    lib.hc_render.restype = C.c_int
    lib.hc_filter_selftest.restype = C.c_int
    return lib


def hc_render(lib, packed, params, force64=False, count=True):
    from pathtracerpython_amd._abi import band_rows
    rows = len(band_rows(params.height, params.row_begin, params.row_end, params.row_step,
                         params.row_phase))
    out = np.zeros((rows, params.width, 3), dtype=np.float64)
    cnt = (C.c_uint64 * 8)()
    rc = lib.hc_render(C.byref(packed.desc), C.byref(params), int(force64),
                       out.ctypes.data_as(C.POINTER(C.c_double)), cnt if count else None)
    assert rc == 0
    names = ("closest_tests", "shadow_tests", "ray_bounces", "shading_points", "light_hits",
             "escapes", "f64_fallbacks", "f64_rescans")
    return out, dict(zip(names, (int(x) for x in cnt)))


def random_scene(tmp_path, n_tris, seed, light_scale=1.0):
    """A Cornell variant with an extra random-triangle object (plain v/f OBJ,
    same ingest as the reference's), written to tmp_path."""
    import shutil
    rs = np.random.RandomState(seed)
    src = os.path.dirname(CORNELL)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp_path / f)
    c = rs.uniform([-3.5, -3.5, -32.0], [3.5, 3.5, -17.0], (n_tris, 3))
    lines = []
    for i in range(n_tris):
        for _ in range(3):
            v = c[i] + rs.normal(0, 0.6, 3)
            lines.append("v %.9f %.9f %.9f" % tuple(v))
    for i in range(n_tris):
        lines.append("f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
    (tmp_path / "rand.obj").write_text("\n".join(lines) + "\n")
    sdl = open(CORNELL).read().replace(
        "output cornell.pnm",
        "object rand.obj 0.2 0.5 0.9 0.3 0.6 0.4 0 3\noutput cornell.pnm")
    (tmp_path / "scene.sdl").write_text(sdl)
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(str(tmp_path / "scene.sdl"))


def clustered_scene(tmp_path, n_tris, seed):
    """A Cornell variant whose extra object is clusters of tiny and
    near-degenerate triangles (vertices 1e-4 to 1e-6 apart around 6 points,
    every third one a sliver): BVH nodes far smaller than their distance from
    the origin, the case where an absent child's empty quantised box could
    round to a point."""
    import shutil
    rs = np.random.RandomState(seed)
    src = os.path.dirname(CORNELL)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp_path / f)
    centres = rs.uniform([-3.5, -3.5, -32.0], [3.5, 3.5, -17.0], (6, 3))
    lines = []
    for i in range(n_tris):
        c = centres[i % 6] + rs.normal(0, 1e-3, 3)
        scale = 10.0 ** rs.uniform(-6, -4)
        a = c + rs.normal(0, scale, 3)
        b = c + rs.normal(0, scale, 3)
        d = (a + b) / 2 + rs.normal(0, scale * (1e-2 if i % 3 == 0 else 1.0), 3)
        for v in (a, b, d):
            lines.append("v %.12f %.12f %.12f" % tuple(v))
    for i in range(n_tris):
        lines.append("f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
    (tmp_path / "clus.obj").write_text("\n".join(lines) + "\n")
    sdl = open(CORNELL).read().replace(
        "output cornell.pnm",
        "object clus.obj 0.2 0.5 0.9 0.3 0.6 0.4 0 3\noutput cornell.pnm")
    (tmp_path / "scene.sdl").write_text(sdl)
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(str(tmp_path / "scene.sdl"))


def multi_mesh_scene(tmp_path, seed, n_tris=(120, 90)):
    """A Cornell variant whose FIRST objects are two random meshes (both large
    enough for the BVH) of different colours, with a small object between
    them: the leaked colour of main.py:70 (first occluder in scene order of
    the last shadow ray) then depends on which BVH object — or wall — is
    the lowest occluding one, across the BVH and the uniform units."""
    import shutil
    rs = np.random.RandomState(seed)
    src = os.path.dirname(CORNELL)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp_path / f)

    def mesh(name, n, lo, hi, sigma):
        c = rs.uniform(lo, hi, (n, 3))
        lines = ["v %.9f %.9f %.9f" % tuple(c[i] + rs.normal(0, sigma, 3))
                 for i in range(n) for _ in range(3)]
        lines += ["f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3) for i in range(n)]
        (tmp_path / name).write_text("\n".join(lines) + "\n")

    mesh("meshA.obj", n_tris[0], [-3.5, -3.5, -30.0], [3.5, 3.0, -18.0], 0.5)
    mesh("meshB.obj", n_tris[1], [-3.0, -2.0, -28.0], [3.0, 3.5, -20.0], 0.7)
    mesh("small.obj", 6, [-1.0, 1.0, -24.0], [1.0, 3.0, -22.0], 0.8)
    sdl = open(CORNELL).read().replace(
        "# left wall RED",
        "object meshA.obj 0.9 0.1 0.8 0.3 0.6 0.3 0 5\n"
        "object small.obj 0.1 0.9 0.9 0.3 0.7 0 0 5\n"
        "object meshB.obj 0.2 0.3 1.0 0.3 0.5 0.4 0 3\n"
        "# left wall RED")
    (tmp_path / "scene.sdl").write_text(sdl)
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(str(tmp_path / "scene.sdl"))


def quad_scene(tmp_path, seed, n_quads=14):
    """A Cornell variant with an object of random parallelograms split along
    a diagonal in every vertex labelling the unit builder distinguishes (the
    vertex opposite the shared diagonal first / second / third in the first
    triangle, either diagonal, both orientations), skewed coplanar quads that
    are no parallelogram, and single triangles.  Coordinates are multiples of
    1/64, so the parallelogram relation D = A + C - B holds exactly in the
    parsed doubles (pt_prepare.h quad_rot)."""
    import shutil
    rs = np.random.RandomState(seed)
    src = os.path.dirname(CORNELL)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp_path / f)
    g = lambda x: np.round(np.asarray(x) * 64.0) / 64.0
    verts, faces = [], []
    patterns = [((0, 1, 2), (0, 2, 3)), ((1, 2, 0), (0, 2, 3)), ((2, 0, 1), (2, 3, 0)),
                ((0, 1, 3), (1, 2, 3)), ((0, 2, 1), (0, 3, 2)), ((3, 0, 1), (1, 2, 3))]
    for q in range(n_quads):
        a = g(rs.uniform([-3.0, -3.0, -30.0], [3.0, 3.0, -19.0]))
        e1 = g(rs.normal(0, 0.9, 3))
        e2 = g(rs.normal(0, 0.9, 3))
        quad = [a, a + e1, a + e1 + e2, a + e2]       # A B C D, A + C = B + D
        if q % 5 == 4:                                  # coplanar, no parallelogram
            quad[3] = a + e2 + g(0.3 * e1)
        base = len(verts)
        verts += quad
        t0, t1 = patterns[q % len(patterns)]
        faces.append(tuple(base + i for i in t0))
        faces.append(tuple(base + i for i in t1))
        if q % 7 == 3:                                  # a single triangle between quads
            b = len(verts)
            verts += [g(a + rs.normal(0, 0.7, 3)) for _ in range(3)]
            faces.append((b, b + 1, b + 2))
    lines = ["v %.6f %.6f %.6f" % tuple(v) for v in verts]
    lines += ["f %d %d %d" % (f[0] + 1, f[1] + 1, f[2] + 1) for f in faces]
    (tmp_path / "quads.obj").write_text("\n".join(lines) + "\n")
    sdl = open(CORNELL).read().replace(
        "output cornell.pnm",
        "object quads.obj 0.8 0.6 0.2 0.3 0.6 0.3 0 4\noutput cornell.pnm")
    (tmp_path / "scene.sdl").write_text(sdl)
    from pathtracerpython_amd import scene_reader
    scene_reader.VERBOSE = False
    return scene_reader.Scene(str(tmp_path / "scene.sdl"))
