#!/usr/bin/env python3
"""Golden-vector generator — TEST INFRASTRUCTURE, runs only in the build
container (it imports the untouched reference from /root/reference, which does
not exist on the GPU box).  Its outputs are the committed fixtures in this
directory; nothing under the product package imports this file.

What it does (SURVEY.md §8c "Deterministic harness"):
  * registers inert stand-ins for the debug/plot modules the reference imports
    but never uses on the numeric path (`ipdb`, `colorama` — utils.py:3-7;
    `pyqtgraph` — plot.py:2-3); they are not installed here;
  * replaces `uniform` in `main` and `utils` (both bound at import,
    main.py:16, utils.py:9) by the keyed Philox4x32-10 draw of philox_ref.py.
    The (pixel, sample, bounce) context comes from main()'s frame locals
    (`i_ray`, `rays_counter`, `bounces_counter`, main.py:186/192/211/236);
  * replaces `main.Pool` (main.py:197/208) by a synchronous pool that returns
    real `multiprocessing.pool.ApplyResult`s, so the `type(...) is ApplyResult`
    check at main.py:227 still holds;
  * replaces `main.make_image` (main.py:288) to capture the averaged colour list
    before min-max normalisation, and also keeps the real make_image output;
  * overrides the SDL `size` (scene_reader.py:153-155) via a Scene subclass.

Usage:  python gen_golden.py [all|scene|kat|mesh|meshkat|k5mini|scenes|render W H SPP B SEED]
"""
import contextlib
import io
import math
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("PT_REFERENCE", "/root/reference")
SCENE = os.path.join(REF, "objs", "cornellroom.sdl")

sys.path.insert(0, HERE)
from philox_ref import keyed_u  # noqa: E402


def _install_stubs():
    def _noop(*a, **k):
        return None

    ipdb = types.ModuleType("ipdb")
    ipdb.set_trace = _noop
    ipdb_main = types.ModuleType("ipdb.__main__")
    ipdb_main.set_trace = _noop
    ipdb.__main__ = ipdb_main

    class _Codes:
        def __getattr__(self, name):
            return ""

    colorama = types.ModuleType("colorama")
    colorama.init = _noop
    colorama.Fore = colorama.Back = colorama.Style = _Codes()

    pg = types.ModuleType("pyqtgraph")
    pg.opengl = types.ModuleType("pyqtgraph.opengl")
    pg.mkQApp = _noop
    for name, mod in {"ipdb": ipdb, "ipdb.__main__": ipdb_main,
                      "colorama": colorama, "pyqtgraph": pg,
                      "pyqtgraph.opengl": pg.opengl}.items():
        sys.modules.setdefault(name, mod)


def import_reference():
    sys.dont_write_bytecode = True        # never write into /root/reference
    _install_stubs()
    sys.path.insert(0, REF)
    import main as ref_main                # noqa: E402
    import utils as ref_utils              # noqa: E402
    import scene_reader as ref_scene       # noqa: E402
    return ref_main, ref_utils, ref_scene


class KeyedRNG:
    """Replacement for random.uniform keyed by (pixel, sample, bounce, slot)."""

    def __init__(self, seed, main_code):
        self.seed = seed
        self.main_code = main_code
        self.ctx = None          # (pixel, sample, bounce) for compute_color
        self.slot = 0
        self.bounce_slots = {}   # (pixel, sample, bounce) -> next bounce slot
        self.forced = None       # list of u's for KATs

    def uniform(self, a, b):
        if self.forced is not None:
            u = self.forced.pop(0)
            return a + (b - a) * u
        caller = sys._getframe(1)
        if caller.f_code is self.main_code:
            loc = caller.f_locals
            key = (loc["i_ray"], loc["rays_counter"], loc["bounces_counter"])
            slot = self.bounce_slots.get(key, 12)
            self.bounce_slots[key] = slot + 1
        else:
            key = self.ctx
            slot = self.slot
            self.slot += 1
        assert key is not None and slot < 16, (key, slot)
        u = keyed_u(self.seed, key[0], key[1], key[2], slot)
        return a + (b - a) * u


def make_sync_pool(ref_main, rng):
    from multiprocessing.pool import ApplyResult

    class SyncPool:
        def __init__(self, *args, **kwargs):
            self._cache = {}

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            return False

        def apply_async(self, func, args):
            if func is ref_main.compute_color:
                loc = sys._getframe(1).f_locals
                rng.ctx = (loc["i_ray"], loc["rays_counter"],
                           loc["bounces_counter"])
                rng.slot = 0
            value = func(*args)
            rng.ctx = None
            res = ApplyResult(self, None, None)
            res._set(0, (True, value))
            return res

    return SyncPool


def render_reference(width, height, spp, bounces, seed, scene=None):
    """Run the unmodified reference main() under the keyed harness (on
    `scene`, an SDL path; default the reference's Cornell room)."""
    ref_main, ref_utils, ref_scene = import_reference()
    rng = KeyedRNG(seed, ref_main.main.__code__)
    ref_main.uniform = rng.uniform
    ref_utils.uniform = rng.uniform
    ref_main.Pool = make_sync_pool(ref_main, rng)
    ref_main.tqdm = lambda it, *a, **k: it

    class SizedScene(ref_scene.Scene):
        def __init__(self, path):
            super().__init__(path)
            self.width, self.height = width, height

    ref_main.Scene = SizedScene
    captured = {}
    real_make_image = ref_utils.make_image

    def capture(x1, y1, x2, y2, w, h, intersections):
        captured["colors"] = np.array([np.asarray(c, dtype=np.float64)
                                       for c, _ in intersections])
        im = real_make_image(x1, y1, x2, y2, w, h, intersections)
        captured["png"] = np.asarray(im, dtype=np.uint8)
        return im

    ref_main.make_image = capture
    argv = sys.argv
    sys.argv = ["main.py", scene or SCENE, "-r", str(spp), "-b", str(bounces)]
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            ref_main.main()
    finally:
        sys.argv = argv
    return captured["colors"], captured["png"]


def gen_render(width, height, spp, bounces, seed):
    colors, png = render_reference(width, height, spp, bounces, seed)
    name = f"render_{width}x{height}_s{spp}_b{bounces}_seed{seed}.npz"
    np.savez_compressed(os.path.join(HERE, name), colors=colors, png=png,
                        width=width, height=height, spp=spp, bounces=bounces,
                        seed=seed)
    print("wrote", name, colors.shape, float(colors.min()), float(colors.max()))


def gen_mesh():
    """The BVH golden: the reference on the edge-case mesh scene of
    mesh_scene.py (written into a temporary directory)."""
    import tempfile
    import mesh_scene as ms
    d = tempfile.mkdtemp(prefix="pt_mesh_")
    sdl = ms.write_mesh_scene(d, os.path.join(REF, "objs"))
    colors, png = render_reference(ms.W, ms.H, ms.SPP, ms.BOUNCES, ms.SEED, scene=sdl)
    np.savez_compressed(os.path.join(HERE, ms.NAME), colors=colors, png=png, width=ms.W,
                        height=ms.H, spp=ms.SPP, bounces=ms.BOUNCES, seed=ms.SEED)
    print("wrote", ms.NAME, colors.shape, float(colors.min()), float(colors.max()))


def gen_mesh_kat():
    """`intersect_objects` (main.py:83-122) of the reference on the edge-case
    mesh scene (mesh_scene.py): the batched closest-hit API over a BVH object,
    with origins in the room, on the mesh's triangles (the sqd > 1e-5
    self-hit rule; duplicates) and at the eye."""
    import tempfile
    import mesh_scene as ms
    ref_main, _, ref_scene = import_reference()
    d = tempfile.mkdtemp(prefix="pt_mesh_kat_")
    sdl = ms.write_mesh_scene(d, os.path.join(REF, "objs"))
    with contextlib.redirect_stdout(io.StringIO()):
        sc = ref_scene.Scene(sdl)
    rs = np.random.RandomState(4321)
    mesh = ms.mesh_triangles()
    objs_plus = sc.objects + [{"geometry": sc.light_obj}]
    io_o, io_d, io_hit, io_p, io_obj, io_light = [], [], [], [], [], []
    for k in range(400):
        if k % 4 == 0:
            o = np.array(sc.eye, dtype=np.float64)
            dd = np.array([rs.uniform(-1, 1), rs.uniform(-1, 1), 0.0]) - o
        elif k % 4 == 1:   # on a mesh triangle (its centroid)
            t = mesh[rs.randint(len(mesh))]
            o = (t[0] + t[1] + t[2]) / 3.0
            dd = rs.normal(0, 1, 3)
        else:
            o = rs.uniform([-3.8, -3.8, -32.7], [3.8, 3.8, -16.6])
            dd = rs.normal(0, 1, 3)
        r = ref_main.intersect_objects((o, dd), sc.objects, sc.light_obj)
        io_o.append(o); io_d.append(dd)
        if r is None:
            io_hit.append(0); io_p.append(np.zeros(3)); io_obj.append(-1); io_light.append(0)
        else:
            p, n, obj, is_light = r
            idx = [i for i, oo in enumerate(objs_plus) if oo["geometry"] is obj["geometry"]][0]
            io_hit.append(1); io_p.append(np.asarray(p, dtype=np.float64))
            io_obj.append(idx); io_light.append(int(is_light))
    # compute_color (main.py:23-80, 142-145) at points on every object's
    # triangles, the mesh's included: shadow rays against the BVH object and
    # the leaked colour of the last one across BVH and uniform occluders
    rng = KeyedRNG(0, None)
    ref_main.uniform = rng.uniform
    import utils as ref_utils   # (already imported by import_reference)
    ref_utils.uniform = rng.uniform
    cc_p, cc_n, cc_obj, cc_u, cc_out = [], [], [], [], []
    for k in range(300):
        oi = rs.randint(len(sc.objects))
        g = sc.objects[oi]["geometry"]
        ti = rs.randint(len(g.triangles))
        t = np.array([list(v) for v in g.triangles[ti]])
        p = rs.dirichlet([1, 1, 1]) @ t
        n = g.normals[ti]
        u12 = [float(x) for x in rs.uniform(0, 1, 12)]
        rng.forced = list(u12)
        col = ref_main.compute_color(sc, sc.objects[oi], p, n)
        assert not rng.forced
        cc_p.append(p); cc_n.append(list(n)); cc_obj.append(oi)
        cc_u.append(u12); cc_out.append(np.asarray(col, dtype=np.float64))
    np.savez_compressed(os.path.join(HERE, "kat_mesh.npz"), io_o=np.array(io_o),
                        io_d=np.array(io_d), io_hit=np.array(io_hit, dtype=np.int32),
                        io_p=np.array(io_p), io_obj=np.array(io_obj, dtype=np.int32),
                        io_light=np.array(io_light, dtype=np.int32),
                        cc_p=np.array(cc_p), cc_n=np.array(cc_n),
                        cc_obj=np.array(cc_obj, dtype=np.int32), cc_u=np.array(cc_u),
                        cc_out=np.array(cc_out))
    print("wrote kat_mesh.npz", int(np.sum(io_hit)), "hits of", len(io_hit))


K5MINI = dict(n_tris=1000, W=8, H=8, spp=2, bounces=3, seed=9)
K5MINI_NAME = "k5mini_render_8x8_s2_b3_seed9.npz"   # (not render_*: the Cornell goldens)


def gen_k5mini():
    """The K5 scene generator (pathtracerpython_amd/synth.py, the BASELINE
    config-5 distribution) at 1,000 triangles, rendered by the reference."""
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from pathtracerpython_amd.synth import write_k5_scene
    c = K5MINI
    d = tempfile.mkdtemp(prefix="pt_k5mini_")
    sdl = write_k5_scene(d, n_tris=c["n_tris"], seed=0, size=c["W"],
                         cornell_dir=os.path.join(REF, "objs"))
    colors, png = render_reference(c["W"], c["H"], c["spp"], c["bounces"], c["seed"], scene=sdl)
    np.savez_compressed(os.path.join(HERE, K5MINI_NAME), colors=colors, png=png, width=c["W"],
                        height=c["H"], spp=c["spp"], bounces=c["bounces"], seed=c["seed"],
                        n_tris=c["n_tris"])
    print("wrote", K5MINI_NAME, colors.shape, float(colors.min()), float(colors.max()))


# goldens of the test scenes built by tests/conftest.py (same writers, same
# seeds): (writer, scene seed, W, H, spp, bounces, render seed)
SCENE_GOLDENS = [
    ("quad_scene", 3, 12, 12, 3, 4, 3),         # parallelogram units (pt_path.h quad_m)
    ("multi_mesh_scene", 3, 10, 10, 2, 3, 3),   # two BVH objects first in scene order
]


def scene_golden_name(writer, sseed, W, H, spp, B, seed):
    return f"{writer}_{sseed}_render_{W}x{H}_s{spp}_b{B}_seed{seed}.npz"


def gen_scene_goldens():
    """The reference on the test scenes of tests/conftest.py (written into a
    temporary directory by the writers the tests use)."""
    import pathlib
    import tempfile
    sys.path.insert(0, os.path.dirname(HERE))
    import conftest
    for writer, sseed, W, H, spp, B, seed in SCENE_GOLDENS:
        d = pathlib.Path(tempfile.mkdtemp(prefix="pt_scene_"))
        getattr(conftest, writer)(d, sseed)
        colors, png = render_reference(W, H, spp, B, seed, scene=str(d / "scene.sdl"))
        name = scene_golden_name(writer, sseed, W, H, spp, B, seed)
        np.savez_compressed(os.path.join(HERE, name), colors=colors, png=png, width=W, height=H,
                            spp=spp, bounces=B, seed=seed, scene_seed=sseed)
        print("wrote", name, colors.shape, float(colors.min()), float(colors.max()))


def gen_scene():
    """Scene dump: what scene_reader.Scene produces (scene_reader.py:49-188)."""
    _, _, ref_scene = import_reference()
    with contextlib.redirect_stdout(io.StringIO()):
        sc = ref_scene.Scene(SCENE)
    out = {}
    tris, norms, areas, obj_id = [], [], [], []
    for i, o in enumerate(sc.objects + [{"geometry": sc.light_obj}]):
        g = o["geometry"]
        for t, n, a in zip(g.triangles, g.normals, g.areas):
            tris.append([list(v) for v in t])
            norms.append(list(n))
            areas.append(a)
            obj_id.append(i)
    out["triangles"] = np.array(tris, dtype=np.float64)
    out["normals"] = np.array(norms, dtype=np.float64)
    out["areas"] = np.array(areas, dtype=np.float64)
    out["obj_id"] = np.array(obj_id, dtype=np.int32)
    keys = ["red", "green", "blue", "ka", "kd", "ks", "kt", "n"]
    out["materials"] = np.array([[o[k] for k in keys] for o in sc.objects])
    out["eye"] = np.array(sc.eye, dtype=np.float64)
    out["ortho"] = np.array(sc.ortho, dtype=np.float64)
    out["size"] = np.array([sc.width, sc.height], dtype=np.int32)
    out["ambient"] = np.float64(sc.ambient)
    out["light_color"] = np.array(sc.light_color, dtype=np.float64)
    out["seed"] = np.int64(sc.seed)
    out["npaths"] = np.int64(sc.npaths)
    out["tonemapping"] = np.float64(sc.tonemapping)
    out["background"] = np.array(sc.background, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "scene_cornell.npz"), **out)
    print("wrote scene_cornell.npz", out["triangles"].shape)


def gen_kat():
    """Known-answer tests for the hot-path leaf functions."""
    ref_main, ref_utils, ref_scene = import_reference()
    with contextlib.redirect_stdout(io.StringIO()):
        sc = ref_scene.Scene(SCENE)
    rs = np.random.RandomState(1234)
    all_tris = [t for o in sc.objects for t in o["geometry"].triangles] + \
        list(sc.light_obj.triangles)
    out = {}

    # --- intersect(ray, triangle) utils.py:98-147 ---------------------------
    # random lines against the scene triangles plus random triangles
    rays_o, rays_d, tri_v, hit, pts = [], [], [], [], []

    def add_case(o, d, tri):
        try:
            p = ref_utils.intersect((np.array(o), np.array(d)), tri)
            h, pp = 1, np.asarray(p, dtype=np.float64)
        except ref_utils.NoIntersection:
            h, pp = 0, np.zeros(3)
        rays_o.append(o); rays_d.append(d)
        tri_v.append([list(v) for v in tri]); hit.append(h); pts.append(pp)

    for _ in range(1500):
        tri = all_tris[rs.randint(len(all_tris))]
        c = np.mean(np.array([list(v) for v in tri]), axis=0)
        o = rs.uniform(-4, 4, 3) + np.array([0, 0, -24.0])
        d = (c + rs.normal(0, 2.0, 3)) - o
        add_case(list(o), list(d), tri)
    for _ in range(500):
        tri = tuple(tuple(rs.uniform(-5, 5, 3)) for _ in range(3))
        o = rs.uniform(-5, 5, 3)
        d = rs.normal(0, 1, 3)
        add_case(list(o), list(d), tri)
    tri = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0))
    add_case([0.25, 0.25, 1.0], [0.0, 0.0, -1.0], tri)     # plain hit
    add_case([0.25, 0.25, 1.0], [0.0, 0.0, 1.0], tri)      # backward (line) hit
    add_case([0.5, 0.0, 1.0], [0.0, 0.0, -1.0], tri)       # on edge -> miss
    add_case([0.0, 0.0, 1.0], [0.0, 0.0, -1.0], tri)       # on vertex -> miss
    add_case([0.25, 0.25, 1.0], [1.0, 0.0, 0.0], tri)      # parallel -> miss
    add_case([0.25, 0.25, 1.0], [1.0, 0.0, -1e-6], tri)    # |dot|<=1e-5 -> miss
    add_case([0.25, 0.25, 1.0], [1.0, 0.0, -1e-3], tri)    # grazing but hit
    add_case([0.6, 0.6, 1.0], [0.0, 0.0, -1.0], tri)       # outside
    out["isect_o"] = np.array(rays_o, dtype=np.float64)
    out["isect_d"] = np.array(rays_d, dtype=np.float64)
    out["isect_tri"] = np.array(tri_v, dtype=np.float64)
    out["isect_hit"] = np.array(hit, dtype=np.int32)
    out["isect_p"] = np.array(pts, dtype=np.float64)

    # --- intersect_objects main.py:83-122 -----------------------------------
    io_o, io_d, io_hit, io_p, io_n, io_obj, io_light = [], [], [], [], [], [], []
    objs_plus = sc.objects + [{"geometry": sc.light_obj}]
    for k in range(600):
        if k % 3 == 0:
            o = np.array(sc.eye, dtype=np.float64)
            d = np.array([rs.uniform(-1, 1), rs.uniform(-1, 1), 0.0]) - o
        else:
            o = rs.uniform([-3.8, -3.8, -32.7], [3.8, 3.8, -16.6])
            d = rs.normal(0, 1, 3)
        r = ref_main.intersect_objects((o, d), sc.objects, sc.light_obj)
        io_o.append(o); io_d.append(d)
        if r is None:
            io_hit.append(0); io_p.append(np.zeros(3)); io_n.append(np.zeros(3))
            io_obj.append(-1); io_light.append(0)
        else:
            p, n, obj, is_light = r
            idx = [i for i, oo in enumerate(objs_plus)
                   if oo["geometry"] is obj["geometry"]][0]
            io_hit.append(1); io_p.append(np.asarray(p, dtype=np.float64))
            io_n.append(np.array(list(n))); io_obj.append(idx)
            io_light.append(int(is_light))
    out["io_o"] = np.array(io_o); out["io_d"] = np.array(io_d)
    out["io_hit"] = np.array(io_hit, dtype=np.int32)
    out["io_p"] = np.array(io_p); out["io_n"] = np.array(io_n)
    out["io_obj"] = np.array(io_obj, dtype=np.int32)
    out["io_light"] = np.array(io_light, dtype=np.int32)

    # --- rotate main.py:148-162 ---------------------------------------------
    rot_n, rot_v, rot_out = [], [], []
    normals = [list(n) for o in sc.objects for n in o["geometry"].normals]
    for k in range(200):
        n = normals[k % len(normals)] if k < 64 else list(
            rs.normal(0, 1, 3) / np.linalg.norm(rs.normal(0, 1, 3)))
        if k >= 64:
            n = rs.normal(0, 1, 3); n = list(n / np.linalg.norm(n))
        v = rs.normal(0, 1, 3)
        r = ref_main.rotate(np.array((0, 1, 0)),
                            np.arccos(np.dot(np.array((0, 1, 0)), n)), v)
        rot_n.append(n); rot_v.append(v); rot_out.append(r)
    out["rot_n"] = np.array(rot_n); out["rot_v"] = np.array(rot_v)
    out["rot_out"] = np.array(rot_out)

    # --- pick_random_triangle / sample_random_pt utils.py:21-46 --------------
    rng = KeyedRNG(0, None)
    ref_utils.uniform = rng.uniform
    ref_main.uniform = rng.uniform
    us = rs.uniform(0, 1, 400)
    picks = []
    for u in us:
        rng.forced = [float(u)]
        picks.append(ref_utils.pick_random_triangle(sc.light_obj.areas))
    out["pick_u"] = us
    out["pick_idx"] = np.array(picks, dtype=np.int32)
    srp_u = rs.uniform(0, 1, (200, 3))
    srp_p = []
    for u3 in srp_u:
        rng.forced = [float(x) for x in u3]
        srp_p.append(ref_utils.sample_random_pt(sc.light_obj.triangles[0]))
    out["srp_u"] = srp_u
    out["srp_p"] = np.array(srp_p)

    # --- compute_color / compute_shadow_rays main.py:23-80,142-145 -----------
    cc_p, cc_n, cc_obj, cc_u, cc_out = [], [], [], [], []
    for k in range(300):
        # shading points on random scene triangles
        oi = rs.randint(len(sc.objects))
        g = sc.objects[oi]["geometry"]
        ti = rs.randint(len(g.triangles))
        t = np.array([list(v) for v in g.triangles[ti]])
        a = rs.dirichlet([1, 1, 1])
        p = a @ t
        n = g.normals[ti]
        u12 = [float(x) for x in rs.uniform(0, 1, 12)]
        rng.forced = list(u12)
        col = ref_main.compute_color(sc, sc.objects[oi], p, n)
        assert not rng.forced
        cc_p.append(p); cc_n.append(list(n)); cc_obj.append(oi)
        cc_u.append(u12); cc_out.append(np.asarray(col, dtype=np.float64))
    out["cc_p"] = np.array(cc_p); out["cc_n"] = np.array(cc_n)
    out["cc_obj"] = np.array(cc_obj, dtype=np.int32)
    out["cc_u"] = np.array(cc_u); out["cc_out"] = np.array(cc_out)

    # --- make_screen_pts utils.py:64-69 and make_image utils.py:150-161 ------
    out["msp_5x3"] = np.array(ref_utils.make_screen_pts(-1, -1, 1, 1, 5, 3),
                              dtype=np.float64)
    cols = rs.uniform(-0.5, 2.0, (36, 3))
    im = ref_utils.make_image(-1, -1, 1, 1, 6, 6,
                              [(c, None) for c in cols])
    out["mi_cols"] = cols
    out["mi_png"] = np.asarray(im, dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "kat_cornell.npz"), **out)
    print("wrote kat_cornell.npz")


RENDER_CONFIGS = [
    (16, 16, 2, 3, 9),
    (64, 64, 1, 1, 9),      # BASELINE config 1 (-b 1 is main.py's default)
    (64, 64, 1, 4, 9),
    (24, 24, 3, 5, 12345),
    (6, 6, 32, 3, 21),      # several lanes per pixel on the GPU (split 4, xor-ordered sums)
]

if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "scene"):
        gen_scene()
    if what in ("all", "kat"):
        gen_kat()
    if what in ("all", "mesh"):
        gen_mesh()
        gen_mesh_kat()
    if what == "meshkat":
        gen_mesh_kat()
    if what in ("all", "k5mini"):
        gen_k5mini()
    if what in ("all", "scenes"):
        gen_scene_goldens()
    if what == "render":
        gen_render(*[int(x) for x in sys.argv[2:7]])
    if what == "all":
        for cfg in RENDER_CONFIGS:
            gen_render(*cfg)
