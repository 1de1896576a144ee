"""GPU parity tests: the HIP path (through the C-ABI) against the reference
goldens and the CPU oracle.  Tolerances: the framebuffer is compared in f64
(PT_FLAG_OUT_F64) at L-inf <= 1e-12 — the kernel keeps all path state in f64
and decides every intersection exactly (f32 filter + f64 fallback), so it
tracks the float64 reference to rounding; the default f32 framebuffer is
checked at <= 1e-6 (f32 output rounding).  BASELINE.json's bar is 1e-4.
At the full bench sizes the oracle checks pixel subsets, and size-independent
properties (hybrid == forced-f64 bitwise, band/sample-split consistency,
determinism) cover the whole image."""
import os

import numpy as np
import pytest

from conftest import (golden_renders, multi_mesh_scene, quad_scene, random_scene, scene_golden_ids,
                      scene_goldens, scene_of_golden)
from oracle import oracle
from pathtracerpython_amd import _native
from pathtracerpython_amd.pack import pack_scene
from pathtracerpython_amd.render import Renderer, from_list_order, to_list_order

pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def R(cornell):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    r = Renderer(cornell)
    yield r
    r.close()


def oracle_rows(packed, W, H, spp, B, seed, rows, flags=0):
    """Oracle colours of whole image rows iy (list), as framebuffer rows."""
    pix = np.array([ix * H + iy for iy in rows for ix in range(W)], dtype=np.int64)
    cols, _ = oracle.render(packed, W, H, spp, B, seed, flags=flags, pixels=pix)
    return cols.reshape(len(rows), W, 3)


# ------------------------------------------------------------ goldens --
@pytest.mark.parametrize("name,g", golden_renders(), ids=[n for n, _ in golden_renders()])
def test_matches_reference_goldens(R, packed, name, g):
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    fb, st = R.render(W, H, spp, B, seed, out_f64=True, stats=True)
    assert np.abs(to_list_order(fb) - g["colors"]).max() <= TOL
    fb32 = R.render(W, H, spp, B, seed)
    assert fb32.dtype == np.float32
    assert np.abs(to_list_order(fb32) - g["colors"]).max() <= 1e-6
    _, ost = oracle.render(packed, W, H, spp, B, seed)
    for k in ost:
        if k not in ("f64_fallbacks", "f64_rescans"):
            assert st[k] == ost[k], k


# --------------------------------------------------------- vs oracle --
@pytest.mark.parametrize("W,H,spp,B,seed,rr", [(96, 96, 4, 5, 3, False), (37, 19, 7, 4, 1, False),
                                               (1, 1, 3, 6, 2, False), (64, 64, 5, 8, 4, True),
                                               (50, 50, 2, 1, 9, False),
                                               # several lanes per pixel (split 8, 32, and 8
                                               # with a ragged 100 = 4 x 13 + 4 x 12 samples)
                                               (40, 24, 64, 3, 6, False), (16, 16, 256, 2, 7, True),
                                               (20, 12, 100, 3, 8, False)])
def test_matches_oracle(R, packed, W, H, spp, B, seed, rr):
    from pathtracerpython_amd._abi import PT_FLAG_RR
    fb = R.render(W, H, spp, B, seed, rr=rr, out_f64=True)
    ref, _ = oracle.render(packed, W, H, spp, B, seed, flags=PT_FLAG_RR if rr else 0)
    assert np.abs(to_list_order(fb) - ref).max() <= TOL


def test_mesh_golden(mesh_golden):
    """The BVH path against the reference itself: the edge-case mesh scene
    (68 triangles above the BVH threshold: duplicates, a shared-edge fan,
    triangles in the back wall's plane; tests/golden/mesh_scene.py) through
    the wavefront kernels (the default for BVH scenes) and the single kernel,
    f64 and f32 framebuffers."""
    sc, g = mesh_golden
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    with Renderer(sc) as r:
        wf = r.render(W, H, spp, B, seed, out_f64=True)
        mk = r.render(W, H, spp, B, seed, out_f64=True, megakernel=True)
        f32 = r.render(W, H, spp, B, seed)
    assert np.array_equal(wf, mk)
    assert np.abs(to_list_order(wf) - g["colors"]).max() <= TOL
    assert np.abs(to_list_order(f32) - g["colors"]).max() <= 1e-6


def test_k5mini_golden(k5mini_golden):
    """The K5 scene generator at 1,000 triangles against the reference's
    own render (wavefront and single kernel, f64 and f32 framebuffers)."""
    sc, g = k5mini_golden
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    with Renderer(sc) as r:
        wf = r.render(W, H, spp, B, seed, out_f64=True)
        mk = r.render(W, H, spp, B, seed, out_f64=True, megakernel=True)
        f32 = r.render(W, H, spp, B, seed)
    assert np.array_equal(wf, mk)
    assert np.abs(to_list_order(wf) - g["colors"]).max() <= TOL
    assert np.abs(to_list_order(f32) - g["colors"]).max() <= 1e-6


@pytest.mark.parametrize("name,writer,g", scene_goldens(), ids=scene_golden_ids())
def test_scene_goldens(tmp_path, name, writer, g):
    """The quad-unit and two-mesh test scenes against the reference's own
    renders (gen_golden.py scenes): default path (wavefront for the BVH
    scene), single kernel, forced f64, f32 framebuffer."""
    sc = scene_of_golden(tmp_path, writer, g)
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    with Renderer(sc) as r:
        fb = r.render(W, H, spp, B, seed, out_f64=True)
        assert np.array_equal(fb, r.render(W, H, spp, B, seed, out_f64=True, megakernel=True))
        assert np.array_equal(fb, r.render(W, H, spp, B, seed, out_f64=True, force_f64=True))
        f32 = r.render(W, H, spp, B, seed)
    assert np.abs(to_list_order(fb) - g["colors"]).max() <= TOL
    assert np.abs(to_list_order(f32) - g["colors"]).max() <= 1e-6


def test_zero_bounces_is_black(R):
    assert not R.render(8, 8, 2, 0, 1).any()


@pytest.fixture(scope="module")
def k2_oracle(packed):
    """The oracle's whole K2 frame (512x512, 64 spp, 4 bounces, seed 9) in
    framebuffer orientation (~4 s on 16 host threads)."""
    ref, _ = oracle.render(packed, 512, 512, 64, 4, 9, threads=oracle.host_threads())
    return from_list_order(ref, 512, 512)


def test_k2_full_size(R, k2_oracle):
    """BASELINE config 2 (512x512, 64 spp, 4 bounces), the bench frame: the
    oracle on EVERY pixel, f64 output <= 1e-12 and the f32 output as bench.py
    times it <= 1e-6 (no pixel above 1e-4, the north star's bar); hybrid ==
    forced-f64 bitwise on the whole image."""
    W = H = 512
    fb = R.render(W, H, 64, 4, 9, out_f64=True)
    assert np.abs(fb - k2_oracle).max() <= TOL
    ref = to_list_order(k2_oracle)
    err32 = np.abs(to_list_order(R.render(W, H, 64, 4, 9).astype(np.float64)) - ref)
    assert err32.max() <= 1e-6 and not (err32 > 1e-4).any()
    f64 = R.render(W, H, 64, 4, 9, out_f64=True, force_f64=True)
    assert np.array_equal(fb, f64)
    assert np.isfinite(fb).all()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_k2_bands_vs_oracle(R, k2_oracle, world):
    """One rank's interleaved band of an N-GPU strong-scaling K2 render (the
    bench's multi-GPU step): the band's lanes per pixel follow its size (8 /
    8 / 16 / 32 at N = 1 / 2 / 4 / 8, choose_split), so every band, first and
    last phase, is checked against the oracle's whole frame: f64 <= 1e-12,
    f32 <= 1e-6."""
    from pathtracerpython_amd.distributed import band_rows_of
    W = H = 512
    for phase in sorted({0, world - 1}):
        rows = band_rows_of(H, phase, world)
        ref = np.stack([k2_oracle[H - 1 - iy] for iy in rows])
        fb = R.render(W, H, 64, 4, 9, out_f64=True, row_step=world, row_phase=phase)
        assert np.abs(fb - ref).max() <= TOL
        f32 = R.render(W, H, 64, 4, 9, row_step=world, row_phase=phase)
        assert np.abs(f32 - ref).max() <= 1e-6


@pytest.mark.parametrize("dtype", ["float32", "float64"])
@pytest.mark.parametrize("H,W,world", [(512, 512, 8), (130, 37, 4), (23, 10, 3), (7, 5, 8), (9, 4, 1)])
def test_assemble_bands_device(dtype, H, W, world):
    """pt_assemble_bands_device (the frame assembly after the RCCL gather)
    equals the host assembly of distributed.assemble, ragged heights and
    16-B / 4-B row pieces included."""
    import torch
    from pathtracerpython_amd.distributed import assemble, assemble_bands_device, max_band_rows
    rs = np.random.RandomState(H * W + world)
    g = rs.rand(world, max_band_rows(H, world), W, 3).astype(dtype)
    out = torch.full((H, W, 3), -1.0, dtype=getattr(torch, dtype), device="cuda")
    assemble_bands_device(torch.from_numpy(g).cuda(), out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), assemble(list(g), H))


def test_k3_shape_with_rr(R, packed):
    """BASELINE config 3 shape (1024x1024, 8 bounces + RR) at 4 spp: oracle
    on 2 rows, bitwise hybrid == f64."""
    W = H = 1024
    fb = R.render(W, H, 4, 8, 5, rr=True, out_f64=True)
    from pathtracerpython_amd._abi import PT_FLAG_RR
    ref = oracle_rows(packed, W, H, 4, 8, 5, [3, 700], flags=PT_FLAG_RR)
    got = np.stack([fb[H - 1 - iy] for iy in (3, 700)])
    assert np.abs(got - ref).max() <= TOL
    assert np.array_equal(fb, R.render(W, H, 4, 8, 5, rr=True, out_f64=True, force_f64=True))


def test_large_image_subset(R, packed):
    """4096x4096 (BASELINE config 4 size) at 1 spp, 2 bounces: rows vs oracle."""
    W = H = 4096
    fb = R.render(W, H, 1, 2, 9)
    rows = [0, 2048, 4095]
    ref = oracle_rows(packed, W, H, 1, 2, 9, rows)
    got = np.stack([fb[H - 1 - iy] for iy in rows]).astype(np.float64)
    assert np.abs(got - ref).max() <= 1e-6


# ----------------------------------------------- size-independent checks --
def test_deterministic_and_seeded(R):
    a = R.render(128, 128, 8, 4, 1)
    b = R.render(128, 128, 8, 4, 1)
    c = R.render(128, 128, 8, 4, 2)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, c)


def test_interleaved_bands_assemble(R):
    """Small images run at the lane cap (min(64, spp) lanes per pixel), full
    frame and bands alike, so their bands assemble to the full frame bit for
    bit."""
    from pathtracerpython_amd.distributed import assemble, max_band_rows
    W, H, world = 160, 130, 4
    full = R.render(W, H, 32, 4, 7, out_f64=True)   # 32 lanes per pixel
    tiles = []
    for r in range(world):
        t = R.render(W, H, 32, 4, 7, out_f64=True, row_step=world, row_phase=r)
        pad = np.zeros((max_band_rows(H, world), W, 3))
        pad[:t.shape[0]] = t
        tiles.append(pad)
    assert np.array_equal(assemble(tiles, H), full)


def test_tail_rows_ragged(R, packed):
    """The single kernel's last rows run at 8x lanes per pixel (launch drain,
    DESIGN.md §4).  999 x 300 at 64 spp runs 16 lanes per pixel, and the tail
    (rows iy >= 281) starts at lane 281 x 999 x 16 = 4,491,504, padded to a wave
    boundary: rows below, at and above the threshold vs the oracle; a 3-way
    interleaved split (99,900 pixels per band: 16 lanes per pixel, their own
    tails) assembles to within rounding of the full frame."""
    from pathtracerpython_amd.distributed import assemble, max_band_rows
    W, H, spp, B, seed = 999, 300, 64, 3, 11
    fb = R.render(W, H, spp, B, seed, out_f64=True)
    rows = [0, 150, 279, 280, 281, 282, 299]
    ref = oracle_rows(packed, W, H, spp, B, seed, rows)
    assert np.abs(np.stack([fb[H - 1 - iy] for iy in rows]) - ref).max() <= TOL
    world = 3
    tiles = []
    for r in range(world):
        t = R.render(W, H, spp, B, seed, out_f64=True, row_step=world, row_phase=r)
        pad = np.zeros((max_band_rows(H, world), W, 3))
        pad[:t.shape[0]] = t
        tiles.append(pad)
    assert np.abs(assemble(tiles, H) - fb).max() <= 1e-13


def test_contiguous_band(R):
    full = R.render(64, 64, 2, 4, 3)
    band = R.render(64, 64, 2, 4, 3, row_begin=10, row_end=30)
    assert np.array_equal(band, full[64 - 30:64 - 10])


def test_sample_split_linearity(R):
    full = R.render(100, 100, 8, 4, 6, out_f64=True)
    a = R.render(100, 100, 4, 4, 6, out_f64=True, sample_begin=0)
    b = R.render(100, 100, 4, 4, 6, out_f64=True, sample_begin=4)
    assert np.abs((a + b) / 2 - full).max() <= 1e-14


def test_progressive_chunks_and_resume(R, tmp_path):
    """progressive.py: 10 spp as chunks of 4 (sample_begin 0, 4, 8) equals
    the one-launch frame to the sum reordering; an interrupted run resumed
    from its checkpoint is bit-identical to the uninterrupted chunked run."""
    from pathtracerpython_amd.progressive import render_progressive
    full = R.render(64, 64, 10, 4, 6, out_f64=True)
    fb = render_progressive(R, 64, 64, 10, 4, 6, chunk_spp=4)
    assert np.abs(fb - full).max() <= 1e-14
    ck = tmp_path / "k.npz"
    assert render_progressive(R, 64, 64, 10, 4, 6, chunk_spp=4, checkpoint=ck,
                              max_chunks=2) is None
    assert np.array_equal(render_progressive(R, 64, 64, 10, 4, 6, chunk_spp=4, checkpoint=ck), fb)


def test_random_mesh_scene(tmp_path):
    sc = random_scene(tmp_path, 300, 21)
    pk = pack_scene(sc)
    with Renderer(sc) as r:
        fb = r.render(48, 48, 4, 5, 8, out_f64=True)
        assert np.array_equal(fb, r.render(48, 48, 4, 5, 8, out_f64=True, force_f64=True))
    ref, _ = oracle.render(pk, 48, 48, 4, 5, 8)
    assert np.abs(to_list_order(fb) - ref).max() <= TOL
    with Renderer(sc) as r:   # wavefront (default for BVH scenes) == single kernel
        assert np.array_equal(fb, r.render(48, 48, 4, 5, 8, out_f64=True, megakernel=True))


@pytest.mark.parametrize("seed", [3, 8])
def test_quad_units_scene(tmp_path, seed):
    """Parallelogram units in every vertex labelling, skewed coplanar pairs
    and single triangles (the render loop's unit form, pt_path.h quad_m):
    hybrid == forced f64 bit for bit, and the oracle to rounding."""
    sc = quad_scene(tmp_path, seed)
    pk = pack_scene(sc)
    with Renderer(sc) as r:
        fb = r.render(64, 64, 8, 5, seed, out_f64=True)
        assert np.array_equal(fb, r.render(64, 64, 8, 5, seed, out_f64=True, force_f64=True))
    ref, _ = oracle.render(pk, 64, 64, 8, 5, seed)
    assert np.abs(to_list_order(fb) - ref).max() <= TOL


@pytest.mark.parametrize("seed", [3, 4])
def test_two_meshes_first_in_scene_order(tmp_path, seed):
    """Two BVH objects ahead of a small object and the walls in scene order
    (the leaked colour of main.py:70 across BVH objects): wavefront ==
    single kernel == forced f64, and the oracle to rounding."""
    sc = multi_mesh_scene(tmp_path, seed)
    pk = pack_scene(sc)
    with Renderer(sc) as r:
        wf = r.render(40, 40, 3, 4, seed, out_f64=True)
        assert np.array_equal(wf, r.render(40, 40, 3, 4, seed, out_f64=True, megakernel=True))
        assert np.array_equal(wf, r.render(40, 40, 3, 4, seed, out_f64=True, force_f64=True))
    ref, _ = oracle.render(pk, 40, 40, 3, 4, seed)
    assert np.abs(to_list_order(wf) - ref).max() <= TOL


@pytest.fixture(scope="module")
def k5small(tmp_path_factory):
    """The K5 recipe (synth.py) with 20k triangles: a BVH scene."""
    from pathtracerpython_amd import scene_reader
    from pathtracerpython_amd.synth import write_k5_scene
    scene_reader.VERBOSE = False
    d = tmp_path_factory.mktemp("k5")
    return scene_reader.Scene(write_k5_scene(str(d), n_tris=20_000, seed=0, size=64))


@pytest.mark.parametrize("W,spp,B,rr", [(64, 4, 4, False), (48, 3, 6, True), (40, 1, 1, False),
                                        (100, 2, 3, False)])
def test_wavefront_k5_equals_single_kernel(k5small, W, spp, B, rr):
    """BVH scenes render through the wavefront kernels (shade + persistent
    walk kernels); the framebuffer must equal the single kernel's bit for bit
    (which equals the forced-f64 render), and the oracle to rounding."""
    pk = pack_scene(k5small)
    with Renderer(k5small) as r:
        wf = r.render(W, W, spp, B, 9, rr=rr, out_f64=True)
        mk = r.render(W, W, spp, B, 9, rr=rr, out_f64=True, megakernel=True)
        assert np.array_equal(wf, mk)
        if W <= 48:
            assert np.array_equal(wf, r.render(W, W, spp, B, 9, rr=rr, out_f64=True,
                                               force_f64=True))
        # a band and a sample slice of the same image (kernel reuse, odd sizes)
        band = r.render(W, W, spp, B, 9, rr=rr, out_f64=True, row_begin=7, row_end=W - 3)
        assert np.array_equal(band, wf[3:W - 7])
    rows = [0, W // 2, W - 1]
    pix = np.array([ix * W + iy for iy in rows for ix in range(0, W, 3)], dtype=np.int64)
    ref, _ = oracle.render(pk, W, W, spp, B, 9, flags=1 if rr else 0, pixels=pix)
    got = np.array([wf[W - 1 - (k % W), k // W] for k in pix])
    assert np.abs(got - ref).max() <= TOL


# ------------------------------------------- batched Pool callables --
def test_intersect_objects_kat(R, packed, kat):
    rays = np.concatenate([kat["io_o"], kat["io_d"]], axis=1)
    tri, P = R.intersect_objects(rays)
    hit = tri >= 0
    assert np.array_equal(hit.astype(np.int32), kat["io_hit"])
    obj = np.where(hit, packed.tri_obj[np.maximum(tri, 0)], -1)
    assert np.array_equal(obj, kat["io_obj"])
    assert np.array_equal((tri >= packed.n_obj_tri).astype(np.int32), kat["io_light"])
    assert np.abs(P[hit] - kat["io_p"][hit]).max() <= 1e-11


def test_mesh_kat_intersect_objects(mesh_golden):
    """The batched closest-hit API over a BVH object (pt_intersect_objects)
    against the reference's intersect_objects on the edge-case mesh scene
    (tests/golden/kat_mesh.npz): origins on the mesh's triangles, exact
    duplicates, triangles in the back wall's plane."""
    from pathtracerpython_amd.pack import pack_scene
    import os
    from conftest import GOLDEN
    sc, _ = mesh_golden
    pk = pack_scene(sc)
    k = np.load(os.path.join(GOLDEN, "kat_mesh.npz"))
    with Renderer(sc) as r:
        tri, P = r.intersect_objects(np.concatenate([k["io_o"], k["io_d"]], axis=1))
    hit = tri >= 0
    assert np.array_equal(hit.astype(np.int32), k["io_hit"])
    assert np.array_equal(np.where(hit, pk.tri_obj[np.maximum(tri, 0)], -1), k["io_obj"])
    assert np.array_equal((tri >= pk.n_obj_tri).astype(np.int32), k["io_light"])
    assert np.abs(P[hit] - k["io_p"][hit]).max() <= 1e-11


def test_mesh_kat_compute_color(mesh_golden):
    """The batched shading API over a scene with a BVH object
    (pt_compute_color: shadow rays through the BVH walks) against the
    reference's compute_color on the edge-case mesh scene."""
    import os
    from conftest import GOLDEN
    sc, _ = mesh_golden
    k = np.load(os.path.join(GOLDEN, "kat_mesh.npz"))
    with Renderer(sc) as r:
        out = r.compute_color(k["cc_obj"], k["cc_p"], k["cc_n"], k["cc_u"])
    assert np.abs(out - k["cc_out"]).max() <= TOL


def test_intersect_objects_outside_box(R, packed):
    rs = np.random.RandomState(0)
    o = rs.uniform(-100, 100, (500, 3))
    d = rs.normal(0, 1, (500, 3))
    rays = np.concatenate([o, d], axis=1)
    tri, P = R.intersect_objects(rays)
    otri, oP = oracle.intersect_objects(packed, rays)
    assert np.array_equal(tri, otri)
    assert np.abs(P - oP).max() <= 1e-9


def _filter_boxes(pk):
    """The two origin boxes of the f32 filter (pt_prepare.h prepare_scene):
    (centre, half width) of the triangles' cube and of the cube with the eye."""
    v = pk.tri_v.reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    cs, xs = 0.5 * (lo + hi), 0.5 * (hi - lo).max()
    lo, hi = np.minimum(lo, pk.eye), np.maximum(hi, pk.eye)
    return cs, xs, 0.5 * (lo + hi), 0.5 * (hi - lo).max()


def test_intersect_objects_bvh_surface_box_only(tmp_path):
    """BVH scene with the eye far off-axis, origins inside the triangles'
    cube but outside the cube with the eye: the BVH walk's error bounds
    assume the latter, so these queries must not take the f32 filter's BVH
    path (k_intersect needs in_a when the scene has a BVH).
    Against the oracle, lines aimed at the meshes' triangles and random."""
    import shutil
    from pathtracerpython_amd import scene_reader
    from conftest import CORNELL
    src = os.path.dirname(CORNELL)
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp_path / f)
    # a BVH-sized mesh in front of the room's open side (z > -16.6), so lines
    # from beside the room reach it without crossing a wall
    rs = np.random.RandomState(11)
    c = rs.uniform([-3.5, -3.5, -15.5], [3.5, 3.5, -9.0], (150, 3))
    lines = ["v %.9f %.9f %.9f" % tuple(c[i] + rs.normal(0, 0.5, 3)) for i in range(150) for _ in range(3)]
    lines += ["f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3) for i in range(150)]
    (tmp_path / "front.obj").write_text("\n".join(lines) + "\n")
    sdl = open(CORNELL).read().replace(
        "output cornell.pnm", "object front.obj 0.2 0.5 0.9 0.3 0.6 0.4 0 3\noutput cornell.pnm")
    (tmp_path / "scene.sdl").write_text(sdl)
    scene_reader.VERBOSE = False
    sc = scene_reader.Scene(str(tmp_path / "scene.sdl"))
    sc.eye = [40.0, 0.0, -13.0]   # far off-axis: the cube with the eye shifts right
    pk = pack_scene(sc)
    mesh = int(pk.tri_obj.max()) - 1   # the last object (the light is n_obj)
    cs, xs, ca, xa = _filter_boxes(pk)
    rs = np.random.RandomState(5)
    o = rs.uniform(cs - 0.99 * xs, cs + 0.99 * xs, (20000, 3))
    o = o[(np.abs(o - ca) > 1.01 * xa).any(axis=1)][:600]
    assert len(o) == 600
    tgt = pk.tri_v[rs.choice(np.flatnonzero(pk.tri_obj == mesh), len(o))]
    w = rs.dirichlet((1, 1, 1), len(o))
    d = np.einsum("ni,nij->nj", w, tgt) - o
    d[::3] = rs.normal(0, 1, (len(d[::3]), 3))
    rays = np.concatenate([o, d], axis=1)
    with Renderer(sc) as r:
        tri, P = r.intersect_objects(rays)
    otri, oP = oracle.intersect_objects(pk, rays)
    assert (pk.tri_obj[otri[otri >= 0]] == mesh).sum() > 200   # most hits on the BVH mesh
    assert np.array_equal(tri, otri)
    assert np.abs(P - oP).max() <= 1e-9


def test_compute_color_kat(R, kat):
    out = R.compute_color(kat["cc_obj"], kat["cc_p"], kat["cc_n"], kat["cc_u"])
    assert np.abs(out - kat["cc_out"]).max() <= TOL


# ------------------------------------------------------------- errors --
@pytest.mark.parametrize("kw", [dict(spp=0), dict(bounces=-1), dict(row_step=0),
                                dict(row_step=2, row_phase=2), dict(width=0)])
def test_invalid_params_raise(R, kw):
    args = dict(width=8, height=8, spp=1, bounces=1)
    args.update(kw)
    with pytest.raises(_native.NativeError):
        R.render(**args)


def test_kernel_timing_and_distributed_world1(R):
    import torch
    from pathtracerpython_amd.distributed import render_distributed
    fb = render_distributed(R, 64, 48, spp=2, bounces=3, seed=1)
    assert R.last_kernel_ms() > 0
    assert np.array_equal(fb, R.render(64, 48, 2, 3, 1))
    assert np.array_equal(render_distributed(R, 64, 48, spp=2, bounces=3, seed=1, transport="host"), fb)
    assert torch.cuda.is_available()


def test_from_list_order_matches_golden_png(R):
    from pathtracerpython_amd.utils import framebuffer_to_image
    name, g = golden_renders()[0]
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    fb = R.render(W, H, spp, B, seed, out_f64=True)
    assert np.array_equal(np.asarray(framebuffer_to_image(fb)), g["png"])
    assert np.abs(fb - from_list_order(g["colors"], W, H)).max() <= TOL


# ------------------------------------------- one-process multi-device --
def test_render_function_devices(cornell):
    """render(..., devices=[0, 0]): the module-level render over several
    handles (pt_render_multi) gives render()'s frame (at the lane cap: bit
    for bit)."""
    from pathtracerpython_amd.render import render
    one = render(cornell, 40, 30, 16, 3, 5)
    assert np.array_equal(render(cornell, 40, 30, 16, 3, 5, devices=[0, 0]), one)
    assert np.array_equal(render(cornell, 40, 30, 16, 3, 5, devices=[0]), one)


def test_render_multi_bands_bitwise(cornell):
    """pt_render_multi deals the rows out interleaved over its handles and
    copies each band into its rows of the host frame: bit-identical to one
    render (here several handles on device 0, which exercises the dealing,
    the strided copies and the concurrency of the handles)."""
    from pathtracerpython_amd.render import MultiRenderer
    W, H = 70, 53
    with Renderer(cornell) as r:
        ref, st = r.render(W, H, 16, 4, 3, out_f64=True, stats=True)
        ref32 = r.render(W, H, 16, 4, 3)
    for n in (1, 2, 3, 5):
        with MultiRenderer(cornell, [0] * n) as m:
            assert np.array_equal(m.render(W, H, 16, 4, 3, out_f64=True), ref)
            assert np.array_equal(m.render(W, H, 16, 4, 3), ref32)
    with MultiRenderer(cornell, [0, 0]) as m:
        band = m.render(W, H, 16, 4, 3, out_f64=True, row_begin=5, row_end=40)
        assert np.array_equal(band, ref[H - 40:H - 5])
        _, mst = m.render(W, H, 16, 4, 3, out_f64=True, stats=True)
        # the reference-semantics counters add up over the bands (the f64
        # fallback counts are diagnostics that depend on wave composition)
        diag = ("f64_fallbacks", "f64_rescans")
        assert {k: v for k, v in mst.items() if k not in diag} == \
            {k: v for k, v in st.items() if k not in diag}


def test_wavefront_walk_counts_and_times(k5small):
    """PT_FLAG_WALK_COUNT (counting walk kernels) and PT_FLAG_KERNEL_TIMES
    leave the framebuffer unchanged and report plausible work (queries, node
    visits and leaf units all present, one walk launch per shade launch but
    the last)."""
    with Renderer(k5small) as r:
        ref = r.render(64, 64, 4, 4, 9, out_f64=True)
        fb, st = r.render_params(r.params(64, 64, 4, 4, 9, out_f64=True, walk_count=True),
                                 stats=True)
        assert np.array_equal(fb, ref)
        assert st["shadow_queries"] > 0 and st["closest_queries"] > 0
        assert st["shadow_node_visits"] > 0 and st["closest_node_visits"] > 0
        assert st["closest_leaf_units"] > 0 and st["shadow_leaf_units"] > 0
        fb, tt = r.render_params(r.params(64, 64, 4, 4, 9, out_f64=True, kernel_times=True),
                                 stats=True)
        assert np.array_equal(fb, ref)
        assert tt["shade_launches"] == tt["shadow_launches"] + 1 == tt["closest_launches"] + 1
        assert tt["shade_ms"] > 0 and tt["shadow_ms"] > 0 and tt["closest_ms"] > 0
        # (C-ABI v7) the shadow list's sort, its own interval: every walk step but the first
        assert tt["sort_launches"] == tt["shadow_launches"] - 1 and tt["sort_ms"] > 0


def test_render_multi_lanes_contract(cornell):
    """at the K2 frame an 8-way split's bands run more lanes per
    pixel than the whole frame (choose_split), so pt_render_multi with the
    default lanes_per_pixel = 0 agrees with one render to rounding only;
    with a fixed lanes_per_pixel both are the same bit for bit."""
    from pathtracerpython_amd.render import MultiRenderer
    W = H = 512
    with Renderer(cornell) as r:
        ref = r.render(W, H, 64, 4, 9, out_f64=True)
        ref8 = r.render_params(r.params(W, H, 64, 4, 9, out_f64=True, lanes_per_pixel=8))
        ref16 = r.render_params(r.params(W, H, 64, 4, 9, out_f64=True, lanes_per_pixel=16))
        ref32 = r.render_params(r.params(W, H, 64, 4, 9, out_f64=True, lanes_per_pixel=32))
    # the whole K2 frame picks 16 lanes per pixel itself (4 samples per lane, round 6)
    assert np.array_equal(ref16, ref)
    assert np.abs(ref8 - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())
    with MultiRenderer(cornell, [0] * 8) as m:
        auto = m.render(W, H, 64, 4, 9, out_f64=True)
        assert np.abs(auto - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())
        assert np.array_equal(m.render(W, H, 64, 4, 9, out_f64=True, lanes_per_pixel=8), ref8)
        assert np.array_equal(m.render(W, H, 64, 4, 9, out_f64=True, lanes_per_pixel=32), ref32)


def test_render_multi_error_drains_launched_devices(cornell):
    """a failure while dealing band i (fault injected after
    bands 0..i-1 were launched, pt_test_fault_inject) returns the error after
    draining those devices; the same handles then render bit-exactly."""
    from pathtracerpython_amd.render import MultiRenderer
    W = H = 256
    with Renderer(cornell) as r:
        ref = r.render_params(r.params(W, H, 64, 4, 5, lanes_per_pixel=16))
    lib = _native.lib()
    with MultiRenderer(cornell, [0] * 4) as m:
        for i in (1, 3):
            lib.pt_test_fault_inject(i)
            try:
                with pytest.raises(_native.NativeError, match=f"device {i}: fault injected"):
                    m.render(W, H, 64, 4, 5, lanes_per_pixel=16)
            finally:
                lib.pt_test_fault_inject(-1)
            assert np.array_equal(m.render(W, H, 64, 4, 5, lanes_per_pixel=16), ref)


def test_render_multi_rejects_mixed_scenes(cornell, tmp_path):
    from pathtracerpython_amd.render import MultiRenderer
    m = MultiRenderer(cornell, [0, 0])
    try:
        other = Renderer(quad_scene(tmp_path, 3))
        m.renderers.append(other)
        with pytest.raises(_native.NativeError, match="another scene"):
            m.render(16, 16, 2, 2, 1)
    finally:
        m.close()


def test_out_row_stride_writes_band_rows_into_a_frame(cornell):
    """out_row_stride: each rank's interleaved band written straight into its
    rows of one frame (device memory here) assembles the whole frame."""
    import torch
    W, H, world = 96, 61, 4
    with Renderer(cornell) as r:
        ref = r.render_params(r.params(W, H, 16, 3, 2, lanes_per_pixel=4))
        frame = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for rank in range(world):
            iy_top = max(range(rank, H, world))
            p = r.params(W, H, 16, 3, 2, row_step=world, row_phase=rank, lanes_per_pixel=4,
                         out_row_stride=world * W * 3)
            r.render_device(p, frame[H - 1 - iy_top].data_ptr(), s)
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy(), ref)
        # pt_render's host copy honours the stride too
        out = np.full((H, 2 * W, 3), -1.0, dtype=np.float32)
        p = r.params(W, H, 16, 3, 2, lanes_per_pixel=4)
        p.out_row_stride = 2 * W * 3
        import ctypes as C
        _native.check(_native.lib().pt_render(r._h, C.byref(p), C.c_void_p(out.ctypes.data), None),
                      "pt_render")
        assert np.array_equal(out[:, :W], ref) and (out[:, W:] == -1.0).all()


@pytest.mark.parametrize("world", [1, 3])
def test_host_frame_bands_in_one_process(cornell, world):
    """HostFrame (distributed.py): each rank's band rendered straight into
    the page-locked shared frame, pt_signal / pt_wait_flags, slot rotation —
    here every rank's handle in one process on device 0.  The frame equals
    one render bit for bit (fixed lanes per pixel), step after step."""
    from pathtracerpython_amd.distributed import HostFrame
    import torch
    W, H = 128, 77
    s = torch.cuda.current_stream().cuda_stream
    with Renderer(cornell) as r:
        ref = r.render_params(r.params(W, H, 32, 4, 7, lanes_per_pixel=8))
        name = HostFrame.new_name()
        frames = [HostFrame(H, W, world, 0, name, create=True)]
        frames += [HostFrame(H, W, world, k, name) for k in range(1, world)]
        try:
            for step in range(5):
                for k, hf in enumerate(frames):
                    p = r.params(W, H, 32, 4, 7, row_step=world, row_phase=k, lanes_per_pixel=8)
                    hf.render(r, p, step, s, timeout_s=60)
                got = frames[0].wait(step, timeout_s=60)
                assert np.array_equal(got, ref), step
                del got
                frames[0].release(step)
        finally:
            for hf in frames[::-1]:
                hf.close()


def test_host_frame_two_rank_processes(cornell, tmp_path):
    """Two rank processes on device 0 (gloo rendezvous) render their bands
    straight into one shared page-locked frame, five steps with a new seed
    each (slot rotation); rank 0's frames equal one render each, bit for bit
    (lanes_per_pixel 4 everywhere)."""
    from conftest import ROOT
    from pathtracerpython_amd.launch import spawn_ranks
    W, H, spp, B, seed, steps = 64, 37, 16, 4, 11, 5
    out = str(tmp_path / "frames.npy")
    rc = spawn_ranks(2, [os.path.join(ROOT, "tests", "rank_worker_hostframe.py"), out, str(W), str(H),
                         str(spp), str(B), str(seed), str(steps), "gpu"])
    assert rc == 0
    got = np.load(out)
    with Renderer(cornell) as r:
        for s in range(steps):
            ref = r.render_params(r.params(W, H, spp, B, seed + s, lanes_per_pixel=4))
            assert np.array_equal(got[s], ref), s


def test_bench_host_frame_path_two_ranks(tmp_path):
    """bench.py's N > 1 host-frame path on one GPU (PT_BENCH_REHEARSE: two
    self-spawned ranks on device 0 over gloo): the line is printed, and the
    frame rank 0 read from host memory matches the oracle over every pixel."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, PT_BENCH_REHEARSE="1")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6",
                          "--warmup", "2", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    line = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["frame"] == "host"
    assert line["linf_checked"] == "all 262144 pixels" and line["pixels_over"]["1e-6"] == 0
    legs = line["frame_modes"]["host"]["legs_ms"]
    assert legs["band_kernel_max"] >= legs["band_kernel_min"] > 0
    # which GPU each rank ran on — here both on device 0, which
    # only the rehearsal lets through (ranks_share_a_gpu names the bus id)
    rk = line["ranks"]
    assert [r["rank"] for r in rk] == [0, 1] and all(r["local_device"] == 0 for r in rk)
    assert rk[0]["pci_bus_id"] == rk[1]["pci_bus_id"] and len(rk[0]["pci_bus_id"]) == 10
    assert line["ranks_share_a_gpu"] == [rk[0]["pci_bus_id"]]
    assert all(r["band_kernel_ms"] > 0 for r in rk)
    assert max(r["band_kernel_ms"] for r in rk) == pytest.approx(legs["band_kernel_max"], abs=2e-4)


def test_bench_refuses_ranks_sharing_a_gpu():
    """Two ranks on one device without PT_BENCH_REHEARSE (PT_BENCH_FORCE_DEVICE0,
    the rank-to-device mistake made on purpose): no line, nonzero status."""
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, PT_BENCH_FORCE_DEVICE0="1")
    env.pop("PT_BENCH_REHEARSE", None)
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "1", "--no-cpu-baseline", "--no-check", "--no-secondary"], env=env,
                         capture_output=True, text=True, timeout=240)
    assert res.returncode != 0
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert "ranks share a GPU" in res.stderr


def test_bench_line_names_its_gpu():
    """The N = 1 line: one rank record, and the device-frame leg's RCCL world
    (1: no gather)."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--no-cpu-baseline", "--no-check"], capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    line = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert len(line["ranks"]) == 1 and line["ranks"][0]["rank"] == 0 and line["ranks_share_a_gpu"] is None
    assert line["frame_modes"]["device"]["rccl_world"] == 1


@pytest.mark.parametrize("inject", ["raise:1", "hang:1"])
def test_bench_headline_survives_a_failing_secondary_leg(inject):
    """VERDICT r04 #1 through bench.py itself (two rank processes on device 0,
    PT_BENCH_REHEARSE): the secondary leg fails or never returns on rank 1,
    and the job still prints ONE line with the host-frame headline — value,
    legs, the whole frame against the oracle — and the leg's error, status 0."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, PT_BENCH_REHEARSE="1", PT_BENCH_INJECT_DEVICE_LEG=inject,
               PT_BENCH_LEG_TIMEOUT_S="10")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                          "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, res.stdout[-2000:]   # the one line, nothing else on stdout
    lines = [json.loads(lines[0])]
    line = lines[0]
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["config"]["frame"] == "host"
    assert line["frame_modes"]["host"]["legs_ms"]["band_kernel_max"] > 0
    assert line["linf_checked"] == "all 262144 pixels" and line["pixels_over"]["1e-6"] == 0
    err = line["frame_modes"]["device"]["error"]
    assert ("rank 1: RuntimeError: injected" in err) if inject.startswith("raise") else \
        ("no outcome within 10 s" in err), err


def test_rccl_gather_on_the_device(cornell, tmp_path):
    """The device-frame transport's RCCL gather, run on the hardware as
    bench.py runs it (gloo control plane + an nccl group for the gather,
    tests/rank_worker_rccl.py).  A one-GPU box allows world 1 only; the
    assembled frame equals a direct render bit for bit."""
    from conftest import ROOT
    from pathtracerpython_amd.launch import spawn_ranks
    out = str(tmp_path / "frame.npy")
    assert spawn_ranks(1, [os.path.join(ROOT, "tests", "rank_worker_rccl.py"), out]) == 0
    with Renderer(cornell) as r:
        ref = r.render(64, 64, 4, 3, 9)
    assert np.array_equal(np.load(out), ref)
