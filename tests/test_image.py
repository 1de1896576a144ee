"""Device image finalisation (pt_image_u8*) against
the reference's make_image (utils.py:150-161): bit-exact uint8.  The golden
PNG arrays were produced by the reference itself (tests/golden/gen_golden.py);
other cases compare with the numpy restatement utils.normalize_to_uint8,
which is the reference's own four lines."""
import warnings

import numpy as np
import pytest

from conftest import golden_renders
from pathtracerpython_amd.render import Renderer, image_u8
from pathtracerpython_amd.utils import normalize_to_uint8

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R(cornell):
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    r = Renderer(cornell)
    yield r
    r.close()


def _numpy_u8(a):
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        return normalize_to_uint8(a)


@pytest.mark.parametrize("name,g", golden_renders(), ids=[n for n, _ in golden_renders()])
def test_device_image_matches_reference_png(R, name, g):
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    img, fb = R.render_image(W, H, spp, B, seed, return_fb=True)
    assert img.dtype == np.uint8 and img.shape == (H, W, 3)
    assert np.array_equal(img, g["png"]), name
    assert np.array_equal(image_u8(fb), g["png"])


@pytest.mark.parametrize("which", ["mesh", "k5mini"])
def test_device_image_matches_reference_png_bvh(mesh_golden, k5mini_golden, which):
    """The BVH scenes' images (the edge-case mesh, the K5 generator at 1,000
    triangles): rendered and finalised on the device, bit-exact against the
    reference's make_image output of its own render."""
    sc, g = mesh_golden if which == "mesh" else k5mini_golden
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    with Renderer(sc) as r:
        img, fb = r.render_image(W, H, spp, B, seed, return_fb=True)
    assert np.array_equal(img, g["png"]), which
    assert np.array_equal(image_u8(fb), g["png"])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (64, 64), (509, 1031)])
def test_image_u8_matches_numpy(dtype, shape):
    rs = np.random.RandomState(sum(shape))
    a = (rs.normal(0.2, 0.7, shape + (3,)) ** 3).astype(dtype)   # negatives, wide range
    assert np.array_equal(image_u8(a), _numpy_u8(a))


def test_image_u8_edge_cases():
    const = np.full((8, 8, 3), 0.25)
    assert np.array_equal(image_u8(const), _numpy_u8(const))   # 0/0 -> 0
    a = np.linspace(-1, 1, 8 * 8 * 3).reshape(8, 8, 3)
    a[3, 4, 1] = np.nan
    assert np.array_equal(image_u8(a), _numpy_u8(a))           # NaN poisons min/max
    b = np.linspace(-1, 1, 8 * 8 * 3).reshape(8, 8, 3)
    b[0, 0, 0] = np.inf
    assert np.array_equal(image_u8(b), _numpy_u8(b))
    c = np.zeros((4, 4, 3))
    c[1, 1, 1] = 1e-300                                        # denormal-scale range
    assert np.array_equal(image_u8(c), _numpy_u8(c))
    for dt in (np.float64, np.float32):   # 63 elements: 15 vector groups + a 3-element tail
        d = np.linspace(-1, 1, 7 * 3 * 3).reshape(7, 3, 3).astype(dt)
        d[-1, -1, -1] = np.nan                                  # NaN in the scalar tail
        assert np.array_equal(image_u8(d), _numpy_u8(d)), dt
        e = np.linspace(-1, 1, 7 * 3 * 3).reshape(7, 3, 3).astype(dt)
        e[2, 1, 0] = -np.inf                                    # -inf minimum: inf - (-inf) paths
        assert np.array_equal(image_u8(e), _numpy_u8(e)), dt
        e[5, 2, 2] = np.inf
        assert np.array_equal(image_u8(e), _numpy_u8(e)), dt


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_image_u8_integer_boundaries(dtype):
    """Values whose scaled form lands on or next to an integer (k / 255 of the
    range, and their float neighbours): where the kernel's division-free form
    must defer to the exact division, since fl(fl(d / m) 255) truncates to
    k - 1 for some of them."""
    k = np.arange(256, dtype=np.float64)
    cols = []
    for lo, span in ((0.0, 255.0), (-0.37, 1.0), (3.0, 1e-3), (-2.5, 7.3)):
        v = (lo + span * k / 255.0).astype(dtype)
        cols += [v, np.nextafter(v, np.inf), np.nextafter(v, -np.inf)]
    a = np.concatenate(cols)
    a = a[: (a.size // 3) * 3].reshape(-1, 1, 3)
    for lo, span in ((0.0, 255.0), (-0.37, 1.0), (3.0, 1e-3), (-2.5, 7.3)):
        b = a.copy()
        b[0, 0, 0] = dtype(lo)
        b[-1, 0, 2] = dtype(lo + span)   # the range the k / 255 points sit on
        assert np.array_equal(image_u8(b), _numpy_u8(b)), (lo, span)


def test_image_u8_large_f32():
    rs = np.random.RandomState(5)
    a = rs.uniform(-3, 7, (2048, 2048, 3)).astype(np.float32)
    assert np.array_equal(image_u8(a), _numpy_u8(a))


def test_cli_png_matches_reference(tmp_path):
    """main.py's CLI (render -> device make_image -> PNG) on the 16x16 golden
    case writes the reference's own image."""
    from PIL import Image
    from conftest import CORNELL
    from pathtracerpython_amd import main as cli
    name, g = [x for x in golden_renders() if x[0].startswith("render_16x16")][0]
    W, H, spp, B, seed = (int(g[k]) for k in ("width", "height", "spp", "bounces", "seed"))
    out, raw = tmp_path / "o.png", tmp_path / "fb.npy"
    cli.main([CORNELL, "--out", str(out), "-r", str(spp), "-b", str(B), "--size", str(W), str(H),
              "--seed", str(seed), "--save-raw", str(raw)])
    assert np.array_equal(np.asarray(Image.open(out)), g["png"])
    assert np.load(raw).shape == (H, W, 3)
    # --chunk-spp 1 --checkpoint: the same frame (sample sums reordered: ~1e-16),
    # resumable; a rerun with the finished checkpoint renders nothing more
    raw2, ck = tmp_path / "fb2.npy", tmp_path / "ck.npz"
    args = [CORNELL, "-r", str(spp), "-b", str(B), "--size", str(W), str(H), "--seed", str(seed),
            "--save-raw", str(raw2), "--chunk-spp", "1", "--checkpoint", str(ck)]
    cli.main(args)
    assert np.abs(np.load(raw2) - np.load(raw)).max() <= 1e-14
    assert ck.exists()
    cli.main(args)
    assert np.abs(np.load(raw2) - np.load(raw)).max() <= 1e-14
