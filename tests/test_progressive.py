"""Chunked, resumable renders (pathtracerpython_amd/progressive.py): the
checkpoint / resume host logic, against a stand-in renderer whose sample s
of a pixel is a known function of (s, pixel) — the keyed-RNG property the
HIP path has (the GPU case is tests/test_gpu.py::test_progressive_*)."""
import json

import numpy as np
import pytest

from pathtracerpython_amd._abi import make_params
from pathtracerpython_amd.progressive import Checkpoint, render_progressive, scene_fingerprint


class _Packed:
    def __init__(self, salt=0.0):
        self.tri_v = np.arange(18, dtype=np.float64).reshape(2, 3, 3) + salt
        self.tri_n = np.ones((2, 3))
        self.tri_area = np.ones(2)
        self.tri_obj = np.zeros(2, dtype=np.int32)
        self.mat = np.ones((1, 8))
        self.eye = np.zeros(3)
        self.ortho = np.array([-1.0, -1.0, 1.0, 1.0])
        self.ambient = 0.5
        self.light_rgb = np.ones(3)


class FakeRenderer:
    """render(...) = mean over samples [sample_begin, +spp) of
    sample(s) = sin(s * 0.37 + pixel) (per channel offset)."""

    def __init__(self, salt=0.0):
        self.packed = _Packed(salt)
        self.launches = []

    def params(self, width, height, spp, bounces, seed, rr, rr_depth, out_f64=False, **kw):
        return make_params(width, height, spp, bounces, 0 if seed is None else seed, 0, rr_depth)

    @staticmethod
    def sample(s, H, W):
        pix = np.arange(H * W * 3, dtype=np.float64).reshape(H, W, 3)
        return np.sin(s * 0.37 + pix * 0.01)

    def render(self, W, H, spp, bounces, seed, rr, rr_depth, out_f64=False, sample_begin=0):
        self.launches.append((sample_begin, spp))
        return sum(self.sample(s, H, W) for s in range(sample_begin, sample_begin + spp)) / spp


def test_chunks_cover_every_sample_once():
    r = FakeRenderer()
    fb = render_progressive(r, 5, 4, spp=11, bounces=2, chunk_spp=4)
    assert r.launches == [(0, 4), (4, 4), (8, 3)]
    ref = sum(FakeRenderer.sample(s, 4, 5) for s in range(11)) / 11
    assert fb.shape == (4, 5, 3) and np.abs(fb - ref).max() <= 1e-15


def test_resume_is_bitwise_the_uninterrupted_run(tmp_path):
    whole = render_progressive(FakeRenderer(), 6, 3, spp=10, bounces=1, chunk_spp=3,
                               checkpoint=tmp_path / "a.npz")
    ck = tmp_path / "b.npz"
    r = FakeRenderer()
    assert render_progressive(r, 6, 3, spp=10, bounces=1, chunk_spp=3, checkpoint=ck,
                              max_chunks=2) is None
    assert r.launches == [(0, 3), (3, 3)]
    r2 = FakeRenderer()
    seen = []
    fb = render_progressive(r2, 6, 3, spp=10, bounces=1, chunk_spp=3, checkpoint=ck,
                            on_chunk=lambda d, n: seen.append((d, n)))
    assert r2.launches == [(6, 3), (9, 1)] and seen == [(9, 10), (10, 10)]
    assert np.array_equal(fb, whole)
    assert not (tmp_path / "b.npz.tmp.npz").exists()
    # a finished checkpoint renders nothing more
    r3 = FakeRenderer()
    assert np.array_equal(render_progressive(r3, 6, 3, spp=10, bounces=1, chunk_spp=3,
                                             checkpoint=ck), whole)
    assert r3.launches == []


@pytest.mark.parametrize("change", [dict(spp=12), dict(bounces=2), dict(seed=5), dict(rr=True),
                                    dict(chunk_spp=4), dict(width=7), "scene"])
def test_checkpoint_of_another_render_is_refused(tmp_path, change):
    ck = tmp_path / "c.npz"
    base = dict(width=6, height=3, spp=10, bounces=1, chunk_spp=3)
    render_progressive(FakeRenderer(), checkpoint=ck, max_chunks=1, **base)
    if change == "scene":
        r, kw = FakeRenderer(salt=1e-9), base
    else:
        r, kw = FakeRenderer(), {**base, **change}
    with pytest.raises(ValueError, match="another render"):
        render_progressive(r, checkpoint=ck, **kw)
    assert r.launches == []


def test_checkpoint_file_is_plain_data(tmp_path):
    ck = tmp_path / "d.npz"
    render_progressive(FakeRenderer(), 4, 2, spp=5, bounces=1, chunk_spp=2, checkpoint=ck,
                       max_chunks=1)
    with np.load(ck, allow_pickle=False) as z:
        assert int(z["done"]) == 2 and z["sum"].shape == (2, 4, 3)
        key = json.loads(str(z["key"]))
    assert key["scene"] == scene_fingerprint(_Packed()) and key["spp"] == 5
    Checkpoint(ck).remove()
    assert not ck.exists()


def test_bad_arguments():
    with pytest.raises(ValueError):
        render_progressive(FakeRenderer(), 2, 2, spp=0)
    with pytest.raises(ValueError):
        render_progressive(FakeRenderer(), 2, 2, spp=4, chunk_spp=0)


def test_cli_checkpoint_needs_chunks(tmp_path):
    """main.py: --checkpoint without --chunk-spp is refused before any
    device work."""
    from conftest import CORNELL
    from pathtracerpython_amd import main as cli
    with pytest.raises(SystemExit, match="--chunk-spp"):
        cli.main([CORNELL, "-r", "2", "--checkpoint", str(tmp_path / "x.npz")])


def test_cli_chunks_need_one_device(tmp_path, monkeypatch):
    """--devices 2 with --chunk-spp (and --checkpoint) is refused
    in the parent, before any rank process starts (it used to render in one
    shot, ignoring both flags)."""
    from conftest import CORNELL
    from pathtracerpython_amd import launch
    from pathtracerpython_amd import main as cli

    def no_spawn(*a, **k):
        raise AssertionError("rank processes started")
    monkeypatch.setattr(launch, "spawn_ranks", no_spawn)
    for extra in ([], ["--checkpoint", str(tmp_path / "x.npz")]):
        with pytest.raises(SystemExit, match="--chunk-spp runs on one device"):
            cli.main([CORNELL, "-r", "4", "--devices", "2", "--chunk-spp", "2"] + extra)
    assert not (tmp_path / "x.npz").exists()


def test_render_devices_validation(cornell):
    from pathtracerpython_amd.render import render
    with pytest.raises(ValueError, match="devices"):
        render(cornell, 4, 4, devices=0)
    with pytest.raises(ValueError, match="devices"):
        render(cornell, 4, 4, devices=[])
    with pytest.raises(ValueError, match="devices"):
        render(cornell, 4, 4, devices=np.int64(0))
