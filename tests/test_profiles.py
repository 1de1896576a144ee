"""The measurement artifacts bench.py reads are current: the PMC traffic files
behind `roofline.traffic` must be stamped with the hash of the kernel sources
as they are now (bench.source_sha), so a kernel edit without a re-measure
(scripts/refresh_profiles.sh + install_profiles.py) turns this suite red
instead of silently dropping the HBM figure from the driver's bench line."""
import json
import os

import pytest

from conftest import ROOT


@pytest.mark.parametrize("config", ["k2", "k5"])
def test_traffic_stamp_matches_kernel_sources(config):
    import bench
    p = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    d = json.load(open(p))
    assert d["source_sha"] == bench.source_sha(), (
        f"{p} was measured on kernel sources {d['source_sha']}, the sources are now "
        f"{bench.source_sha()}: run scripts/refresh_profiles.sh on a GPU box and "
        f"scripts/install_profiles.py")
    assert d["hbm_bytes_per_launch"] > 0
    # ... which is also the id the built library carries (pt_build_id) and the
    # one bench.py checks the stamp against (the loaded library's)
    from pathtracerpython_amd import build
    assert d["source_sha"] == build.embedded_build_id(build.OUT)
    traffic, src = bench.load_traffic(config)
    assert traffic == d["hbm_bytes_per_launch"] and src
    assert d.get("statistic", "median") == "median"   # one statistic for every kernel


def test_source_sha_covers_the_kernel_sources():
    import bench
    csrc = os.path.join(ROOT, "pathtracerpython_amd", "csrc")
    assert sorted(f for f in os.listdir(csrc) if f.endswith((".h", ".hip")))
    assert len(bench.source_sha()) == 16
