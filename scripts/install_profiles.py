"""Install a refresh_profiles.sh run into profiles/ (dev tool, runs here).

    python3 scripts/install_profiles.py TAG

Copies gpurun_out/refresh_TAG/profiles/* into profiles/ after checking that
the stamped traffic files were measured on the current kernel sources (the
hash bench.py checks); refuses otherwise, so a stale measurement never lands.
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"refresh_{tag}", "profiles")
    files = sorted(glob.glob(os.path.join(src, "*")))
    if not files:
        raise SystemExit(f"nothing staged under {src}")
    sha = bench.source_sha()
    for f in files:
        if os.path.basename(f).startswith("traffic_"):
            got = json.load(open(f)).get("source_sha")
            if got != sha:
                raise SystemExit(f"{f}: measured on kernel sources {got}, current {sha}: re-measure")
    for f in files:
        shutil.copy(f, os.path.join(ROOT, "profiles", os.path.basename(f)))
        print("installed", os.path.basename(f))


if __name__ == "__main__":
    main()
