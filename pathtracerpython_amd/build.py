"""Build libpt_hip.so in-tree with hipcc for gfx950 (no JIT cache: the built
library travels with the repository snapshot to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "_lib", "libpt_hip.so")
SOURCES = ["pt_hip.hip"]
DEPS = SOURCES + ["pt_core.h", "pt_math.h", "pt_path.h", "pt_prepare.h", "pt_image.h", "pt_ingest.h", "pt_wavefront.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: every f64 operation rounds separately, as the reference's
# numpy does; the f32 filter writes its fmaf() explicitly.
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-Wall"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in DEPS] + [os.path.join(ROOT, "include", "pt_capi.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force=False, verbose=True):
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
