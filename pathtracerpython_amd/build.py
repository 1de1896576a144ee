"""Build libpt_hip.so in-tree with hipcc for gfx950 (no JIT cache: the built
library travels with the repository snapshot to the GPU box).

Every build is stamped with the content hash of the sources it was compiled
from (`source_sha`: csrc/*.h, csrc/*.hip, include/pt_capi.h, and the compile
recipe: FLAGS and each unit's own flags, UNITS), compiled in as
PT_BUILD_ID and exported by `pt_build_id()`.  Staleness is decided by that
hash, not by file times, and `_native.lib()` refuses a library whose id is not
the hash of the sources on disk, so a measurement always names the sources of
the binary that produced it (bench.py reports the loaded library's id)."""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
HEADER = os.path.join(ROOT, "include", "pt_capi.h")
OUT = os.path.join(HERE, "_lib", "libpt_hip.so")
SOURCES = ["pt_hip.hip"]
# translation units compiled on their own, with extra code-generation flags,
# and linked into the library: the K2 kernel (pt_k2.hip) and the wavefront
# shade step (pt_shade.hip) under LLVM's iterative ILP scheduler (the walk
# kernels lose under it)
_ILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
UNITS = {"pt_k2.hip": _ILP, "pt_shade.hip": _ILP}
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -ffp-contract=off: every f64 operation rounds separately, as the reference's
# numpy does; the f32 filter writes its fmaf() explicitly.
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]
# the id string in the library: MARKER followed by the 16 hex digits
MARKER = b"PT_BUILD_ID="
ID_LEN = 16


def source_files(csrc=CSRC, header=HEADER):
    return [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))
            if f.endswith((".h", ".hip"))] + [header]


def recipe(flags=None, units=None):
    """The compile recipe as text: the common flags and each unit's own (the
    same sources under other code-generation flags are another binary)."""
    flags = FLAGS if flags is None else flags
    units = UNITS if units is None else units
    return "\0".join([ARCH] + list(flags) + ["%s:%s" % (u, " ".join(units[u])) for u in sorted(units)])


def source_sha(csrc=CSRC, header=HEADER, flags=None, units=None):
    """Content hash of the kernel sources and the compile recipe (16 hex
    digits)."""
    h = hashlib.sha256()
    for p in source_files(csrc, header):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(recipe(flags, units).encode())
    return h.hexdigest()[:ID_LEN]


def embedded_build_id(path):
    """The PT_BUILD_ID a built library carries, read from its bytes (no load,
    no HIP runtime), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(MARKER)
    if i < 0:
        return None
    s = data[i + len(MARKER):i + len(MARKER) + ID_LEN]
    return s.decode("ascii", "replace")


def _stale(out=OUT, csrc=CSRC):
    return embedded_build_id(out) != source_sha(csrc)


def variant_id(sha, defines):
    """The id of a build with -D switches: the sources' hash folded with the
    sorted switches, so a variant never carries the default build's id — it
    loads only with PT_ALLOW_FOREIGN_BUILD=1 and is always named by its own id
    (ADVICE r05)."""
    if not defines:
        return sha
    h = hashlib.sha256((sha + "\0" + "\0".join(sorted(defines))).encode())
    return h.hexdigest()[:ID_LEN]


def compile_lib(out, defines=(), csrc=CSRC, verbose=True):
    """hipcc the library into `out`, stamped with the hash of `csrc`'s sources
    (dev variants pass -D switches or raw flags: their id also covers them,
    variant_id)."""
    sha = variant_id(source_sha(csrc), tuple(defines))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # (an item starting with "-" is a raw compiler flag, e.g. -mllvm options;
    # "UNIT=name.hip:flags ..." replaces that unit's own flags)
    unit_flags = dict(UNITS)
    for d in defines:
        if d.startswith("UNIT="):
            name, _, fl = d[5:].partition(":")
            if name not in UNITS:
                raise ValueError("UNIT= names one of %s" % sorted(UNITS))
            unit_flags[name] = fl.split()
    defines = [d for d in defines if not d.startswith("UNIT=")]
    common = FLAGS + [f"-DPT_BUILD_ID=\"{sha}\""] + [d if d.startswith("-") else "-D" + d for d in defines]
    objs = []
    # (a variant's own scheduler strategy replaces a unit's)
    own_sched = any(d.startswith("-amdgpu-sched-strategy") for d in defines)
    for unit, extra in [(u, []) for u in SOURCES] + list(unit_flags.items()):
        if own_sched:
            extra = []
        obj = "%s.%s.o" % (out, os.path.splitext(unit)[0])
        cmd = [HIPCC] + common + extra + ["-c", "-o", obj, os.path.join(csrc, unit)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-fPIC", "-shared", "--hip-link", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    for obj in objs:
        os.remove(obj)
    os.replace(out + ".tmp", out)
    return out


def build(force=False, verbose=True):
    if not force and not _stale():
        return OUT
    return compile_lib(OUT, verbose=verbose)


def build_variant(name, defines):
    """Dev: the library with compile-time switches (-D...) as
    _lib/variants/<name>.so, for the timing scripts (PT_HIP_LIB)."""
    return compile_lib(os.path.join(HERE, "_lib", "variants", name + ".so"), defines, verbose=False)


if __name__ == "__main__":
    # python -m pathtracerpython_amd.build [--force]
    # python -m pathtracerpython_amd.build --variant NAME FOO=1 BAR=2 ...
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        build(force="--force" in sys.argv)
