"""ISA attribution of k_render's unit loop (dev tool, CPU only).

Compiles pathtracerpython_amd/csrc/pt_hip.hip for gfx950 to assembly (device
only, the library's flags plus any -D switches given), extracts
k_render<false,false,false> (the K2 kernel) and its uniform-unit loop (the
depth-2 loop that loads the 128-B unit records), and prints every basic block
of the loop with its VALU / SALU / SMEM counts, marking the rare blocks (f64:
the fallbacks and the shadow-bit rebuild).  --listing prints the hot blocks'
instructions.
    python3 scripts/isa_unit_loop.py [--listing] [--csrc DIR] [-DNAME=VALUE ...]"""
import collections
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pathtracerpython_amd import build  # noqa: E402

KERNEL = "_Z8k_renderILb0ELb0ELb0EE"


def compile_asm(defines, csrc=build.CSRC):
    out = os.path.join(tempfile.gettempdir(), "pt_isa_%d.s" % os.getpid())
    # the K2 kernel's translation unit and its flags (build.UNITS), when the
    # tree has one (an earlier round's, --csrc: pt_hip.hip)
    unit = "pt_k2.hip" if os.path.exists(os.path.join(csrc, "pt_k2.hip")) else "pt_hip.hip"
    cmd = [build.HIPCC, "--offload-arch=" + build.ARCH, "-O3", "-std=c++17", "-ffp-contract=off",
           "--cuda-device-only", "-S", "-DPT_BUILD_ID=\"isa\"", "-o", out] + \
          build.UNITS.get(unit, []) + defines + [os.path.join(csrc, unit)]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    with open(out) as f:
        return f.read().split("\n")


def main():
    listing = "--listing" in sys.argv
    defines = [a for a in sys.argv[1:] if a.startswith("-") and a not in ("--listing", "--csrc")]
    # --csrc DIR: another source tree (e.g. an earlier round's, from git archive)
    csrc = sys.argv[sys.argv.index("--csrc") + 1] if "--csrc" in sys.argv else build.CSRC
    s = compile_asm(defines, csrc)
    start = next(i for i, l in enumerate(s) if l.startswith(KERNEL))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    f = s[start:end]
    meta = [l.strip() for l in s[end:end + 80] if any(k in l for k in ("NumVgprs:", "NumSgprs:", "ScratchSize:",
                                                                        "Occupancy:", "SGPRBlocks", "VGPRSpill",
                                                                        "SGPRSpill"))]
    # the unit loop: of the depth-2 loops whose header loads unit records, the
    # largest (the uniform units' fused pass; the light units' loop is small)
    best, size = None, -1
    for i, l in enumerate(f):
        if "Inner Loop Header: Depth=2" in l:
            lab = (f[i] if f[i].startswith(".LBB") else f[i - 1]).split(":")[0]
            nm = lab.replace(".LBB", "BB")
            n = sum(1 for x in f if ("Header=" + nm) in x)
            if n > size:   # (the fused pass is by far the largest depth-2 loop)
                best, size = lab, n
    if best is None:
        raise SystemExit("unit loop not found")
    name = best.replace(".LBB", "BB")
    blocks = []   # (label, [instructions])
    cur = None
    for l in f:
        t = l.strip()
        if l.startswith(".LBB") or t.startswith("; %bb"):
            in_loop = l.startswith(best + ":") or ("Header=" + name) in l
            cur = [t.split()[0].rstrip(":") if l.startswith(".LBB") else t.split()[1], []] if in_loop else None
            if cur:
                blocks.append(cur)
            continue
        if cur is not None and t and not t.startswith(";") and not t.startswith(".") and not t.startswith("s_nop") \
                and "ASM" not in t:
            cur[1].append(t)
        elif cur is not None and t.startswith("s_nop"):
            cur[1].append(t)
    tot = collections.Counter()
    print(f"k_render<false,false,false> unit loop ({best}), {len(blocks)} blocks; {' | '.join(meta)}")
    print(f"{'block':>10} {'VALU':>5} {'SALU':>5} {'SMEM':>5} {'nop':>4}  kind")
    for lab, ins in blocks:
        c = collections.Counter()
        for t in ins:
            op = t.split()[0]
            if op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("s_load") or op.startswith("s_buffer_load"):
                c["smem"] += 1
            elif op == "s_nop":
                c["nop"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
        rare = any("_f64" in t for t in ins)
        kind = "rare (f64)" if rare else "hot"
        for k in c:
            tot[(kind, k)] += c[k]
        print(f"{lab:>10} {c['valu']:>5} {c['salu']:>5} {c['smem']:>5} {c['nop']:>4}  {kind}")
        if listing and not rare:
            for t in ins:
                print("           ", t)
    for kind in ("hot", "rare (f64)"):
        print(f"{kind:>12}: VALU {tot[(kind, 'valu')]}, SALU {tot[(kind, 'salu')]}, SMEM {tot[(kind, 'smem')]}, "
              f"s_nop {tot[(kind, 'nop')]}")


if __name__ == "__main__":
    main()
