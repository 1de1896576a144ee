"""Synthetic scenes for the configurations BASELINE.json names.

K5 ("Synthetic 100k-triangle random mesh 1024x1024 256 spp", SURVEY.md
§8(d)): the Cornell walls and light plus n random small triangles —
centroids uniform in the box interior x in [-3.8, 3.8], y in [-3.84, 3.8],
z in [-32.7, -16.6], vertices = centroid + N(0, 0.05^2) per coordinate,
numpy default_rng(seed), one white object (kd .7).  Written as plain v/f OBJ
files referenced by an SDL `object` line, so the scene goes through the same
ingest as the reference's scenes (scene_reader / pt_obj_load).

    python -m pathtracerpython_amd.synth out_dir [n_tris] [seed]
"""
import os
import shutil
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
CORNELL_DIR = os.path.join(os.path.dirname(_HERE), "scenes", "cornell")
WALLS = ("leftwall.obj", "rightwall.obj", "floor.obj", "back.obj", "ceiling.obj")


def write_k5_scene(out_dir, n_tris=100_000, seed=0, size=1024, cornell_dir=CORNELL_DIR):
    """Write the K5 scene into out_dir; returns the SDL path."""
    os.makedirs(out_dir, exist_ok=True)
    for f in WALLS + ("luzcornell.obj",):
        shutil.copy(os.path.join(cornell_dir, f), os.path.join(out_dir, f))
    rng = np.random.default_rng(seed)
    c = rng.uniform([-3.8, -3.84, -32.7], [3.8, 3.8, -16.6], (n_tris, 3))
    v = c[:, None, :] + rng.normal(0.0, 0.05, (n_tris, 3, 3))
    v = v.reshape(-1, 3)
    lines = ["# K5 synthetic mesh: %d random triangles, default_rng(%d)" % (n_tris, seed)]
    lines += ["v %.17g %.17g %.17g" % tuple(x) for x in v.tolist()]
    lines += ["f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3) for i in range(n_tris)]
    with open(os.path.join(out_dir, "random_mesh.obj"), "w") as f:
        f.write("\n".join(lines) + "\n")
    sdl = [
        "# K5: Cornell walls + light + %d random triangles (SURVEY.md 8(d))" % n_tris,
        "eye 0.0 0.0 5.7",
        "size %d %d" % (size, size),
        "ortho -1 -1 1 1",
        "background 0.0 0.0 0.0",
        "ambient 0.5",
        "light luzcornell.obj 1.0 1.0 1.0",
        "seed 9",
        "object leftwall.obj 1.0 0.0 0.0 0.3 0.7 0 0 5",
        "object rightwall.obj 0.0 1.0 0.0 0.3 0.7 0 0 5",
        "object floor.obj 1.0 1.0 1.0 0.3 0.7 0 0 5",
        "object back.obj 1.0 1.0 1.0 0.3 0.7 0 0 5",
        "object ceiling.obj 1.0 1.0 1.0 0.3 0.7 0 0 5",
        "object random_mesh.obj 1.0 1.0 1.0 0.3 0.7 0 0 5",
    ]
    path = os.path.join(out_dir, "k5.sdl")
    with open(path, "w") as f:
        f.write("\n".join(sdl) + "\n")
    return path


if __name__ == "__main__":
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    print(write_k5_scene(out, n, seed))
