"""The edge-case mesh scene of the BVH golden (TEST INFRASTRUCTURE: used by
gen_golden.py to render the reference on it, and by the tests to render the
same scene through the oracle, the host build and the GPU).

The Cornell room (reference `objs/cornellroom.sdl`) plus one object of 68
triangles — above the BVH threshold (pt_prepare.h kBvhMinTris = 64), so the
mesh runs through the BVH walks and the wavefront kernels, which the Cornell
goldens never reach:
  * 48 random triangles in the room,
  * 8 exact duplicates of the first 8 (later in scene order: closest-hit ties
    go to the first, main.py:100-104),
  * a fan of 8 triangles around one centre vertex (every edge shared),
  * 4 triangles in the back wall's plane z = -32.76, over the wall (coplanar
    with the wall's triangles: the sqd > 1e-5 self-hit rule, main.py:46-51).
Coordinates are multiples of 1/64 (exact in the parsed doubles).  The mesh
object comes before the cubes, so the leaked colour of the last shadow ray
(main.py:70) mixes BVH and uniform occluders.
"""
import os
import shutil

import numpy as np

W, H, SPP, BOUNCES, SEED = 12, 12, 2, 3, 5
NAME = "mesh_render_12x12_s2_b3_seed5.npz"   # (not render_*: the Cornell goldens)


def _q(x):
    return np.round(np.asarray(x, dtype=np.float64) * 64.0) / 64.0


def mesh_triangles():
    rs = np.random.RandomState(2024)
    tris = []
    for _ in range(48):
        c = rs.uniform([-3.4, -3.4, -31.0], [3.4, 3.4, -18.0])
        tris.append([_q(c + rs.normal(0.0, 0.7, 3)) for _ in range(3)])
    tris += [list(t) for t in tris[:8]]                      # exact duplicates
    centre = _q([0.5, 0.25, -24.0])
    ring = [_q(centre + 1.2 * np.array([np.cos(a), 0.6 * np.sin(a), 0.8 * np.sin(a)]))
            for a in np.arange(8) * (2 * np.pi / 8)]
    for i in range(8):                                        # the fan
        tris.append([centre, ring[i], ring[(i + 1) % 8]])
    z = -32.76                                                # the back wall's plane
    for _ in range(4):
        xy = rs.uniform([-3.5, -3.5], [3.5, 3.5])
        tris.append([np.array([*_q(xy + rs.normal(0.0, 0.9, 2)), z]) for _ in range(3)])
    return tris


def write_mesh_scene(out_dir, cornell_dir):
    """Write the scene into out_dir (Cornell OBJs copied from cornell_dir);
    returns the SDL path."""
    os.makedirs(out_dir, exist_ok=True)
    for f in os.listdir(cornell_dir):
        if f.endswith(".obj"):
            shutil.copy(os.path.join(cornell_dir, f), os.path.join(out_dir, f))
    tris = mesh_triangles()
    lines = ["# edge-case mesh (tests/golden/mesh_scene.py)"]
    for t in tris:
        for v in t:
            lines.append("v %.17g %.17g %.17g" % tuple(v))
    lines += ["f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3) for i in range(len(tris))]
    with open(os.path.join(out_dir, "edge.obj"), "w") as f:
        f.write("\n".join(lines) + "\n")
    sdl = "\n".join([
        "eye 0.0 0.0 5.7",
        "size %d %d" % (W, H),
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
        "object edge.obj 0.2 0.6 0.9 0.3 0.7 0.5 0 5",
        "object cube1.obj 1.0 1.0 1.0 0.3 0.7 0.9 0 5",
        "object cube2.obj 1.0 1.0 1.0 0.3 0.7 0.6 0 5",
    ]) + "\n"
    path = os.path.join(out_dir, "mesh.sdl")
    with open(path, "w") as f:
        f.write(sdl)
    return path
