"""Estimate (host only): a per-wave, per-object box cull in K2's unit pass.
Before an object's units (a cube's faces), a wave tests its rays against
the object's bounding box; when no lane's shadow segment k (two-sided, the
reference's line semantics) meets the box, the object's units skip ray k's
plane checks and tests.  Counts, over the kernel's waves (8 pixels of a row
x 8 lanes), the VALU of the unit pass's shadow part under a cost model:
plane check 14 per (wave, unit, ray), full test 30 more when some lane
needs it (segment crosses the unit's plane), box test 15 per (wave,
object, ray).  Paths as scripts/micro/shadow_coherence.py.
Usage: object_cull.py [crop_px]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402  (host-side estimate)
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.pack import pack_scene  # noqa: E402

CROP = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W = H = 512
LANES = 8
PLANE, TEST, BOX = 14, 30, 15
rng = np.random.default_rng(1)
scene_reader.VERBOSE = False
pk = pack_scene(scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl")))
tv, tn, obj = pk.tri_v, pk.tri_n, pk.tri_obj
n_obj_tri = pk.n_obj_tri
keys, unit_of_tri, unit_obj = {}, np.zeros(len(tv), dtype=np.int64), {}
for t in range(len(tv)):
    n = tn[t] / np.linalg.norm(tn[t])
    k = (int(obj[t]), tuple(np.round(n, 6)), round(float(n @ tv[t, 0]), 6))
    unit_of_tri[t] = keys.setdefault(k, len(keys))
    unit_obj[unit_of_tri[t]] = int(obj[t])
planes = np.zeros((len(keys), 4))
for (o, n, c), u in keys.items():
    planes[u, :3], planes[u, 3] = n, c
ou = sorted({int(unit_of_tri[t]) for t in range(n_obj_tri)})
objs = sorted({unit_obj[u] for u in ou})
boxes = {o: (tv[:n_obj_tri][obj[:n_obj_tri] == o].reshape(-1, 3).min(0) - 1e-6,
             tv[:n_obj_tri][obj[:n_obj_tri] == o].reshape(-1, 3).max(0) + 1e-6) for o in objs}
light = np.arange(n_obj_tri, len(tv))
la = pk.tri_area[light] / pk.tri_area[light].sum()

x0 = (W - CROP) // 2
ix, iy = np.meshgrid(np.arange(x0, x0 + CROP), np.arange(x0, x0 + CROP))
ix, iy = np.repeat(ix.reshape(-1), LANES), np.repeat(iy.reshape(-1), LANES)
eye = pk.eye
xs = np.linspace(pk.ortho[0], pk.ortho[2], W)[ix]
ys = np.linspace(pk.ortho[1], pk.ortho[3], H)[iy]
o = np.repeat(eye[None], len(ix), 0)
d = np.stack([xs - eye[0], ys - eye[1], -eye[2] * np.ones_like(xs)], 1)
alive = np.ones(len(ix), dtype=bool)


def light_points(n):
    t = light[rng.choice(len(light), n, p=la)]
    u = rng.random((n, 2))
    s = np.sqrt(u[:, 0])
    b = np.stack([1 - s, s * (1 - u[:, 1]), s * u[:, 1]], 1)
    return np.einsum("nk,nkc->nc", b, tv[t])


def seg_box(P, L, lo, hi):
    """two-sided segment [2P - L, L] meets the box (slab test)"""
    A, Bp = 2 * P - L, L
    dd = Bp - A
    with np.errstate(divide="ignore", invalid="ignore"):
        t0 = (lo - A) / dd
        t1 = (hi - A) / dd
    tmin = np.nanmax(np.minimum(t0, t1), 1)
    tmax = np.nanmin(np.maximum(t0, t1), 1)
    return (tmin <= tmax) & (tmax >= 0) & (tmin <= 1)


tot = {"base": 0, "cull": 0}
for b in range(4):
    tri, P = oracle.intersect_objects(pk, np.concatenate([o, d], 1))
    hit = alive & (tri >= 0) & (tri < n_obj_tri)
    hP = P @ planes[ou, :3].T - planes[ou, 3]
    nw = len(P) // 64
    base = cull = 0
    boxmiss = np.zeros(len(objs))
    for k in range(3):
        L = light_points(len(P))
        hL = L @ planes[ou, :3].T - planes[ou, 3]
        need = hit[:, None] & (hP * hL < 0) & ~(np.abs(hP) < 1e-9)
        wneed = need[:nw * 64].reshape(nw, 64, -1).any(1)          # (wave, unit)
        base += nw * len(ou) * PLANE + wneed.sum() * TEST
        for j, ob in enumerate(objs):
            cols = [i for i, u in enumerate(ou) if unit_obj[u] == ob]
            if len(cols) < 2:     # single-unit objects: no box
                cull += nw * len(cols) * PLANE + wneed[:, cols].sum() * TEST
                continue
            inb = hit & seg_box(P, L, *boxes[ob])
            wbox = inb[:nw * 64].reshape(nw, 64).any(1)
            boxmiss[j] += (~wbox).sum()
            cull += nw * BOX + wbox.sum() * len(cols) * PLANE + (wneed[:, cols] & wbox[:, None]).sum() * TEST
    tot["base"] += base
    tot["cull"] += cull
    print(json.dumps({"bounce": b, "waves": nw, "shadow_valu_base": int(base), "shadow_valu_cull": int(cull),
                      "ratio": round(cull / base, 3),
                      "box_miss_frac": {str(ob): round(boxmiss[j] / (3 * nw), 3)
                                        for j, ob in enumerate(objs) if boxmiss[j] or True}}), flush=True)
    n = tn[np.maximum(tri, 0)]
    n = n / np.linalg.norm(n, axis=1, keepdims=True)
    n = np.where(((n * d).sum(1) > 0)[:, None], -n, n)
    u1, u2 = rng.random(len(P)), rng.random(len(P))
    r, ph = np.sqrt(u1), 2 * np.pi * u2
    t1 = np.cross(n, np.where(np.abs(n[:, :1]) > 0.9, [[0, 1, 0]], [[1, 0, 0]]))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(n, t1)
    d = (r * np.cos(ph))[:, None] * t1 + (r * np.sin(ph))[:, None] * t2 + np.sqrt(1 - u1)[:, None] * n
    o, alive = P, hit
print(json.dumps({"total_ratio": round(tot["cull"] / tot["base"], 3),
                  "units_per_object": {str(ob): sum(unit_obj[u] == ob for u in ou) for ob in objs}}))
