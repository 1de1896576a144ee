"""Estimate (host only): would regrouping K2's lanes by shading origin cut
the unit pass's wave-level shadow tests?  (DESIGN.md §12 "a regrouping of
shadow rays by origin".)

The K2 kernel tests a uniform unit against a ray unless no lane of the wave
needs it (the plane skip, a wave-wide vote).  A lane needs unit u for shadow
ray k when the segment P -> L_k crosses u's plane.  This script traces
Cornell paths on the host (the oracle's intersect_objects for the hits,
cosine-weighted bounces, area-weighted light points), forms waves as the
kernel does (8 consecutive pixels of a row x 8 lanes) or regrouped inside a
pool of lanes by the origin's plane unit and a cell on it, and counts the
(wave, ray, unit) tests each grouping executes.  Prints one JSON line per
bounce and grouping.
Usage: shadow_coherence.py [crop_px] [cells]"""
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
CELLS = int(sys.argv[2]) if len(sys.argv) > 2 else 4
W = H = 512
LANES = 8
rng = np.random.default_rng(1)
scene_reader.VERBOSE = False
sc = scene_reader.Scene(os.path.join(ROOT, "scenes/cornell/cornellroom.sdl"))
pk = pack_scene(sc)
tv, tn, obj = pk.tri_v, pk.tri_n, pk.tri_obj
n_obj_tri = pk.n_obj_tri
# plane units: object triangles grouped by (object, plane)
keys, unit_of_tri = {}, np.zeros(len(tv), dtype=np.int64)
for t in range(len(tv)):
    n = tn[t] / np.linalg.norm(tn[t])
    c = float(n @ tv[t, 0])
    k = (int(obj[t]), tuple(np.round(n, 6)), round(c, 6))
    unit_of_tri[t] = keys.setdefault(k, len(keys))
planes = np.zeros((len(keys), 4))
for (o, n, c), u in keys.items():
    planes[u, :3], planes[u, 3] = n, c
obj_units = sorted({int(unit_of_tri[t]) for t in range(n_obj_tri)})
light = np.arange(n_obj_tri, len(tv))
la = pk.tri_area[light] / pk.tri_area[light].sum()
print(json.dumps({"units": len(keys), "object_units": len(obj_units), "crop": CROP, "cells": CELLS}),
      flush=True)

# lanes: the crop's pixels in the kernel's order (row-major within the band,
# 8 lanes per pixel), one sample each
x0 = (W - CROP) // 2
ix, iy = np.meshgrid(np.arange(x0, x0 + CROP), np.arange(x0, x0 + CROP))   # row = iy
ix, iy = ix.reshape(-1), iy.reshape(-1)
ix, iy = np.repeat(ix, LANES), np.repeat(iy, LANES)
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


def count(need, order, wave=64):
    """tests executed: sum over waves of any(need) per (ray, unit)."""
    nd = need[order]
    n = (len(nd) // wave) * wave
    return int(nd[:n].reshape(-1, wave, *nd.shape[1:]).any(1).sum())


for b in range(4):
    rays = np.concatenate([o, d], 1)
    tri, P = oracle.intersect_objects(pk, rays)
    hit = alive & (tri >= 0) & (tri < n_obj_tri)   # light hits end the path
    uP = np.where(tri >= 0, unit_of_tri[np.maximum(tri, 0)], -1)
    # shadow rays of the live lanes; dead lanes need nothing
    need = np.zeros((len(P), 3, len(obj_units)), dtype=bool)
    hP = P @ planes[obj_units, :3].T - planes[obj_units, 3]
    for k in range(3):
        L = light_points(len(P))
        hL = L @ planes[obj_units, :3].T - planes[obj_units, 3]
        cop = np.abs(hP) < 1e-9
        need[:, k] = hit[:, None] & (hP * hL < 0) & ~cop
    # groupings
    nat = np.arange(len(P))
    res = {"bounce": b, "live": int(hit.sum()), "lane_tests": int(need.sum()),
           "kernel_order": count(need, nat)}
    # cell on the origin's unit: quantise the two coordinates off the normal
    ax = np.abs(planes[np.maximum(uP, 0), :3]).argmax(1)
    lo, hi = P.min(0), P.max(0)
    q = np.clip(((P - lo) / np.maximum(hi - lo, 1e-12) * CELLS).astype(int), 0, CELLS - 1)
    qa = np.where(ax == 0, q[:, 1], q[:, 0])
    qb = np.where(ax == 2, q[:, 1], q[:, 2])
    key = np.where(hit, (uP * CELLS + qa) * CELLS + qb, 1 << 30)
    for pool in (256, 1024, 4096):
        order = np.concatenate([s + np.argsort(key[s:s + pool], kind="stable")
                                for s in range(0, len(P), pool)])
        res[f"sorted_{pool}"] = count(need, order)
    res["ratio_256"] = round(res["sorted_256"] / max(1, res["kernel_order"]), 3)
    res["ratio_4096"] = round(res["sorted_4096"] / max(1, res["kernel_order"]), 3)
    print(json.dumps(res), flush=True)
    # next bounce: cosine-weighted about the normal facing the ray
    n = tn[np.maximum(tri, 0)]
    n = n / np.linalg.norm(n, axis=1, keepdims=True)
    n = np.where(((n * d).sum(1) > 0)[:, None], -n, n)
    u1, u2 = rng.random(len(P)), rng.random(len(P))
    r, ph = np.sqrt(u1), 2 * np.pi * u2
    t1 = np.cross(n, np.where(np.abs(n[:, :1]) > 0.9, [[0, 1, 0]], [[1, 0, 0]]))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(n, t1)
    d = (r * np.cos(ph))[:, None] * t1 + (r * np.sin(ph))[:, None] * t2 + np.sqrt(1 - u1)[:, None] * n
    o = P
    alive = hit
