"""Flatten a `Scene` into the plain arrays of `pt_scene_desc` (include/pt_capi.h).

Triangle order is the reference's iteration order in intersect_objects
(main.py:91-96): every object's triangles in scene order, then the light's.
Object triangles come first, so the shadow-ray occluder set of
compute_shadow_rays (main.py:42, objects only) is the prefix [0, n_obj_tri).
"""
import ctypes as C

import numpy as np

from ._abi import PtSceneDesc

MAT_KEYS = ('red', 'green', 'blue', 'ka', 'kd', 'ks', 'kt', 'n')


def _mesh_arrays(g):
    """(tri_v (n,3,3), tri_n (n,3), area (n,)) float64 of an Obj: the native
    reader's arrays as they are, else built from the reference's lists."""
    a = getattr(g, 'arrays', None)
    if a is not None:
        return a['tri_v'], a['tri_n'], a['tri_area']
    n = len(g.triangles)
    tv = np.array([[v[:3] for v in t] for t in g.triangles], dtype=np.float64).reshape(n, 3, 3)
    tn = np.array([nv[:3] for nv in g.normals], dtype=np.float64).reshape(n, 3)
    return tv, tn, np.array(g.areas, dtype=np.float64).reshape(n)


class PackedScene:
    """Owns the numpy arrays a PtSceneDesc points into."""

    def __init__(self, scene):
        if scene.light_obj is None:
            raise ValueError("scene has no light (SDL `light` keyword)")
        n_obj = len(scene.objects)
        geoms = [o['geometry'] for o in scene.objects] + [scene.light_obj]
        parts = [_mesh_arrays(g) for g in geoms]
        counts = [p[2].shape[0] for p in parts]
        self.n_obj_tri = int(sum(counts[:-1]))
        if counts[-1] == 0:
            raise ValueError("light object has no triangles")
        self.n_obj = n_obj
        self.tri_v = np.ascontiguousarray(np.concatenate([p[0] for p in parts]).reshape(-1, 3, 3))
        self.tri_n = np.ascontiguousarray(np.concatenate([p[1] for p in parts]).reshape(-1, 3))
        self.tri_area = np.ascontiguousarray(np.concatenate([p[2] for p in parts]))
        self.tri_obj = np.ascontiguousarray(
            np.repeat(np.arange(n_obj + 1, dtype=np.int32), counts).astype(np.int32))
        self.mat = np.ascontiguousarray(np.array(
            [[float(o[k]) for k in MAT_KEYS] for o in scene.objects],
            dtype=np.float64).reshape(-1, 8))
        self.eye = np.array(scene.eye, dtype=np.float64)
        self.ortho = np.array(scene.ortho, dtype=np.float64)
        self.ambient = float(scene.ambient)
        lc = list(scene.light_color) + [0.0] * 3
        self.light_rgb = np.array(lc[:3], dtype=np.float64)
        self.desc = self._make_desc()

    @property
    def n_tri(self):
        return self.tri_v.shape[0]

    def _make_desc(self):
        d = PtSceneDesc()
        d.n_tri = self.n_tri
        d.n_obj_tri = self.n_obj_tri
        d.n_obj = self.n_obj
        dp = C.POINTER(C.c_double)
        d.tri_v = self.tri_v.ctypes.data_as(dp)
        d.tri_n = self.tri_n.ctypes.data_as(dp)
        d.tri_area = self.tri_area.ctypes.data_as(dp)
        d.tri_obj = self.tri_obj.ctypes.data_as(C.POINTER(C.c_int32))
        d.mat = self.mat.ctypes.data_as(dp)
        d.eye[:] = [float(x) for x in self.eye]
        d.ortho[:] = [float(x) for x in self.ortho]
        d.ambient = self.ambient
        d.light_rgb[:] = [float(x) for x in self.light_rgb]
        return d


def pack_scene(scene):
    return PackedScene(scene)
