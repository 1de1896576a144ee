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


class PackedScene:
    """Owns the numpy arrays a PtSceneDesc points into."""

    def __init__(self, scene):
        if scene.light_obj is None:
            raise ValueError("scene has no light (SDL `light` keyword)")
        tris, norms, areas, obj_ids = [], [], [], []
        n_obj = len(scene.objects)
        for oi, obj in enumerate(scene.objects):
            g = obj['geometry']
            for t, n, a in zip(g.triangles, g.normals, g.areas):
                tris.append([v[:3] for v in t])
                norms.append(n[:3])
                areas.append(a)
                obj_ids.append(oi)
        self.n_obj_tri = len(tris)
        lg = scene.light_obj
        for t, n, a in zip(lg.triangles, lg.normals, lg.areas):
            tris.append([v[:3] for v in t])
            norms.append(n[:3])
            areas.append(a)
            obj_ids.append(n_obj)
        if len(tris) == self.n_obj_tri:
            raise ValueError("light object has no triangles")
        self.n_obj = n_obj
        self.tri_v = np.ascontiguousarray(np.array(tris, dtype=np.float64).reshape(-1, 3, 3))
        self.tri_n = np.ascontiguousarray(np.array(norms, dtype=np.float64).reshape(-1, 3))
        self.tri_area = np.ascontiguousarray(np.array(areas, dtype=np.float64))
        self.tri_obj = np.ascontiguousarray(np.array(obj_ids, dtype=np.int32))
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
