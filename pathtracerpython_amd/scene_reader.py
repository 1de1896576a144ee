"""SDL / OBJ scene ingest — drop-in mirror of the reference's `scene_reader`.

Same classes (`Scene`, `Obj`), attribute names, keyword handling and error
behaviour as /root/reference/scene_reader.py:1-188, so code written against
the reference keeps working.  The per-triangle normal and area are computed
with the reference's own operation order (vector.py:143-173) so the values
are bit-identical to the reference's — the keyed-RNG parity tests depend on
that (the normal feeds the bounce rotation, the areas feed the light-pick
CDF).

OBJ files are read by the native reader of libpt_hip.so (pt_obj_load,
SURVEY.md §8(f) row 2) when it is available: same semantics, bit-identical
normals and areas, ~100x faster on large meshes.  The mesh then stays in
numpy arrays (`Obj.arrays`), and the reference's list attributes
(triangles, normals, areas, vertexes, faces) are built on first access.
Inputs outside the native reader's subset, or a missing library, fall back
to the Python reader below, which raises what the reference raises.
"""
import ctypes as C
from math import sqrt
from os.path import dirname, join

VERBOSE = True
NATIVE_OBJ = True   # use pt_obj_load when libpt_hip.so is present


def _log(msg):
    if VERBOSE:
        print(msg)


def _sub(a, b):
    # vector.py:125-127: V.__sub__ is self + (-vec), i.e. (-b_i) + a_i
    return ((-b[0]) + a[0], (-b[1]) + a[1], (-b[2]) + a[2])


def _cross(u, v):
    # vector.py:143-146
    return (u[1] * v[2] - u[2] * v[1],
            u[2] * v[0] - u[0] * v[2],
            u[0] * v[1] - u[1] * v[0])


def _size(v):
    # vector.py:111-113: sqrt(sum(c**2)); sum starts at int 0
    s = 0
    for c in v:
        s = s + c ** 2
    return sqrt(s)


def calc_normal(tri):
    """normalize(cross(v2 - v1, v3 - v1)) — scene_reader.py:5-8, vector.py:172."""
    c = _cross(_sub(tri[1], tri[0]), _sub(tri[2], tri[0]))
    k = 1 / _size(c)
    return (c[0] * k, c[1] * k, c[2] * k)


def triangle_area(tri):
    """|cross(v2 - v1, v3 - v1)| / 2 — vector.py:164-165."""
    return _size(_cross(_sub(tri[1], tri[0]), _sub(tri[2], tri[0]))) / 2


def _tokens(line):
    # scene_reader.py:11-26: split on single spaces, drop empty tokens
    return [t for t in line.split(' ') if t not in ('', ' ')]


def _strip_comments(lines):
    """scene_reader.py:29-46: strip leading spaces, drop '#' lines and tails."""
    kept = []
    for line in lines:
        i = 0
        while line[i] == ' ':          # IndexError on an all-space last line,
            i += 1                     # as in the reference
        line = line[i:]
        if line[0] == '#':
            continue
        if '#' in line:
            line = line.split('#')[0]
        kept.append(line.replace('\n', '').replace('\t', ' '))
    return kept


def _native_obj(path):
    """(arrays dict, skipped raw lines) from pt_obj_load, or None when the
    library is missing or the file is outside the native reader's subset."""
    if not NATIVE_OBJ:
        return None
    try:
        import numpy as np
        from . import _native
        lib = _native.lib()
        load = lib.pt_obj_load
    except Exception:
        return None
    m = C.POINTER(_native.PtMesh)()
    if load(path.encode(), C.byref(m)) != 0:
        return None
    try:
        M = m.contents
        nv, nt, ns = M.n_vert, M.n_tri, M.n_skip

        def arr(ptr, shape, dt):
            n = int(np.prod(shape))
            if n == 0:
                return np.zeros(shape, dtype=dt)
            return np.ctypeslib.as_array(ptr, (n,)).astype(dt, copy=True).reshape(shape)

        out = {"vert": arr(M.vert, (nv, 3), np.float64),
               "face": arr(M.face, (nt, 3), np.int64),
               "tri_v": arr(M.tri_v, (nt, 3, 3), np.float64),
               "tri_n": arr(M.tri_n, (nt, 3), np.float64),
               "tri_area": arr(M.tri_area, (nt,), np.float64)}
        skips = [(int(M.skip_off[i]), int(M.skip_len[i])) for i in range(ns)]
    finally:
        lib.pt_mesh_free(m)
    return out, skips


class Obj:
    """Triangle mesh from an OBJ file: `v` and `f` records only
    (scene_reader.py:49-104).  Faces with more than three indices are fan
    triangulated; negative indices count back from the last vertex read."""

    _LAZY = ('triangles', 'areas', 'normals', 'vertexes', 'faces', 'vtx_idx')

    def __init__(self, path):
        _log('Reading ' + path)
        self.arrays = None
        nat = _native_obj(path)
        if nat is not None:
            self.arrays, skips = nat
            if skips and VERBOSE:
                with open(path, 'rb') as f:
                    raw = f.read()
                for off, ln in skips:
                    t = _tokens(_strip_comments([raw[off:off + ln].decode() + '\n'])[0])
                    _log(f'{path}\n\tSkipping command \'{t[0]}\' ! '
                         f'\n\tParameters: {t[1:]}')
            return
        self.triangles = []
        self.areas = []
        self.normals = []
        self.vertexes = []
        self.faces = []
        self.vtx_idx = 0
        self.read_obj(path)

    def __getattr__(self, name):
        # the reference's list attributes, built from the native arrays on
        # first access (only called when normal lookup fails)
        if name not in Obj._LAZY or self.__dict__.get('arrays') is None:
            raise AttributeError(name)
        a = self.arrays
        verts = [tuple(v) for v in a['vert'].tolist()]
        faces = a['face'].tolist()
        self.vertexes = verts
        self.vtx_idx = len(verts)
        self.faces = faces
        # from the parse-time vertex triples (a negative index means the
        # vertices read so far, not the final list)
        self.triangles = [tuple(tuple(v) for v in t) for t in a['tri_v'].tolist()]
        self.normals = [tuple(n) for n in a['tri_n'].tolist()]
        self.areas = a['tri_area'].tolist()
        return getattr(self, name)

    def parse_vertex(self, tokens):
        self.vertexes.append(tuple(float(x) for x in tokens))
        self.vtx_idx += 1

    def parse_face(self, tokens):
        idx = []
        for tok in tokens:
            i = int(tok)
            idx.append(self.vtx_idx + i if i < 0 else i - 1)
        if len(idx) > 3:
            tris = [(idx[0], idx[j], idx[j + 1]) for j in range(1, len(idx) - 1)]
        else:
            tris = [idx]
        self.faces.extend(tris)
        for f in tris:
            tri = (self.vertexes[f[0]], self.vertexes[f[1]], self.vertexes[f[2]])
            self.triangles.append(tri)
            self.normals.append(calc_normal(tri))
            self.areas.append(triangle_area(tri))

    def read_obj(self, path):
        with open(path, 'r') as f:
            lines = _strip_comments(f.readlines())
        for line in lines:
            tokens = _tokens(line)
            if not tokens:
                continue
            if tokens[0] == 'v':
                self.parse_vertex(tokens[1:])
            elif tokens[0] == 'f':
                self.parse_face(tokens[1:])
            else:
                _log(f'{path}\n\tSkipping command \'{tokens[0]}\' ! '
                     f'\n\tParameters: {tokens[1:]}')


class Scene:
    """SDL scene (scene_reader.py:107-188).  Keywords: eye size ortho
    background ambient light npaths tonemapping seed object output.
    `background`, `npaths`, `tonemapping`, `output` and object `kt` are read
    but unused by the renderer, as in the reference; `seed` is unused by the
    reference and is this build's RNG key."""

    def __init__(self, path):
        self.eye = None
        self.width = None
        self.height = None
        self.ortho = None
        self.background = None
        self.ambient = None
        self.light_obj = None
        self.light_color = None
        self.npaths = None
        self.tonemapping = None
        self.seed = None
        self.objects = []
        self.path = path
        self.read_scene(path)

    def __repr__(self):
        return (f'<Scene\n\t eye = {self.eye}\n\t width = {self.width}'
                f'\n\t height = {self.height}\n\t ortho = {self.ortho}'
                f'\n\t background = {self.background}'
                f'\n\t ambient = {self.ambient}'
                f'\n\t light_obj = {self.light_obj}'
                f'\n\t light_color = {self.light_color}'
                f'\n\t npaths = {self.npaths}'
                f'\n\t tonemapping = {self.tonemapping}'
                f'\n\t seed = {self.seed}\n\t objects = {self.objects}\n>')

    def read_scene(self, path):
        try:
            with open(path, 'r') as f:
                lines = _strip_comments(f.readlines())
        except OSError:
            print('Could not open file!')
            raise
        base = dirname(path)
        for line in lines:
            t = _tokens(line)
            if not t:
                continue
            key = t[0]
            if key == 'eye':
                self.eye = [float(x) for x in t[1:4]]
            elif key == 'size':
                self.width, self.height = int(t[1]), int(t[2])
            elif key == 'ortho':
                self.ortho = [float(x) for x in t[1:5]]
            elif key == 'background':
                self.background = [float(x) for x in t[1:4]]
            elif key == 'ambient':
                self.ambient = float(t[1])
            elif key == 'light':
                self.light_obj = Obj(join(base, t[1]))
                self.light_color = [float(x) for x in t[2:6]]
            elif key == 'npaths':
                self.npaths = int(t[1])
            elif key == 'tonemapping':
                self.tonemapping = float(t[1])
            elif key == 'seed':
                self.seed = int(t[1])
            elif key == 'object':
                names = ('red', 'green', 'blue', 'ka', 'kd', 'ks', 'kt', 'n')
                obj = {'geometry': Obj(join(base, t[1]))}
                for i, name in enumerate(names):
                    obj[name] = float(t[2 + i])
                self.objects.append(obj)
            elif key == 'output':
                self.output = join(base, t[1])
            else:
                _log(f'Scene {path}\n\tSkipping command \'{key}\'!'
                     f' Parameters: {t[1:]}')
