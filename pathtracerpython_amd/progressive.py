"""Chunked, resumable renders: checkpoint / resume of a long spp run
(SURVEY.md §5).

The reference has no checkpoint; its natural boundary is the per-pixel sum
over samples, `pixel_color_list` (main.py:185, :271), divided by the sample
count at the end (main.py:274-280).  Here a render of `spp` samples runs as
consecutive launches of `chunk_spp` samples each (pt_render_params'
sample_begin, include/pt_capi.h): the keyed RNG makes sample s of a pixel the
same draw whichever launch renders it, so the chunks of a run are the samples
of the one-launch render, split.  The host keeps the float64 running sum
(chunk mean x chunk samples) and, given a checkpoint path, writes it after
every chunk; a run started again with the same scene and parameters resumes
after the last chunk written.

Exactness: a chunked frame agrees with the one-launch frame to ~1e-15
relative (only the order in which a pixel's samples are summed differs); a
resumed run is bit-identical to the same chunking run without interruption.
"""
import hashlib
import json
import os

import numpy as np


def scene_fingerprint(packed):
    """sha256 over the packed scene arrays the kernels read (pack.py)."""
    h = hashlib.sha256()
    for a in (packed.tri_v, packed.tri_n, packed.tri_area, packed.tri_obj, packed.mat,
              packed.eye, packed.ortho, packed.light_rgb):
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    h.update(np.float64(packed.ambient).tobytes())
    return h.hexdigest()


class Checkpoint:
    """The running sum of a chunked render in one .npz file (written whole
    to a temporary name, then renamed over the old one: a crash mid-write
    leaves the previous checkpoint)."""

    def __init__(self, path):
        self.path = str(path)

    def load(self, key):
        """(sum (H, W, 3) f64, samples done) when the file holds a run with
        this key; None when there is no file.  A file of another run is an
        error, not a silent restart."""
        if not os.path.exists(self.path):
            return None
        with np.load(self.path, allow_pickle=False) as z:
            got = json.loads(str(z["key"]))
            if got != key:
                raise ValueError(f"checkpoint {self.path} belongs to another render: {got} != {key}")
            return np.array(z["sum"], dtype=np.float64), int(z["done"])

    def save(self, key, acc, done):
        tmp = self.path + ".tmp.npz"
        np.savez(tmp, key=np.array(json.dumps(key, sort_keys=True)), sum=acc,
                 done=np.int64(done))
        os.replace(tmp, self.path)

    def remove(self):
        if os.path.exists(self.path):
            os.remove(self.path)


def render_progressive(renderer, width=None, height=None, spp=1, bounces=1, seed=None, rr=False,
                       rr_depth=3, chunk_spp=16, checkpoint=None, max_chunks=None,
                       on_chunk=None):
    """Render `spp` samples per pixel in launches of `chunk_spp`.

    renderer: a render.Renderer.  checkpoint: a path (or Checkpoint) to
    resume from and write after each chunk.  max_chunks: stop after this many
    chunks in this call (the run is then incomplete: returns None).
    on_chunk(done, spp): progress callback after each chunk.
    Returns the framebuffer (H, W, 3) float64 — the mean over all samples —
    once every sample is done."""
    spp, chunk_spp = int(spp), int(chunk_spp)
    if spp < 1 or chunk_spp < 1:
        raise ValueError("spp and chunk_spp must be >= 1")
    p0 = renderer.params(width, height, spp, bounces, seed, rr, rr_depth, out_f64=True)
    W, H = p0.width, p0.height
    key = {"scene": scene_fingerprint(renderer.packed), "width": W, "height": H, "spp": spp,
           "bounces": int(bounces), "seed": int(p0.seed), "rr": bool(rr),
           "rr_depth": int(rr_depth), "chunk_spp": chunk_spp}
    ck = checkpoint if isinstance(checkpoint, Checkpoint) or checkpoint is None \
        else Checkpoint(checkpoint)
    state = ck.load(key) if ck is not None else None
    acc, done = state if state is not None else (np.zeros((H, W, 3), dtype=np.float64), 0)
    if acc.shape != (H, W, 3) or not 0 <= done <= spp:
        raise ValueError(f"checkpoint state does not fit the render: {acc.shape}, {done} samples")
    chunks = 0
    while done < spp:
        if max_chunks is not None and chunks >= max_chunks:
            return None
        n = min(chunk_spp, spp - done)
        fb = renderer.render(W, H, n, bounces, seed, rr, rr_depth, out_f64=True,
                             sample_begin=done)
        acc += fb * n
        done += n
        chunks += 1
        if ck is not None:
            ck.save(key, acc, done)
        if on_chunk is not None:
            on_chunk(done, spp)
    return acc / spp
