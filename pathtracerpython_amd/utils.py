"""Camera and image helpers with the reference's semantics (utils.py:55-69,
150-161).  Host-side, outside the timed hot path (the camera is computed on
the device inside the render kernel; these are for drop-in callers)."""
import numpy as np


def make_screen_pts(x0, y0, x1, y1, n_pxls_x, n_pxls_y):
    """Screen points (x, y, 0), x outer / y inner — utils.py:64-69."""
    return [(x, y, 0) for x in np.linspace(x0, x1, n_pxls_x)
            for y in np.linspace(y0, y1, n_pxls_y)]


def make_rays(start_pt, pts):
    """(origin, pt - origin), direction not normalised — utils.py:55-61."""
    return [(start_pt, np.array(pt) - np.array(start_pt)) for pt in pts]


def normalize_to_uint8(mat):
    """Global min-max -> x255 -> uint8 truncation, utils.py:158-161."""
    mat = np.asarray(mat, dtype=np.float64)
    mat = mat - np.min(mat)
    mat = mat / np.max(mat)
    mat = mat * 255
    return mat.astype('uint8')


def make_image(x1, y1, x2, y2, width, height, intersections):
    """utils.py:150-161: list entry `counter` goes to mat[H-1-(counter % W),
    counter // W] (correct orientation only when W == H, as in the
    reference), then min-max normalised to uint8.  Returns a PIL image."""
    from PIL import Image
    mat = np.zeros((height, width, 3), dtype='float64')
    for counter, (color, _) in enumerate(intersections):
        mat[height - 1 - counter % width, counter // width] = np.array(color)
    return Image.fromarray(normalize_to_uint8(mat))


def framebuffer_to_image(fb):
    """PIL image of a render() framebuffer, as make_image would produce from
    the same colours (identical placement for square images)."""
    from PIL import Image
    fb = np.asarray(fb)
    H, W = fb.shape[:2]
    if H == W:
        return Image.fromarray(normalize_to_uint8(fb))
    from .render import to_list_order
    return make_image(0, 0, 0, 0, W, H, [(c, None) for c in to_list_order(fb)])
