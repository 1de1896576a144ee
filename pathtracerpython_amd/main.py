#!/usr/bin/env python3
"""Command line mirror of the reference's main.py (main.py:125-139, :165-293).

    python -m pathtracerpython_amd.main objs/cornellroom.sdl --out out.png -r 1 -b 2

Same positional scene argument and flags (-r spp, -b bounces, --out,
--show-img); the whole spp x bounce loop runs on the GPU (render.py).  Extra
flags of this build: --seed (RNG key; default the SDL `seed`), --rr
(Russian roulette), --size W H (override the SDL size), --devices.  The
reference's interactive 3-D viewer flags (--show-scene, --show-normals,
--show-screen, --show-inter -> plot.py) are accepted and ignored with a
notice: the pyqtgraph viewer is out of scope.
"""
import argparse
import sys

import numpy as np


def setup(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('scene', help='SDL scene')
    parser.add_argument('--out', help='Output image')
    parser.add_argument('-r', dest='n_rays', type=int, default=1, help='Number of rays per pixel')
    parser.add_argument('-b', dest='n_bounces', type=int, default=1, help='Number of bounces')
    parser.add_argument('--show-img', default=False, action='store_true')
    parser.add_argument('--show-scene', default=False, action='store_true')
    parser.add_argument('--show-normals', default=False, action='store_true')
    parser.add_argument('--show-screen', default=False, action='store_true')
    parser.add_argument('--show-inter', default=False, action='store_true')
    parser.add_argument('--seed', type=int, default=None, help='RNG key (default: SDL seed)')
    parser.add_argument('--rr', default=False, action='store_true', help='Russian roulette')
    parser.add_argument('--size', type=int, nargs=2, metavar=('W', 'H'), default=None)
    parser.add_argument('--save-raw', default=None,
                        help='also save the float framebuffer (.npy, before normalisation)')
    return parser.parse_args(argv)


def main(argv=None):
    args = setup(argv)
    from .render import Renderer
    from .scene_reader import Scene
    from .utils import framebuffer_to_image
    scene = Scene(args.scene)
    W, H = (args.size if args.size else (scene.width, scene.height))
    print(f'Number of objects: {len(scene.objects)}')
    print(f'Number of triangles: {sum(len(o["geometry"].triangles) for o in scene.objects)}')
    if args.show_scene or args.show_normals or args.show_screen or args.show_inter:
        print('note: the 3-D scene viewer (plot.py) is not part of this build; ignoring --show-*',
              file=sys.stderr)
    with Renderer(scene) as r:
        if W == H:   # make_image on the device (utils.py:150-161)
            arr, fb = r.render_image(W, H, spp=args.n_rays, bounces=args.n_bounces,
                                     seed=args.seed, rr=args.rr, return_fb=True)
        else:        # the reference's placement for W != H (utils.py:154-156), on the host
            fb = r.render(W, H, spp=args.n_rays, bounces=args.n_bounces, seed=args.seed,
                          rr=args.rr)
            arr = None
        print(f'render: {W}x{H}, {args.n_rays} spp, {args.n_bounces} bounces, '
              f'kernel {r.last_kernel_ms():.3f} ms')
    if args.save_raw:
        np.save(args.save_raw, fb)
    if arr is not None:
        from PIL import Image
        im = Image.fromarray(arr)
    else:
        im = framebuffer_to_image(fb)
    if args.out is not None:
        im.save(args.out)
    if args.show_img:
        im.show()
    return fb


if __name__ == '__main__':
    main()
