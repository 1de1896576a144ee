#!/usr/bin/env python3
"""Command line mirror of the reference's main.py (main.py:125-139, :165-293).

    python -m pathtracerpython_amd.main objs/cornellroom.sdl --out out.png -r 1 -b 2

Same positional scene argument and flags (-r spp, -b bounces, --out,
--show-img); the whole spp x bounce loop runs on the GPU (render.py).  Extra
flags of this build: --seed (RNG key; default the SDL `seed`), --rr
(Russian roulette), --size W H (override the SDL size), --devices N (N GPUs:
one rank process per GPU, rows interleaved, one RCCL gather; launch.py),
--chunk-spp K [--checkpoint F] (the samples in launches of K, resumable from
F; progressive.py).  The
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
    parser.add_argument('--devices', type=int, default=1,
                        help='GPUs: one rank process each (torch.distributed over RCCL); '
                             'started here unless already under torch.distributed.run')
    parser.add_argument('--chunk-spp', type=int, default=None,
                        help='render the -r samples in launches of this many (progressive.py)')
    parser.add_argument('--checkpoint', default=None,
                        help='with --chunk-spp: .npz written after every chunk; a rerun '
                             'resumes from it')
    return parser.parse_args(argv)


def render_ranks(scene, args, W, H):
    """This rank's band (rows iy % world == rank) into a device tile, one
    RCCL gather to rank 0, the frame assembled there.  Returns (image array
    or None, f64 framebuffer) on rank 0, (None, None) elsewhere."""
    import torch
    import torch.distributed as dist
    from .distributed import assemble_bands_device, gather_tiles, max_band_rows
    from .launch import pg_timeout, rank_env
    from .render import Renderer, image_u8_device
    rank, local, world = rank_env()
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout())
    ok = False
    try:
        with Renderer(scene) as r:
            p = r.params(W, H, args.n_rays, args.n_bounces, args.seed, args.rr, out_f64=True,
                         row_step=world, row_phase=rank)
            tile = torch.zeros((max_band_rows(H, world), W, 3), dtype=torch.float64, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            r.render_device(p, tile.data_ptr(), s)
            tiles = gather_tiles(tile)
            if rank == 0:
                print(f'render: {W}x{H}, {args.n_rays} spp, {args.n_bounces} bounces on {world} '
                      f'GPUs, rank-0 kernel {r.last_kernel_ms():.3f} ms')
        if rank != 0:
            ok = True
            return None, None
        frame = assemble_bands_device(torch.stack(tiles),
                                      torch.empty((H, W, 3), dtype=torch.float64, device="cuda"))
        arr = None
        if W == H:
            img = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
            image_u8_device(frame.data_ptr(), W, H, True, img.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
            arr = img.cpu().numpy()
        ok = True
        return arr, frame.cpu().numpy()
    finally:
        # the closing barrier only on success: after an error here the peers
        # may be blocked in the gather and would never reach it (the parent,
        # launch.spawn_ranks, stops them once this rank exits non-zero)
        if ok:
            dist.barrier()
        dist.destroy_process_group()


def check_args(args):
    """Reject flag combinations before any rank process starts."""
    if args.checkpoint and not args.chunk_spp:
        raise SystemExit('--checkpoint needs --chunk-spp')
    if args.chunk_spp and args.devices > 1:
        raise SystemExit('--chunk-spp runs on one device (--devices 1)')


def main(argv=None):
    args = setup(argv)
    check_args(args)
    from .launch import rank_env, spawn_ranks, under_launcher
    if args.devices > 1 and not under_launcher():
        # one fresh process per GPU; this parent never touches the GPU
        raise SystemExit(spawn_ranks(args.devices, ['-m', 'pathtracerpython_amd.main'] +
                                     list(sys.argv[1:] if argv is None else argv)))
    from .render import Renderer
    from .scene_reader import Scene
    scene = Scene(args.scene)
    W, H = (args.size if args.size else (scene.width, scene.height))
    print(f'Number of objects: {len(scene.objects)}')
    print(f'Number of triangles: {sum(len(o["geometry"].triangles) for o in scene.objects)}')
    if args.show_scene or args.show_normals or args.show_screen or args.show_inter:
        print('note: the 3-D scene viewer (plot.py) is not part of this build; ignoring --show-*',
              file=sys.stderr)
    rank, _, world = rank_env()
    if world != args.devices:
        raise SystemExit(f'--devices {args.devices} but WORLD_SIZE={world}')
    if world > 1:
        arr, fb = render_ranks(scene, args, W, H)
        if rank != 0:
            return None
        return finish(args, arr, fb)
    with Renderer(scene) as r:
        chunks = []
        if args.chunk_spp:   # chunked, resumable (progressive.py)
            from .progressive import render_progressive
            from .render import image_u8

            def progress(d, n):
                chunks.append(d)
                print(f'samples {d}/{n}', flush=True)
            fb = render_progressive(r, W, H, args.n_rays, args.n_bounces, args.seed, args.rr,
                                    chunk_spp=args.chunk_spp, checkpoint=args.checkpoint,
                                    on_chunk=progress)
            arr = image_u8(fb) if W == H else None
        elif W == H:   # make_image on the device (utils.py:150-161)
            arr, fb = r.render_image(W, H, spp=args.n_rays, bounces=args.n_bounces,
                                     seed=args.seed, rr=args.rr, return_fb=True)
        else:        # the reference's placement for W != H (utils.py:154-156), on the host
            fb = r.render(W, H, spp=args.n_rays, bounces=args.n_bounces, seed=args.seed,
                          rr=args.rr)
            arr = None
        last = f'kernel {r.last_kernel_ms():.3f} ms' if chunks or not args.chunk_spp \
            else 'all samples from the checkpoint'
        print(f'render: {W}x{H}, {args.n_rays} spp, {args.n_bounces} bounces, {last}')
    return finish(args, arr, fb)


def finish(args, arr, fb):
    """--save-raw / --out / --show-img of a rendered frame (rank 0)."""
    from .utils import framebuffer_to_image
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
