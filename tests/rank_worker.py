"""One rank of tests/test_launch.py (CPU, gloo): started by
pathtracerpython_amd.launch.spawn_ranks exactly as bench.py / the CLI start
their GPU ranks.  Renders this rank's interleaved row band with the CPU
oracle (standing in for the HIP tile, which needs a GPU), gathers the tiles to
rank 0 with distributed.gather_tiles and assembles the frame with
distributed.deinterleave (equal bands) or distributed.assemble (ragged bands;
on a GPU both are pt_assemble_bands_device);
rank 0 saves it to argv[1].  With PT_TEST_FAIL_RANK=r, rank r raises right
after the rendezvous (the others go on into the gather and block there): the
fail-fast test of launch.spawn_ranks."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import oracle  # noqa: E402
from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.distributed import (assemble, band_rows_of, deinterleave,  # noqa: E402
                                              gather_tiles, max_band_rows)
from pathtracerpython_amd.launch import pg_timeout, rank_env  # noqa: E402
from pathtracerpython_amd.pack import pack_scene  # noqa: E402


def main():
    out, W, H, spp, B, seed = sys.argv[1], *map(int, sys.argv[2:7])
    rank, local, world = rank_env()
    dist.init_process_group("gloo", timeout=pg_timeout())
    assert dist.get_rank() == rank and dist.get_world_size() == world
    if os.environ.get("PT_TEST_FAIL_RANK") == str(rank):
        raise RuntimeError(f"rank {rank}: injected failure after the rendezvous")
    scene_reader.VERBOSE = False
    pk = pack_scene(scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl")))
    rows = band_rows_of(H, rank, world)
    pix = np.array([ix * H + iy for iy in rows for ix in range(W)], dtype=np.int64)
    cols, _ = oracle.render(pk, W, H, spp, B, seed, pixels=pix, threads=2)
    tile = torch.zeros((max_band_rows(H, world), W, 3), dtype=torch.float64)
    tile[:len(rows)] = torch.from_numpy(cols.reshape(len(rows), W, 3))
    tiles = gather_tiles(tile)
    if rank == 0:
        if H % world == 0:   # equal bands: the strided device-style copy
            frame = deinterleave(torch.stack(tiles), torch.empty((H, W, 3), dtype=torch.float64)).numpy()
        else:                # ragged bands (pt_assemble_bands_device on a GPU)
            frame = assemble([t.numpy() for t in tiles], H)
        np.save(out, frame)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
