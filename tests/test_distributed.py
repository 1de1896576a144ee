"""Multi-rank partition + gather (pathtracerpython_amd/distributed.py) over
gloo with world_size 2 on CPU; tiles are produced by the oracle here (the
HIP tile path is covered by the gpu tests), so this checks the interleaved
row partition, the gather and the assembly."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import CORNELL, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, spp, B, seed, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from oracle import oracle
    from pathtracerpython_amd import scene_reader
    from pathtracerpython_amd.distributed import (assemble, band_rows_of, gather_tiles,
                                                  max_band_rows)
    from pathtracerpython_amd.pack import pack_scene
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene_reader.VERBOSE = False
    pk = pack_scene(scene_reader.Scene(CORNELL))
    rows = band_rows_of(H, rank, world)
    pix = np.array([ix * H + iy for iy in rows for ix in range(W)], dtype=np.int64)
    cols, _ = oracle.render(pk, W, H, spp, B, seed, pixels=pix, threads=2)
    tile = np.zeros((max_band_rows(H, world), W, 3), dtype=np.float32)
    tile[:len(rows)] = cols.reshape(len(rows), W, 3)
    got = gather_tiles(torch.from_numpy(tile))
    if rank == 0:
        fb = assemble([t.numpy() for t in got], H)
        q.put(fb)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_assemble_full_frame(packed):
    from oracle import oracle
    from pathtracerpython_amd.render import from_list_order
    W, H, spp, B, seed = 12, 11, 2, 3, 9   # H not divisible by world: ragged bands
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, spp, B, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    fb = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _ = oracle.render(packed, W, H, spp, B, seed)
    ref = from_list_order(full, W, H).astype(np.float32)
    assert np.array_equal(fb, ref)
