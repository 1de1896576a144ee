"""One rank of tests/test_gpu.py::test_rccl_gather_on_the_device (GPU): the
device-frame transport's collective as bench.py runs it — the default group
gloo (the control plane), an RCCL group made for the gather
(`dist.new_group(backend="nccl")`), one dist.gather of a device tile rendered
by this rank's GPU to rank 0.  On a one-GPU box only world 1 is possible (RCCL
refuses two ranks on one device), so the gather moves rank 0's own tile; it
still runs RCCL's communicator set-up and gather kernel on the hardware.
argv: out.npy"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pathtracerpython_amd import scene_reader  # noqa: E402
from pathtracerpython_amd.distributed import assemble_bands_device, max_band_rows  # noqa: E402
from pathtracerpython_amd.launch import init_gloo, pg_timeout, rank_env  # noqa: E402
from pathtracerpython_amd.render import Renderer  # noqa: E402


def main():
    rank, local, world = rank_env()
    torch.cuda.set_device(local)
    init_gloo()
    grp = dist.new_group(backend="nccl", timeout=pg_timeout())
    scene_reader.VERBOSE = False
    W = H = 64
    with Renderer(scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl"))) as r:
        p = r.params(W, H, 4, 3, 9, row_step=world, row_phase=rank)
        rows = max_band_rows(H, world)
        tile = torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda")
        r.render_device(p, tile.data_ptr(), torch.cuda.current_stream().cuda_stream)
        gathered = torch.empty((world, rows, W, 3), dtype=torch.float32, device="cuda") if rank == 0 else None
        dist.gather(tile, gather_list=list(gathered.unbind(0)) if rank == 0 else None, dst=0, group=grp)
        if rank == 0:
            frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
            assemble_bands_device(gathered, frame)
            np.save(sys.argv[1], frame.cpu().numpy())
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group(grp)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
