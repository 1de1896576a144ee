"""One rank of tests/test_launch.py::test_render_distributed_host_errors
(CPU, gloo): distributed.render_distributed(transport="host") when a rank
cannot open the shared host frame.  argv: out_prefix, who —
  "rank0": rank 0's creation fails (on a CPU box pt_host_map has no device);
  "rank1": rank 0 creates the frame (shared memory only), rank 1's open
           raises.
Each rank writes the error it got (or "no error") to out_prefix.<rank>; the
test checks that every rank raised the same error, in seconds (no rank left
in a barrier, rank 0 not spinning on the ready flags)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch.distributed as dist  # noqa: E402

from pathtracerpython_amd import distributed  # noqa: E402
from pathtracerpython_amd._abi import make_params  # noqa: E402
from pathtracerpython_amd._native import NativeError  # noqa: E402
from pathtracerpython_amd.launch import pg_timeout, rank_env  # noqa: E402


class StubRenderer:   # params only: no rank gets as far as rendering
    def params(self, width, height, spp, bounces, seed, rr=False, rr_depth=3, **kw):
        return make_params(width, height, spp, bounces, seed or 0, **kw)


def main():
    out, who = sys.argv[1], sys.argv[2]
    rank, _, world = rank_env()
    dist.init_process_group("gloo", timeout=pg_timeout())
    if who == "rank1":
        real = distributed.HostFrame

        class Failing(real):
            def __init__(self, *a, create=False, **kw):
                if rank == 1:
                    raise OSError("injected: rank 1 cannot open the frame")
                super().__init__(*a, create=create, map_device=False, **kw)
        distributed.HostFrame = Failing
    try:
        distributed.render_distributed(StubRenderer(), 8, 6, 1, 1, 9, transport="host")
        msg = "no error"
    except NativeError as e:
        msg = str(e)
    with open(f"{out}.{rank}", "w") as f:
        f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
