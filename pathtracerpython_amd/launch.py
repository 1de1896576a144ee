"""Rank processes for the multi-GPU paths (bench.py, the CLI's --devices).

One process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm).  Under
torch.distributed.run the ranks come from the environment; a plain
`python bench.py --gpus N` / `python -m pathtracerpython_amd.main --devices N`
starts them itself with `spawn_ranks`: N fresh child processes of the same
command line with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set.  The parent
never touches the GPU (no HIP call, so no exec-after-GPU-init hazard) and
returns the first non-zero exit status of its children.  This replaces the
reference's only parallelism, the multiprocessing.Pool over rays
(main.py:197-231).
"""
import os
import socket
import subprocess
import sys


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher():
    return "WORLD_SIZE" in os.environ


PKG_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def spawn_ranks(n, argv, python=None):
    """Run `python argv...` as N rank processes on 127.0.0.1 (the package's
    parent directory on their PYTHONPATH, so `-m pathtracerpython_amd.main`
    resolves); returns the first non-zero exit status (0 when all succeed)."""
    port = free_port()
    procs = []
    pp = os.environ.get("PYTHONPATH", "")
    pp = PKG_PARENT + (os.pathsep + pp if pp else "")
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PYTHONPATH=pp)
        procs.append(subprocess.Popen([python or sys.executable] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def rank_env():
    """(rank, local_rank, world) from the environment (1 process: 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
