"""Rank processes for the multi-GPU paths (bench.py, the CLI's --devices).

One process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm).  Under
torch.distributed.run the ranks come from the environment; a plain
`python bench.py --gpus N` / `python -m pathtracerpython_amd.main --devices N`
starts them itself with `spawn_ranks`: N fresh child processes of the same
command line with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set.  The parent
never touches the GPU (no HIP call, so no exec-after-GPU-init hazard).  It
polls its children and, on the first non-zero exit, terminates the others
(a rank blocked in the rendezvous or a collective would otherwise wait for
the backend's timeout) and returns that status.  This replaces the
reference's only parallelism, the multiprocessing.Pool over rays
(main.py:197-231), whose worker errors surface at `.get()` (main.py:204,228).
"""
import datetime
import os
import socket
import subprocess
import sys
import time

# rendezvous / collective timeout of the rank process groups (bench.py,
# main.py): a job here is seconds long, so a rank that waits this long on its
# peers has lost one of them
PG_TIMEOUT_S = float(os.environ.get("PT_PG_TIMEOUT_S", "300"))


def pg_timeout():
    return datetime.timedelta(seconds=PG_TIMEOUT_S)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher():
    return "WORLD_SIZE" in os.environ


PKG_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stop(procs, grace=5.0):
    """Terminate the still-running children (SIGTERM, then SIGKILL after
    `grace` seconds) and reap them."""
    live = [p for p in procs if p.poll() is None]
    for p in live:
        p.terminate()
    deadline = time.monotonic() + grace
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def spawn_ranks(n, argv, python=None, poll_s=0.05):
    """Run `python argv...` as N rank processes on 127.0.0.1 (the package's
    parent directory on their PYTHONPATH, so `-m pathtracerpython_amd.main`
    resolves).  Returns 0 when all succeed; on the first non-zero exit the
    remaining ranks are terminated and that status is returned."""
    port = free_port()
    procs = []
    pp = os.environ.get("PYTHONPATH", "")
    pp = PKG_PARENT + (os.pathsep + pp if pp else "")
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       PYTHONPATH=pp)
            procs.append(subprocess.Popen([python or sys.executable] + list(argv), env=env))
        while True:
            rcs = [p.poll() for p in procs]
            bad = next((rc for rc in rcs if rc not in (None, 0)), None)
            if bad is not None:
                _stop(procs)
                return bad
            if all(rc == 0 for rc in rcs):
                return 0
            time.sleep(poll_s)
    finally:
        _stop(procs)   # (KeyboardInterrupt, a failed Popen: no orphans)


def init_gloo():
    """The ranks' gloo process group (the control plane), with gloo's
    connection messages (C++ writes to stdout) sent to stderr: rank 0's stdout
    carries the one result line of bench.py."""
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        dist.init_process_group("gloo", timeout=pg_timeout())
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def rank_env():
    """(rank, local_rank, world) from the environment (1 process: 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
