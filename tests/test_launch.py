"""The self-spawn multi-rank path of bench.py and the CLI (--gpus N /
--devices N without torch.distributed.run): launch.spawn_ranks starts N fresh
rank processes with the rendezvous in their environment; here worlds 2 and 8
over gloo on CPU, tiles from the oracle (tests/rank_worker.py), device-style
assembly with distributed.deinterleave."""
import os

import numpy as np
import pytest

from conftest import ROOT


@pytest.mark.parametrize("world,H", [(2, 12), (8, 16), (8, 13)])
def test_spawn_ranks_gloo_frame(tmp_path, packed, world, H):
    """world 8 = the driver's 8-GPU run (here gloo over CPU processes); H = 13:
    ragged bands of 2 and 1 rows."""
    from oracle import oracle
    from pathtracerpython_amd.launch import spawn_ranks
    from pathtracerpython_amd.render import from_list_order
    W, spp, B, seed = 10, 2, 3, 9
    out = str(tmp_path / "frame.npy")
    rc = spawn_ranks(world, [os.path.join(ROOT, "tests", "rank_worker.py"), out,
                             str(W), str(H), str(spp), str(B), str(seed)])
    assert rc == 0
    full, _ = oracle.render(packed, W, H, spp, B, seed)
    assert np.array_equal(np.load(out), from_list_order(full, W, H))


def test_spawn_reports_failure():
    from pathtracerpython_amd.launch import spawn_ranks
    assert spawn_ranks(2, ["-c", "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"]) == 3


def test_spawn_fails_fast_when_a_rank_dies_after_rendezvous(tmp_path, monkeypatch):
    """Rank 1 raises after init_process_group while rank 0 goes on into the
    gather: the parent must see rank 1's status and stop rank 0 within
    seconds, not at the process group's timeout (reference: worker errors
    re-raised at .get(), main.py:204)."""
    import time
    from pathtracerpython_amd.launch import spawn_ranks
    monkeypatch.setenv("PT_TEST_FAIL_RANK", "1")
    monkeypatch.setenv("PT_PG_TIMEOUT_S", "600")   # a blocked gather would wait this long
    t0 = time.monotonic()
    rc = spawn_ranks(2, [os.path.join(ROOT, "tests", "rank_worker.py"), str(tmp_path / "f.npy"),
                         "10", "12", "2", "3", "9"])
    dt = time.monotonic() - t0
    assert rc != 0
    assert dt < 60, dt
    assert not (tmp_path / "f.npy").exists()


def test_spawn_stops_siblings_of_a_failed_rank():
    """A rank that never exits on its own (blocked) is terminated once a
    sibling fails."""
    import time
    from pathtracerpython_amd.launch import spawn_ranks
    t0 = time.monotonic()
    rc = spawn_ranks(2, ["-c", "import os, sys, time\n"
                               "if os.environ['RANK'] == '1': sys.exit(5)\n"
                               "time.sleep(600)"])
    assert rc == 5 and time.monotonic() - t0 < 30


def test_deinterleave_matches_assemble():
    import torch
    from pathtracerpython_amd.distributed import assemble, deinterleave
    rs = np.random.RandomState(0)
    for world, rows in ((1, 5), (2, 4), (4, 3), (8, 2)):
        g = torch.from_numpy(rs.rand(world, rows, 7, 3))
        out = deinterleave(g, torch.empty((world * rows, 7, 3), dtype=torch.float64))
        assert np.array_equal(out.numpy(), assemble([t.numpy() for t in g], world * rows))


def test_cli_devices_flag_parses():
    from pathtracerpython_amd.main import setup
    a = setup(["scene.sdl", "--devices", "4", "-r", "8"])
    assert a.devices == 4 and a.n_rays == 8


@pytest.mark.parametrize("world,H", [(2, 12), (8, 13)])
def test_host_frame_protocol_gloo(tmp_path, packed, world, H):
    """distributed.HostFrame across rank processes without a GPU: the shared
    /dev/shm frame, the ready flags, pt_wait_flags and the two-slot rotation
    (each step a different seed) — rank 0's frames equal the oracle's."""
    from oracle import oracle
    from pathtracerpython_amd.launch import spawn_ranks
    from pathtracerpython_amd.render import from_list_order
    W, spp, B, seed, steps = 10, 2, 3, 9, 5
    out = str(tmp_path / "frames.npy")
    rc = spawn_ranks(world, [os.path.join(ROOT, "tests", "rank_worker_hostframe.py"), out,
                             str(W), str(H), str(spp), str(B), str(seed), str(steps), "cpu"])
    assert rc == 0
    got = np.load(out)
    assert got.shape == (steps, H, W, 3)
    for s in range(steps):
        full, _ = oracle.render(packed, W, H, spp, B, seed + s)
        assert np.array_equal(got[s], from_list_order(full, W, H).astype(np.float32)), s


def test_host_frame_file_lifecycle():
    """Rank 0 creates the shared file exclusively and removes it on close;
    the slots and the rows of each band are where render() puts them."""
    from pathtracerpython_amd.distributed import HostFrame
    name = HostFrame.new_name()
    a = HostFrame(13, 10, 4, 0, name, create=True, map_device=False)
    with pytest.raises(FileExistsError):
        HostFrame(13, 10, 4, 0, name, create=True, map_device=False)
    b = HostFrame(13, 10, 4, 3, name, map_device=False)
    assert b.band_rows == [11, 7, 3] and a.band_rows == [12, 8, 4, 0]
    b.frame(1)[0, 0, 0] = 7.0
    assert a.frame(3)[0, 0, 0] == 7.0 and a.frame(0)[0, 0, 0] == 0.0   # 2 slots
    assert a.band_target(0) == (None, 0)   # no device mapping
    with pytest.raises(ValueError):
        a.render(None, None, 0, None)
    b.close()
    a.close()
    assert not os.path.exists(os.path.join("/dev/shm", name))


@pytest.mark.parametrize("who,match", [("rank0", "rank 0: NativeError: pt_host_map failed"),
                                       ("rank1", "rank 1: OSError: injected")])
def test_render_distributed_host_errors(tmp_path, who, match):
    """render_distributed(transport="host") exchanges the frame's
    open errors before any rank renders or waits, so a failure on rank 0
    (creation) or on another rank (open) raises the same error on every rank
    within seconds — not a barrier or a flag wait until the timeout."""
    import time
    import torch
    from pathtracerpython_amd.launch import spawn_ranks
    if torch.cuda.is_available() and who == "rank0":
        pytest.skip("a GPU is visible: rank 0's pt_host_map would succeed")
    out = str(tmp_path / "err")
    t0 = time.monotonic()
    rc = spawn_ranks(2, [os.path.join(ROOT, "tests", "rank_worker_hf_error.py"), out, who])
    assert rc == 0 and time.monotonic() - t0 < 60
    msgs = [open(f"{out}.{r}").read() for r in range(2)]
    assert msgs[0] == msgs[1] and match in msgs[0], msgs
