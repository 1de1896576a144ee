"""bench.py --gpus N prints its headline line whatever the
secondary (device-frame, RCCL-gather) leg does.  The leg runs only after rank
0's line is complete; an exception on any rank is recorded under
frame_modes.device, a leg that never returns is ended by a watchdog that
prints the headline line first — one parsed JSON line, status 0, every time.
gloo world 2 on CPU (tests/bench_leg_worker.py); the GPU suite runs the same
injection through bench.py itself (test_gpu.py)."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

WORKER = os.path.join(ROOT, "tests", "bench_leg_worker.py")


def run(world, inject=None, timeout_s=None, delay0=0):
    env = dict(os.environ, PT_TEST_RANK0_DELAY=str(delay0))
    env.pop("PT_BENCH_INJECT_DEVICE_LEG", None)
    if inject:
        env["PT_BENCH_INJECT_DEVICE_LEG"] = inject
    if timeout_s:
        env["PT_BENCH_LEG_TIMEOUT_S"] = str(timeout_s)
    t0 = time.monotonic()
    res = subprocess.run([sys.executable, WORKER, "spawn", str(world)], env=env, capture_output=True,
                         text=True, timeout=240)
    lines = [ln for ln in res.stdout.splitlines() if ln.strip()]
    # rank 0's stdout is the one line (gloo's messages go to stderr)
    assert all(ln.startswith("{") for ln in lines), res.stdout[-2000:]
    return res, [json.loads(ln) for ln in lines], time.monotonic() - t0


def check_headline(line, world):
    assert line["n_gpus"] == world and line["value"] == 3052.0
    assert line["frame_modes"]["host"]["legs_ms"]["band_kernel_max"] == 5.49
    assert line["linf_vs_cpu_ref"] == 6.0e-8


def test_secondary_leg_runs():
    res, lines, _ = run(2)
    assert res.returncode == 0, res.stderr[-2000:]
    assert len(lines) == 1
    check_headline(lines[0], 2)
    assert lines[0]["frame_modes"]["device"]["legs_ms"]["gather"] == 3.0   # 1 + 2 over the ranks


@pytest.mark.parametrize("who", [0, 1])
def test_secondary_leg_raises(who):
    res, lines, dt = run(2, inject=f"raise:{who}")
    assert res.returncode == 0, res.stderr[-2000:]
    assert len(lines) == 1
    check_headline(lines[0], 2)
    err = lines[0]["frame_modes"]["device"]["error"]
    assert f"rank {who}: RuntimeError: injected device-leg failure" in err
    assert dt < 60


@pytest.mark.parametrize("who,delay0", [(0, 0), (1, 0), (1, 6)])
def test_secondary_leg_hangs(who, delay0):
    """The leg never returns on one rank (a collective that never completes):
    the watchdogs end every rank after the budget, rank 0's printing the
    headline line with the error first.  The budget counts from when every
    rank has reached the leg (delay0: rank 0 arrives later than the budget)."""
    res, lines, dt = run(2, inject=f"hang:{who}", timeout_s=4, delay0=delay0)
    assert res.returncode == 0, res.stderr[-2000:]
    assert len(lines) == 1
    check_headline(lines[0], 2)
    assert "no outcome within 4 s" in lines[0]["frame_modes"]["device"]["error"]
    assert dt < 90


def test_line_printed_once_on_a_single_rank():
    res, lines, _ = run(1, inject="raise:0")
    assert res.returncode == 0 and len(lines) == 1
    assert "rank 0: RuntimeError" in lines[0]["frame_modes"]["device"]["error"]


def test_duplicate_devices():
    """bench.py refuses a line when two ranks report one PCI bus id
    (VERDICT r05 #3); distinct ids pass."""
    import bench
    rk = [{"rank": r, "pci_bus_id": "0000:%02x:00" % b} for r, b in enumerate((0x05, 0x15, 0x05, 0x25, 0x15))]
    assert bench.duplicate_devices(rk) == ["0000:05:00", "0000:15:00"]
    assert bench.duplicate_devices(rk[:2]) == [] and bench.duplicate_devices(rk[:1]) == []
