#!/usr/bin/env python3
"""Benchmark: Mega path-samples/sec on the Cornell box (BASELINE.json metric).

One step = one render of a fixed frame (the whole main.py:186-280 loop:
every pixel, every sample, every bounce, the /spp average) with the scene
resident in HBM, ending with the framebuffer in HOST memory — SURVEY.md
§8(d)'s metric is N_ps / render wall-time including the kernel and the D2H.
Two frame transports (--frame):
  host (default)  every rank's render writes its band straight into its rows
                  of one page-locked frame in /dev/shm shared by the ranks of
                  the node (distributed.HostFrame): the framebuffer crosses
                  PCIe while the kernel runs, each GPU over its own link; a
                  per-rank flag written on the render's stream (pt_signal)
                  tells rank 0 the frame is complete (pt_wait_flags).  Frames
                  rotate over 2 slots, so the next step's render is queued
                  before rank 0 waits for this one.
  device          each rank renders into a device tile; N > 1: ONE gather of
                  the tiles to rank 0 (RCCL over xGMI) and the device band
                  assembly (pt_assemble_bands_device); then rank 0's PCIe copy
                  of the frame to pinned host memory.
The other transport is measured after the headline one with the same steps
and reported under `frame_modes`, with per-leg times (max / min band kernel
over ranks; device: gather, assembly, D2H on rank 0's stream).

Workloads (--config, BASELINE.json configs):
  k2 (default)  Cornell 512x512, 64 spp, 4 bounces (configs[1], the config the
                metric is quoted on).
  k4            Cornell 4096x4096, --spp (default 64; BASELINE's 4096 takes
                ~3.2 s per step on 8 GPUs), 4 bounces: the K4 frame shape.
  k5            100k-triangle synthetic mesh 1024x1024, 256 spp, 4 bounces
                (the BVH / wavefront path).
Scaling (--scaling): strong (default) — the frame is fixed and N GPUs split
its rows interleaved (rank r renders iy % N == r), so the 1/2/4/8 curve is
tile-parallel scaling of one frame; weak (k2 only) — a 512 x (512 N) frame,
512 rows per GPU.

Multi-GPU: one process per GPU over torch.distributed (backend nccl = RCCL).
Launched by torch.distributed.run (RANK / WORLD_SIZE in the environment), or,
for `python bench.py --gpus N`, by this script itself: the parent spawns N
fresh rank processes (it never touches the GPU) and exits with their status.

Printed on rank 0: one JSON line with the driver's fields plus
  roofline     : the dominant kernel's achieved rate against its roof.
                 k2/k4: k_render, FP32 VALU: reference-semantics ray-triangle
                 tests (exact, from a counting launch) x 47 FLOP (SURVEY.md
                 §8d) / HIP-event kernel time, vs 157.3 TF/s.  k5: the BVH
                 walk kernel with the larger own time (a profiling launch
                 that runs the two walks one after the other), L2 roof
                 (~34.5 TB/s):
                 algorithmic bytes (node + leaf records + query records, from
                 a counting launch) / its HIP-event time.  traffic: rocprofv3
                 PMC bytes per launch from profiles/, only when measured on the
                 current kernel sources (tests/test_profiles.py).
  cpu_baseline : the C oracle (f64 restatement of the reference loop, test
                 infrastructure) on this host's CPU share, on a bounded sample
  linf_vs_cpu_ref : per-pixel L-inf of this run's f32 framebuffer (as timed,
                 read from host memory) vs the oracle — k2: every pixel of the
                 frame (the oracle frame the cpu_baseline leg renders), with
                 the counts of pixels above 1e-6 and 1e-4; k4/k5: a pixel sample
"""
import argparse
import hashlib
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 9
FLOP_PER_TEST = 47          # Moller-Trumbore with line semantics
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector (VALU) peak
HBM_PEAK_GBS = 8000.0
# MI355X_MICROARCH.md "L2 (per XCD)": the L2's rate, ~34.5 TB/s aggregate —
# the roof of the K5 walks, whose BVH records are served from the XCDs' L2
L2_PEAK_GBS = 34500.0
# MI355X_MICROARCH.md "Indexed rows": rows served from the XCDs' L2, gathered
# by every CU into LDS, 16.8-18.8 TB/s chip-wide (a measured lower bound of
# what a gather reaches; reported as a secondary figure)
L2_GATHER_GBS = 18800.0
METRIC = "Mega path-samples/sec on Cornell box; per-pixel L-inf vs CPU ref"

CONFIGS = {
    "k2": dict(W=512, H=512, spp=64, bounces=4, steps=200, warmup=5,
               workload="Cornell box (objs/cornellroom.sdl) 512x512 64 spp 4 bounces"),
    "k4": dict(W=4096, H=4096, spp=64, bounces=4, steps=10, warmup=1,
               workload="Cornell box 4096x4096 (K4 frame shape) {spp} spp 4 bounces"),
    "k5": dict(W=1024, H=1024, spp=256, bounces=4, steps=3, warmup=1,
               workload="Synthetic 100k-triangle random mesh in the Cornell box 1024x1024 "
                        "256 spp 4 bounces (BVH, wavefront kernels)"),
}
# k5 walk kernels' algorithmic bytes: a 4-wide node record
# (QNode) per node visit, a leaf-unit record (UnitC) per leaf-unit test, and
# per shadow ray (one query of the one-ray walks) its fields of the query
# record read (origin, group, direction, range bracket, key2/leak: 44 B), the
# list entry (4 B) and its result written (<= 8 B)
QNODE_B, UNITC_B, SHADOWQ_B, SHADOW_RES_B = 64, 64, 48, 8
# closest walks: per query the whole WfClosestQ record read (48 B: origin,
# group, direction, the uniform units' candidates), the list entry (4 B) and
# the result written (a1, a2, b1, i1: 16 B)
CLOSESTQ_B, CLOSEST_RES_B = 52, 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="k2")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--spp", type=int, default=None, help="override spp (k4)")
    ap.add_argument("--frame", choices=("host", "device"), default="host",
                    help="how the framebuffer reaches host memory (module docstring)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip L-inf vs the CPU oracle")
    ap.add_argument("--no-secondary", action="store_true",
                    help="do not measure the other frame transport after the headline one")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    a.steps = c["steps"] if a.steps is None else a.steps
    a.warmup = c["warmup"] if a.warmup is None else a.warmup
    if a.scaling == "weak" and a.config != "k2":
        ap.error("--scaling weak is defined for k2 only")
    return a


def source_sha():
    """Content hash of the kernel sources on disk (pathtracerpython_amd/build.py;
    the id every build carries)."""
    from pathtracerpython_amd.build import source_sha as sha
    return sha()


def lib_build_id():
    """The id of the library this process loaded (pt_build_id): the sources
    the measured binary was compiled from.  _native.lib() refuses a library
    whose id differs from the sources on disk unless PT_ALLOW_FOREIGN_BUILD=1
    (dev variants), so the line always names the binary it measured."""
    from pathtracerpython_amd import _native
    return _native.build_id()


def load_traffic_record(config):
    """profiles/traffic_<config>.json when measured on the loaded library's
    sources, else None."""
    p = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    return d if d.get("source_sha") == lib_build_id() else None


def load_traffic(config):
    p = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    if d.get("source_sha") != lib_build_id():
        return None, (f"stale: {p} was measured on kernel sources {d.get('source_sha')}, "
                      f"the loaded library is {lib_build_id()}")
    return d.get("hbm_bytes_per_launch"), d.get("source")


def device_identity():
    """This rank's GPU as the driver can check it: the torch device index and
    the PCI location (domain:bus:device) and UUID of that device."""
    import torch
    dev = torch.cuda.current_device()
    pr = torch.cuda.get_device_properties(dev)
    return {"local_device": dev,
            "pci_bus_id": "%04x:%02x:%02x" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id),
            "uuid": str(getattr(pr, "uuid", ""))}


def rank_records(me, dist, world):
    """Every rank's record (rank order), on every rank (control group: gloo)."""
    if world == 1:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def duplicate_devices(ranks):
    """PCI bus ids that more than one rank reports (a rank-to-device mistake:
    N ranks on fewer than N GPUs would still print a plausible line)."""
    seen, dup = set(), []
    for r in ranks:
        b = r["pci_bus_id"]
        if b in seen and b not in dup:
            dup.append(b)
        seen.add(b)
    return dup


def rank_legs(vals, dist, world):
    """(max, min) over ranks of this rank's value (control group: gloo)."""
    if world == 1:
        return vals, vals
    import torch
    t = torch.tensor([vals, -vals], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(-t[1])


class LineOut:
    """Rank 0's one JSON line, printed exactly once: by the main thread when
    the job completes, or by the secondary leg's watchdog (bounded_leg)."""

    def __init__(self):
        self.lock = threading.Lock()
        self.printed = False

    def emit(self, result):
        with self.lock:
            if self.printed or result is None:
                return False
            print(json.dumps(result), flush=True)
            self.printed = True
            return True


def injected_leg(run, rank):
    """PT_BENCH_INJECT_DEVICE_LEG=raise:R | hang:R (tests only): rank R's
    secondary leg raises / never returns instead of running (the failure
    modes of a collective that has never run on the hardware)."""
    spec = os.environ.get("PT_BENCH_INJECT_DEVICE_LEG")
    if not spec:
        return run
    how, _, who = spec.partition(":")
    if int(who or 0) != rank:
        return run
    if how == "raise":
        def bad():
            raise RuntimeError("injected device-leg failure (PT_BENCH_INJECT_DEVICE_LEG)")
        return bad
    if how == "hang":
        return lambda: threading.Event().wait()
    raise ValueError(f"PT_BENCH_INJECT_DEVICE_LEG={spec!r}: raise:R or hang:R")


def bounded_leg(run, timeout_s, name, rank, world, dist, on_timeout, poll_s=0.2, cleanup=None):
    """Run the secondary transport `run()` on every rank AFTER the headline
    result is complete, bounded and non-fatal: returns
    (value or None, error or None).

    Each rank posts its outcome ("ok" or its error) to the process group's
    key-value store — not through a collective, so a rank that failed before
    a collective its peers are blocked in still gets its error out.  A monitor
    thread on every rank watches the store and the clock:
      * every rank posted "ok": the leg's value is returned;
      * some rank posted an error, or no outcome within timeout_s (e.g. an
        RCCL collective that never completes): rank 0's on_timeout(message)
        prints the line with the headline and that error, and every rank ends
        with status 0 — os._exit, since a thread blocked inside a collective
        cannot be unwound (cleanup(), e.g. removing the shared frame's file,
        runs first)."""
    lock = threading.Lock()
    done = threading.Event()
    store = dist.distributed_c10d._get_default_store() if world > 1 else None
    keys = [f"pt_bench/{name}/{r}" for r in range(world)]

    def posted():
        """(rank, outcome) of the ranks that have posted so far."""
        if store is None:
            return []
        got = []
        for r, k in enumerate(keys):
            if store.check([k]):
                got.append((r, store.get(k).decode()))
        return got

    def fire(msg):
        with lock:
            if done.is_set():
                return
            print(f"bench: {msg}; ending the job with the headline result", file=sys.stderr, flush=True)
            if store is not None:   # the peers report it too
                try:
                    if not store.check([keys[rank]]):
                        store.set(keys[rank], msg)
                except Exception:   # noqa: BLE001 (the store's host is gone)
                    pass
            if rank == 0:
                on_timeout(msg)
            if cleanup is not None:
                try:
                    cleanup()
                except Exception:   # noqa: BLE001 (best effort on the way out)
                    pass
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)

    def monitor():
        t_end = time.monotonic() + timeout_s
        while not done.wait(poll_s):
            try:
                errs = [o for _, o in posted() if o != "ok"]
            except Exception:   # noqa: BLE001 (the store went away: the job is ending)
                errs = []
            if errs:
                fire("; ".join(errs))
            if time.monotonic() > t_end:
                fire(f"{name}: no outcome within {timeout_s:.0f} s (watchdog on rank {rank})")
    if world > 1:
        # the budget starts when every rank is here (rank 0 checked parity
        # meanwhile); the control group is gloo, not the transport under test
        dist.barrier()
    th = threading.Thread(target=monitor, daemon=True)
    th.start()
    try:
        val, err = run(), None
    except Exception as e:   # noqa: BLE001 (reported in the line)
        val, err = None, f"rank {rank}: {type(e).__name__}: {e}"
        print(f"bench: {name} failed: {err}", file=sys.stderr, flush=True)
    if store is not None:
        # every rank's outcome, polled (a blocking store wait would hold the
        # GIL and starve the monitor); the monitor ends a wait that cannot end
        try:
            store.set(keys[rank], "ok" if err is None else err)
            while True:
                got = posted()
                if len(got) == world:
                    break
                time.sleep(poll_s)
        except Exception as e:   # noqa: BLE001 (the store's host, rank 0, is gone)
            fire(f"{name}: the ranks' store is gone ({type(e).__name__}: {e})")
        errs = [o for _, o in got if o != "ok"]   # every rank's (one may follow from another)
        err = "; ".join(errs) if errs else None
    with lock:
        done.set()
    th.join()
    return (None if err else val), err


def exit_guard(seconds):
    """After the line is out: if the teardown (barriers, unmapping, process
    group shutdown) hangs, end the process with status 0 anyway."""
    t = threading.Timer(seconds, lambda: os._exit(0))
    t.daemon = True
    t.start()
    return t


def run_host_frame(ctx, steps, warmup, base):
    """The host-frame transport: returns (elapsed s over `steps` steps, rank
    0's render-launch ms per step, the frame of the last step on rank 0 or
    None, the next free step number)."""
    import torch
    r, p, hf, stream, rank, world, dist = (ctx[k] for k in ("r", "p", "hf", "stream", "rank", "world",
                                                            "dist"))

    def loop(first, n, evs=None):
        ev = (lambda i: evs[i]) if evs else (lambda i: None)
        if rank == 0:
            if n > 0:
                hf.render(r, p, first, stream, events=ev(0))
            for i in range(n):
                if i + 1 < n:
                    hf.render(r, p, first + i + 1, stream, events=ev(i + 1))
                hf.wait(first + i)
                hf.release(first + i)
        else:
            for i in range(n):
                hf.render(r, p, first + i, stream, events=ev(i))

    loop(base, warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    loop(base + warmup, steps, evs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    last = base + warmup + steps - 1
    fb = hf.frame(last).copy() if rank == 0 else None
    return elapsed, [a.elapsed_time(b) for a, b in evs], fb, last + 1


def run_device_frame(ctx, steps, warmup):
    """The device-frame transport: render into a device tile, N > 1: RCCL
    gather + device assembly on rank 0, then rank 0's D2H copy to pinned host
    memory.  Returns (elapsed s, rank 0's per-step leg ms {render, gather,
    assembly, d2h}, the last frame on rank 0 or None)."""
    import torch
    from pathtracerpython_amd.distributed import assemble_bands_device
    r, p, stream, rank, world, dist = (ctx[k] for k in ("r", "p", "stream", "rank", "world", "dist"))
    H, W, max_rows = ctx["H"], ctx["W"], ctx["max_rows"]
    # the gather's own group: RCCL (nccl backend) over xGMI; the default group
    # (gloo) only carries the control traffic
    group = dist.new_group(backend="nccl", timeout=ctx["pg_timeout"]) if world > 1 else None
    tile = torch.zeros((max_rows, W, 3), dtype=torch.float32, device="cuda")
    host = gathered = frame = None
    if rank == 0:
        host = torch.empty((H, W, 3), dtype=torch.float32).pin_memory()
        if world > 1:
            gathered = torch.empty((world, max_rows, W, 3), dtype=torch.float32, device="cuda")
            frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        else:
            frame = tile

    def step(ev=None):
        rec = (lambda k: ev[k].record()) if ev else (lambda k: None)
        rec(0)
        r.render_device(p, tile.data_ptr(), stream.cuda_stream)
        rec(1)
        if world > 1:
            dist.gather(tile, gather_list=list(gathered.unbind(0)) if rank == 0 else None, dst=0,
                        group=group)
        rec(2)
        if rank == 0:
            if world > 1:
                assemble_bands_device(gathered, frame, stream.cuda_stream)
            rec(3)
            host.copy_(frame[:H], non_blocking=True)
        rec(4)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    legs = {k: [e[j].elapsed_time(e[j + 1]) for e in evs]
            for j, k in enumerate(("render", "gather", "assembly", "d2h"))}
    # the gather's communicator as RCCL reports it (1: no gather at N = 1)
    legs["rccl_world"] = dist.get_world_size(group) if group is not None else 1
    if group is not None:
        dist.destroy_process_group(group)
    return elapsed, legs, (host.numpy().copy() if rank == 0 else None)


def main():
    args = parse()
    from pathtracerpython_amd.launch import init_gloo, pg_timeout, rank_env, spawn_ranks, under_launcher
    if args.gpus > 1 and not under_launcher():
        sys.exit(spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    import numpy as np
    import torch
    import torch.distributed as dist

    rank, local, world = rank_env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # PT_BENCH_REHEARSE=1 (tests only): every rank on device 0, the
    # host-frame transport — the N > 1 code path on a one-GPU box (its
    # timings mean nothing: the ranks share the GPU)
    rehearse = os.environ.get("PT_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
        args.frame = "host"
    elif os.environ.get("PT_BENCH_FORCE_DEVICE0") == "1":
        # (tests only) the rank-to-device mistake on purpose, without the
        # rehearsal's licence: the job must refuse to print a line
        local = 0
        args.frame = "host"
    torch.cuda.set_device(local)
    if world > 1:
        # the control plane (barriers, the frame's name, error exchange, max
        # over ranks) runs over gloo on the host: the headline (host frame)
        # needs no collective on the GPUs, and a failing RCCL leg cannot take
        # it down; the device-frame leg makes its own RCCL group for its gather
        init_gloo()

    from oracle.oracle import host_threads
    from pathtracerpython_amd import scene_reader
    from pathtracerpython_amd.distributed import HostFrame, band_rows_of
    from pathtracerpython_amd.render import Renderer
    scene_reader.VERBOSE = False
    cfg = dict(CONFIGS[args.config])
    if args.spp:
        cfg["spp"] = args.spp
    W, H, SPP, B = cfg["W"], cfg["H"], cfg["spp"], cfg["bounces"]
    if args.scaling == "weak":
        H = cfg["H"] * world

    def bcast(obj):   # rank 0's object to every rank
        if world == 1:
            return obj
        o = [obj]
        dist.broadcast_object_list(o, src=0)
        return o[0]

    if args.config == "k5":
        from pathtracerpython_amd.synth import write_k5_scene
        tmp = tempfile.mkdtemp(prefix="k5_")
        sdl = bcast(write_k5_scene(tmp, n_tris=100_000, seed=0, size=W) if rank == 0 else None)
        scene = scene_reader.Scene(sdl)   # one writer, every rank reads the same files
    else:
        scene = scene_reader.Scene(os.path.join(ROOT, "scenes", "cornell", "cornellroom.sdl"))
    r = Renderer(scene)
    p = r.params(W, H, SPP, B, SEED, row_begin=0, row_end=H, row_step=world, row_phase=rank)
    rows = r.band_rows(p)
    assert rows == len(band_rows_of(H, rank, world))
    stream = torch.cuda.current_stream()
    name = bcast(HostFrame.new_name() if rank == 0 else None)
    # the shared host frame (rank 0 creates the file first); if any rank
    # cannot map it (no /dev/shm, page-locking refused), every rank falls back
    # to the device-frame transport and the line says why
    hf, hf_err = None, None

    def open_frame(create):
        try:
            return HostFrame(H, W, world, rank, name, create=create), None
        except Exception as e:   # noqa: BLE001 (reported in the line)
            return None, f"rank {rank}: {type(e).__name__}: {e}"
    if rank == 0:
        hf, hf_err = open_frame(True)
    if world > 1:
        dist.barrier()
        if rank != 0:
            hf, hf_err = open_frame(False)
        errs = [None] * world
        dist.all_gather_object(errs, hf_err)
        hf_err = next((e for e in errs if e), None)
    if hf_err:
        if hf is not None:
            hf.close()
            hf = None
        if args.frame == "host":
            args.frame = "device"
            if rank == 0:
                print(f"bench: host frame unavailable ({hf_err}); timing the device frame",
                      file=sys.stderr, flush=True)
    ctx = dict(r=r, p=p, hf=hf, stream=stream.cuda_stream, rank=rank, world=world, dist=dist,
               H=H, W=W, max_rows=(H + world - 1) // world, pg_timeout=pg_timeout())
    paths = W * H * SPP

    def host_mode(base):
        el, ks, fb, nxt = run_host_frame(ctx, args.steps, args.warmup, base)
        el, _ = rank_legs(el, dist, world)
        km = float(np.mean(ks))
        kmax, kmin = rank_legs(km, dist, world)
        ms = el / args.steps * 1e3
        return {"ms_per_step": round(ms, 4), "value": round(paths / (ms * 1e-3) / 1e6, 2),
                "legs_ms": {"band_kernel_max": round(kmax, 4), "band_kernel_min": round(kmin, 4),
                            "after_kernel": round(ms - kmax, 4)},
                "_k_ms": km, "_fb": fb, "_next": nxt}

    def device_mode():
        dctx = dict(ctx, stream=stream)
        el, legs, fb = run_device_frame(dctx, args.steps, args.warmup)
        el, _ = rank_legs(el, dist, world)
        km = float(np.mean(legs["render"]))
        kmax, kmin = rank_legs(km, dist, world)
        ms = el / args.steps * 1e3
        lg = {"band_kernel_max": round(kmax, 4), "band_kernel_min": round(kmin, 4)}
        if rank == 0:
            for k in ("gather", "assembly", "d2h"):
                lg[k] = round(float(np.mean(legs[k])), 4)
        return {"ms_per_step": round(ms, 4), "value": round(paths / (ms * 1e-3) / 1e6, 2),
                "legs_ms": lg, "rccl_world": legs["rccl_world"], "_k_ms": km, "_fb": fb}

    # 1. the headline transport
    head = host_mode(0) if args.frame == "host" else device_mode()
    other_name = "device" if args.frame == "host" else "host"
    # which GPU every rank ran on, with its own band kernel time: the line
    # certifies that N ranks used N distinct GPUs; two ranks
    # on one device end the job without a line, except in the one-GPU
    # rehearsal (PT_BENCH_REHEARSE), where the ranks share device 0 on purpose
    ranks = rank_records(dict(rank=rank, **device_identity(), band_kernel_ms=round(head["_k_ms"], 4)),
                         dist, world)
    dup = duplicate_devices(ranks)
    if dup and not rehearse:
        print(f"bench: ranks share a GPU ({', '.join(dup)}): {ranks}; no line printed "
              "(one rank per GPU is the contract)", file=sys.stderr, flush=True)
        if hf is not None:
            hf.discard()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)
    k_ms = head["_k_ms"]
    fb = head["_fb"]
    ms_per_step = head["ms_per_step"]
    value = head["value"]

    # 2. rank 0: the complete line from the headline alone (roofline, parity,
    # CPU baseline) — before the secondary transport runs at all
    result = None
    if rank == 0:
        from oracle import oracle
        if args.config == "k5":
            roofline = k5_roofline(r, p, k_ms)
        else:
            roofline = k_render_roofline(r, p, k_ms, W, rows, SPP, args.config)
        linf = checked = over = None
        cpu = None
        want_cpu = not args.no_cpu_baseline and world == 1
        if args.config == "k2" and (want_cpu or not args.no_check):
            # the whole frame on the oracle: the parity check over every
            # pixel, and (N = 1) the CPU baseline's timing of the same job
            threads = host_threads()
            t1 = time.perf_counter()
            ref, _ = oracle.render(r.packed, W, H, SPP, B, SEED, threads=threads)
            cdt = time.perf_counter() - t1
            if want_cpu:
                cpu = cpu_record(W * H * SPP, cdt, threads,
                                 f"the whole {W}x{H} {SPP} spp {B}-bounce job")
            if not args.no_check:
                from pathtracerpython_amd.render import to_list_order
                err = np.abs(to_list_order(fb.astype(np.float64)) - ref).max(axis=1)
                linf = float(err.max())
                checked = f"all {W * H} pixels"
                over = {"1e-6": int((err > 1e-6).sum()), "1e-4": int((err > 1e-4).sum())}
        elif args.config == "k5" and (want_cpu or not args.no_check):
            # fixed rows (bottom, middle, top), every pixel's 256 samples on
            # the brute-force oracle: the parity check, and (N = 1) the CPU
            # baseline's timing of the same pixels
            chk = k5_check_pixels(W, H)
            pix = np.array([ix * H + iy for ix, iy in chk], dtype=np.int64)
            threads = host_threads()
            t1 = time.perf_counter()
            ref, _ = oracle.render(r.packed, W, H, SPP, B, SEED, pixels=pix, threads=threads)
            cdt = time.perf_counter() - t1
            if want_cpu:
                cpu = cpu_record(len(pix) * SPP, cdt, threads,
                                 f"{len(pix)} pixels on rows 0, H/2, H-1 at {SPP} spp (brute force over "
                                 f"all triangles, as the reference; the parity pixels)")
            if not args.no_check:
                got = np.array([fb[H - 1 - iy, ix] for ix, iy in chk], dtype=np.float64)
                err = np.abs(got - ref).max(axis=1)
                linf = float(err.max())
                checked = f"{len(chk)} pixels on rows 0, H/2, H-1 (all {SPP} samples each)"
                over = {"1e-6": int((err > 1e-6).sum()), "1e-4": int((err > 1e-4).sum())}
        else:
            if not args.no_check:
                chk = [(ix, iy) for iy in (0, H // 4 + 1, H // 2, H - 1)
                       for ix in range(0, W, max(1, W // 128))]
                checked = f"{len(chk)} pixels on rows 0, H/4+1, H/2, H-1"
                pix = np.array([ix * H + iy for ix, iy in chk], dtype=np.int64)
                ref, _ = oracle.render(r.packed, W, H, SPP, B, SEED, pixels=pix, threads=host_threads())
                got = np.array([fb[H - 1 - iy, ix] for ix, iy in chk], dtype=np.float64)
                err = np.abs(got - ref).max(axis=1)
                linf = float(err.max())
                over = {"1e-6": int((err > 1e-6).sum()), "1e-4": int((err > 1e-4).sum())}
            if want_cpu:
                cpu = cpu_baseline(oracle, r.packed, W, H, SPP, B, args.config)
        parallel = f"rows interleaved over {world} GPU" + ("s" if world > 1 else "") + \
            (", bands written into one shared page-locked host frame" if args.frame == "host" else
             (" + RCCL gather + device assembly" if world > 1 else "") + " + D2H copy")
        wl = cfg["workload"].format(spp=SPP)
        if args.scaling == "weak":
            wl = "Cornell box 512 x (512 N) 64 spp 4 bounces, 512 rows per GPU (weak scaling)"
        result = {
            "metric": METRIC,
            "value": value, "unit": "Mpath-samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f32+f64", "data": "synthetic",
            "config": {"workload": wl, "width": W, "height": H, "spp": SPP, "bounces": B,
                       "seed": SEED, "parallelism": parallel, "frame": args.frame,
                       "control_plane": "gloo (host)" if world > 1 else None,
                       "timed_step": "render + the framebuffer in host memory (SURVEY.md §8(d): "
                                     "kernel + D2H), " +
                                     ("each GPU writing its band into one shared page-locked frame"
                                      if args.frame == "host" else
                                      "RCCL gather + device assembly (N > 1) + D2H copy")},
            "frame_modes": {args.frame: {k: v for k, v in head.items() if not k.startswith("_")},
                            other_name: {"pending": "runs after the headline"}},
            "ranks": ranks,
            "ranks_share_a_gpu": dup or None,
            "host_frame_error": hf_err,
            "linf_vs_cpu_ref": linf, "linf_checked": checked, "pixels_over": over,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }

    # 3. the other transport, after the headline line is complete: bounded and
    # non-fatal (a failure or a hang is recorded under frame_modes, the
    # headline line is printed regardless)
    if args.no_secondary:
        run = {"skipped": "--no-secondary"}
    elif other_name == "host" and hf is None:
        run = {"skipped": f"host frame unavailable: {hf_err}"}
    elif rehearse and not os.environ.get("PT_BENCH_INJECT_DEVICE_LEG"):
        run = {"skipped": "PT_BENCH_REHEARSE (the ranks share one GPU: no RCCL gather)"}
    elif rehearse:
        # the injection tests on one GPU: a gloo collective stands in for the
        # gather (RCCL refuses two ranks on one device)
        def run():
            dist.all_reduce(torch.ones(1))
            return {"skipped": "PT_BENCH_REHEARSE: a gloo collective stood in for the RCCL gather"}
    else:
        nxt = head.get("_next", 0)
        run = device_mode if other_name == "device" else (lambda: host_mode(nxt))
    budget = float(os.environ.get("PT_BENCH_LEG_TIMEOUT_S", "0")) or \
        120.0 + 4.0 * (args.steps + args.warmup) * ms_per_step * 1e-3
    ok = finish_line(result, other_name, run, budget, rank, world, dist, head_fb=fb,
                     cleanup=hf.discard if hf is not None else None)
    # after a failed leg the peers may be gone: no collective in the teardown
    if world > 1 and ok:
        dist.barrier()
    if hf is not None:
        hf.close()
    r.close()
    if world > 1 and ok:
        dist.barrier()
        dist.destroy_process_group()
    if world > 1 and not ok:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    return result


def finish_line(result, other_name, run, budget_s, rank, world, dist, head_fb=None, cleanup=None):
    """The end of a bench job, on every rank: the other frame transport
    `run()` (or a dict saying why it is skipped) bounded and non-fatal
    (bounded_leg), then rank 0 prints its line — with the other transport's
    legs, or its error — exactly once.  `result`: rank 0's complete line
    (None elsewhere); head_fb: the headline's last frame on rank 0, compared
    bit for bit with the other transport's.  Returns False when the leg
    failed: its peers may have left, so no collective may follow."""
    import numpy as np
    out = LineOut()
    if isinstance(run, dict):
        other, err = run, None
    else:
        def on_timeout(msg):
            result["frame_modes"][other_name] = {"error": msg}
            out.emit(result)
        other, err = bounded_leg(injected_leg(run, rank), budget_s, f"{other_name}-frame leg", rank,
                                 world, dist, on_timeout, cleanup=cleanup)
    if rank == 0:
        if err:
            other = {"error": err}
        elif other.get("_fb") is not None and head_fb is not None:
            # both transports ran the same launches: the same frame to the bit
            result["frame_modes"]["frames_bitwise_equal"] = bool(np.array_equal(other["_fb"], head_fb))
        result["frame_modes"][other_name] = {k: v for k, v in other.items() if not k.startswith("_")}
        out.emit(result)
    exit_guard(120.0)   # the line is out: a hanging teardown must not hold the job
    return err is None


def k5_check_pixels(W, H):
    """K5's parity pixels: 22 evenly spaced pixels on each of the bottom,
    middle and top image rows (66)."""
    import numpy as np
    cols = [int(round(c)) for c in np.linspace(0, W - 1, 22)] if W > 1 else [0]
    return [(ix, iy) for iy in (0, H // 2, H - 1) for ix in cols]


def k_render_roofline(r, p, k_ms, W, rows, SPP, config):
    """k_render against the FP32 VALU roof: exact reference-semantics test
    count of this rank's launch (separate counting launch) x 47 FLOP."""
    from pathtracerpython_amd._abi import PT_FLAG_COUNT, with_flags
    _, st = r.render_params(with_flags(p, PT_FLAG_COUNT, out_row_stride=0), stats=True)
    tests = st["closest_tests"] + st["shadow_tests"]
    achieved = tests * FLOP_PER_TEST / (k_ms * 1e-3) / 1e12
    traffic, tsrc = load_traffic(config)
    return {"bound": "valu", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
            "traffic": traffic,
            "kernel": "k_render<false,false,false>",
            "compute_pipe": "VALU f32 (no MFMA: scalar ray-triangle tests, not a contraction)",
            "work_per_launch": {"ray_triangle_tests": tests,
                                "tests_per_path_sample": round(tests / (W * rows * SPP), 2),
                                "flop_per_test": FLOP_PER_TEST,
                                "f64_fallback_tests": st["f64_fallbacks"],
                                "f64_rescans": st["f64_rescans"]},
            "kernel_ms_mean": round(k_ms, 4),
            "hbm_frac": (round(traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
                         if traffic else None),
            "traffic_source": tsrc, "kernel_source_sha": lib_build_id()}


def k5_roofline(r, p, render_ms):
    """The wavefront render's two walk kernels (k_wf_shadow, k_wf_closest):
    algorithmic bytes of their launches (counting launch) over their own
    HIP-event time (a PT_FLAG_KERNEL_TIMES launch of the production kernels,
    which runs the two walks of a step one after the other on one stream, so
    neither time includes waiting for CUs the other holds), against the L2
    roof — the BVH (9.6 MB of nodes and leaf records) is served from the
    XCDs' L2 (~92% hit) and the rate of its record reads exceeds HBM's peak.
    The top-level object is the walk with the larger own time per render, the
    other one is `other_walk`.  `traffic` is the PMC bytes the walk moves
    beyond L2 (TCC FETCH_SIZE + WRITE_SIZE: Infinity Cache hits included, so
    an upper bound of its HBM bytes), reported against HBM's peak as
    beyond_l2_frac."""
    from pathtracerpython_amd._abi import PT_FLAG_KERNEL_TIMES, PT_FLAG_WALK_COUNT, with_flags
    _, wc = r.render_params(with_flags(p, PT_FLAG_WALK_COUNT, out_row_stride=0), stats=True)
    _, kt = r.render_params(with_flags(p, PT_FLAG_KERNEL_TIMES, out_row_stride=0), stats=True)
    traffic = load_traffic_record("k5")

    def walk(kind):
        nl = max(1, kt[f"{kind}_launches"])
        q_b = SHADOWQ_B + SHADOW_RES_B if kind == "shadow" else CLOSESTQ_B + CLOSEST_RES_B
        total = (wc[f"{kind}_node_visits"] * QNODE_B + wc[f"{kind}_leaf_units"] * UNITC_B +
                 wc[f"{kind}_queries"] * q_b)
        per_launch = total / nl
        launch_ms = kt[f"{kind}_ms"] / nl
        achieved = per_launch / (launch_ms * 1e-3) / 1e9
        tr = None
        if traffic:
            tr = traffic.get("hbm_bytes_per_launch" if kind == "shadow" else "closest_hbm_bytes_per_launch")
        return {"bound": "l2", "achieved": round(achieved, 2), "peak": L2_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / L2_PEAK_GBS, 4), "traffic": tr,
                "peak_source": "MI355X_MICROARCH.md 'L2 (per XCD)': ~34.5 TB/s aggregate",
                "gather_lower_bound": {"peak": L2_GATHER_GBS, "frac": round(achieved / L2_GATHER_GBS, 4),
                                       "source": "MI355X_MICROARCH.md 'Indexed rows': L2-served gather "
                                                 "into LDS, 16.8-18.8 TB/s"},
                "traffic_level": "beyond L2 (TCC FETCH_SIZE + WRITE_SIZE, FETCH doubled for gfx950; "
                                 "Infinity Cache hits included: an upper bound of HBM bytes)",
                "kernel": f"k_wf_{kind}<true,false> (persistent " +
                          ("one-ray shadow walks)" if kind == "shadow" else "closest-hit walks)"),
                "beyond_l2_frac": (round(tr / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if tr else None),
                "work_per_launch": {"queries": wc[f"{kind}_queries"] / nl,
                                    "node_visits": wc[f"{kind}_node_visits"] / nl,
                                    "leaf_unit_tests": wc[f"{kind}_leaf_units"] / nl,
                                    "bytes": per_launch,
                                    "bytes_model": f"{QNODE_B} B per 4-wide node visit + {UNITC_B} B "
                                                   f"per leaf unit + {q_b} B per query (its record "
                                                   f"read, list entry, result written)"},
                "kernel_ms_mean": round(launch_ms, 4), "launches_per_render": nl,
                "kernel_ms_per_render": round(kt[f"{kind}_ms"], 2),
                "time_basis": "own time: the walks of a step run one after the other in this "
                              "profiling launch (PT_FLAG_KERNEL_TIMES)"}
    sh, cl = walk("shadow"), walk("closest")
    top, other = (sh, cl) if kt["shadow_ms"] >= kt["closest_ms"] else (cl, sh)
    top = dict(top)
    top.update({"note": "latency-bound pointer chasing over an L2-resident BVH: the peak is the "
                        "L2's rate of MI355X_MICROARCH.md (~34.5 TB/s; the measured L2-served "
                        "gather rate, 18.8 TB/s, is gather_lower_bound); the record reads run "
                        "above HBM's 8 TB/s, the PMC bytes beyond L2 are traffic / beyond_l2_frac",
                "other_walk": other,
                "render_ms_mean": round(render_ms, 3),
                "kernel_ms_per_render_serial": {"shade": round(kt["shade_ms"], 2),
                                                "shadow": round(kt["shadow_ms"], 2),
                                                "closest": round(kt["closest_ms"], 2)},
                "traffic_source": traffic.get("source") if traffic else
                load_traffic("k5")[1], "kernel_source_sha": lib_build_id()})
    return top


def cpu_record(n_paths, seconds, threads, sample):
    return {"value": float("%.4g" % (n_paths / seconds / 1e6)), "unit": "Mpath-samples/s",
            "cores": threads, "kind": "port",
            "host_cpus_visible": len(os.sched_getaffinity(0)),
            "sample": f"oracle/pt_oracle.c (f64 C restatement of main.py:186-280) on {sample}: "
                      f"{n_paths} path samples in {seconds:.1f} s on {threads} threads "
                      f"(this GPU's CPU share: OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')})"}


def cpu_baseline(oracle, packed, W, H, SPP, B, config):
    """The C oracle on this host's CPU share, on a bounded sample (~5-30 s)
    (k2: bench.main times the whole frame, which is also its parity check)."""
    import numpy as np
    threads = oracle.host_threads()
    if config == "k4":
        rows = list(range(0, H, 64))
        pix = np.array([ix * H + iy for iy in rows for ix in range(0, W, 4)], dtype=np.int64)
        sample = f"{len(pix)} pixels (every 4th column of every 64th row) at {SPP} spp"
    else:
        rs = np.random.RandomState(1)
        pix = np.sort(rs.choice(W * H, 24, replace=False)).astype(np.int64)
        sample = f"24 random pixels at {SPP} spp (brute force over all triangles, as the reference)"
    t1 = time.perf_counter()
    oracle.render(packed, W, H, SPP, B, SEED, pixels=pix, threads=threads)
    return cpu_record(len(pix) * SPP, time.perf_counter() - t1, threads, sample)


if __name__ == "__main__":
    main()
