"""Rank process for tests/test_bench_legs.py: the end of a bench.py job
(bench.finish_line: the secondary frame transport, bounded and non-fatal, then
rank 0's one line) over gloo on CPU.  The headline result is a synthetic line
of bench.py's shape (no GPU here); the secondary leg is a gloo collective,
as the device frame's gather is one, which PT_BENCH_INJECT_DEVICE_LEG makes
fail or hang on a chosen rank.

    python tests/bench_leg_worker.py spawn N   # the parent: N rank processes
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main():
    import torch
    import torch.distributed as dist
    import bench
    from pathtracerpython_amd.launch import init_gloo, rank_env
    rank, _, world = rank_env()
    init_gloo()
    result = None
    if rank == 0:
        result = {"metric": bench.METRIC, "value": 3052.0, "unit": "Mpath-samples/s", "n_gpus": world,
                  "ms_per_step": 5.5, "config": {"frame": "host"},
                  "frame_modes": {"host": {"ms_per_step": 5.5, "value": 3052.0,
                                           "legs_ms": {"band_kernel_max": 5.49, "band_kernel_min": 5.48,
                                                       "after_kernel": 0.01}},
                                  "device": {"pending": "runs after the headline"}},
                  "linf_vs_cpu_ref": 6.0e-8, "linf_checked": "all 262144 pixels"}

    def leg():   # a collective across the ranks, as the RCCL gather is
        t = torch.full((4,), float(rank + 1))
        dist.all_reduce(t)
        return {"ms_per_step": 5.6, "value": 3000.0, "legs_ms": {"gather": float(t[0])}}
    budget = float(os.environ.get("PT_BENCH_LEG_TIMEOUT_S", "60"))
    if rank == 0:   # bench.py's rank 0 checks parity before the leg while the others wait
        import time
        time.sleep(float(os.environ.get("PT_TEST_RANK0_DELAY", "0")))
    if bench.finish_line(result, "device", leg, budget, rank, world, dist):
        dist.barrier()   # bench.main's teardown: collectives only after a clean leg
        dist.destroy_process_group()
    else:
        os._exit(0)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "spawn":
        from pathtracerpython_amd.launch import spawn_ranks
        sys.exit(spawn_ranks(int(sys.argv[2]), [os.path.abspath(__file__)]))
    rank_main()
