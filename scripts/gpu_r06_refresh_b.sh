#!/bin/bash
# round 6 final measurements, part B: the K5 profile refresh (kernel stats of
# the bench render and of a serialised-walks render, PMC traffic of the walks
# stamped with the build id, the K5 bench line) and every single-GPU BASELINE
# configuration at full size (scripts/run_configs.py), the K4-frame bench line
set -o pipefail
mkdir -p gpurun_out/r06_final
PARTS=k5 bash scripts/refresh_profiles.sh r06 > gpurun_out/r06_final/refresh_k5.log 2>&1
rc=$?; tail -2 gpurun_out/r06_final/refresh_k5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config k4 > gpurun_out/refresh_r06/profiles/r06_bench_k4.json 2> gpurun_out/r06_final/bench_k4.err
rc=$?; cat gpurun_out/refresh_r06/profiles/r06_bench_k4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u scripts/run_configs.py 2>&1 | grep -v amdgpu.ids > gpurun_out/refresh_r06/profiles/r06_configs.jsonl
rc=$?; cat gpurun_out/refresh_r06/profiles/r06_configs.jsonl; exit $rc
