#!/bin/bash
# round 6 final measurements, part A (after the kernel sources are frozen):
# the GPU suite, the K2 profile refresh (PMC traffic stamped with the build id,
# SQ counters, rocprof stats of the bench command, the bench line) and the
# band-scaling sweep.  Install with: python3 scripts/install_profiles.py r06
set -o pipefail
mkdir -p gpurun_out/r06_final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_final/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06_final/gputest.log; [ $rc -eq 0 ] || exit $rc
PARTS=k2 bash scripts/refresh_profiles.sh r06 > gpurun_out/r06_final/refresh_k2.log 2>&1
rc=$?; tail -2 gpurun_out/r06_final/refresh_k2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/prof_scaling.py 20 2>&1 | grep -v amdgpu.ids > gpurun_out/refresh_r06/profiles/r06_scaling_final.jsonl
rc=$?; cat gpurun_out/refresh_r06/profiles/r06_scaling_final.jsonl; exit $rc
