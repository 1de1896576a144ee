#!/bin/bash
# round 6, call c: the GPU suite on the plane-axis unit kernel (PT_AXIS_UNITS),
# K2 A/B: plane-axis units, the per-unit constant moves (PT_MICRO 5 / 6), del's
# |t| term before the vote (PT_DEL_PRE); the K5 frame hash
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06c/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06c/k2_variants.txt || exit 3
timeout -k 10 200 python3 scripts/prof_k5.py 2 1024 256 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06c/k5_main.txt
