#!/bin/bash
# round 6, call c: K2 A/B of the per-unit constant moves (PT_MICRO 5 / 6) and
# of del's |t| term before the vote (PT_DEL_PRE); the GPU suite's K2 checks
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k2 or golden or oracle or quad or two_meshes" > gpurun_out/r06c/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06c/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06c/k2_variants.txt
