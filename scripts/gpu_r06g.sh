#!/bin/bash
# round 6, call g: the GPU suite on the kernel with the branch-free closest_add,
# |L - P|^2 reused and 4 samples per lane (16 lanes per pixel at K2); K2 A/B of
# the samples-per-lane rule, the reuse, the tail rows' share
set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06g/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06g/k2_variants.txt
