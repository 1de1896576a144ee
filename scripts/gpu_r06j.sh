#!/bin/bash
# round 6, call j: the K2 kernel in its own translation unit under LLVM's
# iterative ILP scheduler (pt_k2.hip, build.UNITS): the GPU suite, K2 timing,
# the K5 proxy (the walk kernels keep the default scheduler)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06j
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06j/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06j/gputest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids; done | tee gpurun_out/r06j/k2.txt
timeout -k 10 200 python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06j/k5.txt
