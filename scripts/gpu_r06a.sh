#!/bin/bash
# round 6, call a: parity suite, K2 margin-merge A/B, K5 hand-written scan A/B
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r06a/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06a/k2_variants.txt || exit 3
ROUNDS=2 LIMIT=200 bash scripts/variants.sh k5_ python3 scripts/prof_k5.py 2 1024 256 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06a/k5_variants.txt
