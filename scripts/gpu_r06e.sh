#!/bin/bash
# round 6, call e: the GPU suite on the kernel with ray 0's skip value, del's
# |t| term before the vote, the vote as one minimum and the light's quad form;
# K2 A/B against the light's general form (k2_nolq) and call d's kernel (k2_base)
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06e/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06e/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06e/k2_variants.txt
