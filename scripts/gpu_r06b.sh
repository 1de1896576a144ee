#!/bin/bash
# round 6, call b: parity suite (incl. the bench rank-record tests), K2 A/B of
# the lean closest range and the med3 max, the med3 NaN probe, K5 A/B of the
# closest list sorted by origin cell (own times + TCC hit rates)
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 60 ./scripts/micro/med3_nan > gpurun_out/r06b/med3_nan.txt 2>&1; tail -1 gpurun_out/r06b/med3_nan.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r06b/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06b/k2_variants.txt || exit 3
ROUNDS=2 LIMIT=200 bash scripts/variants.sh k5_ python3 scripts/prof_k5.py 2 1024 256 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06b/k5_variants.txt || exit 4
PREFIX=k5_ bash scripts/pmc_variants_wf.sh r06b 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06b/k5_pmc.txt
