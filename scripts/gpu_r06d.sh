#!/bin/bash
# round 6, call d: K2 A/B on the round-6 kernel (merged margins, lean closest
# range): ray 0's skip value (PT_MICRO 5), del's |t| term before the vote
# (PT_DEL_PRE), both, the shadow vote as one minimum (PT_VOTE_MIN3)
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "k2_full or golden or quad" > gpurun_out/r06d/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/r06d/gputest.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06d/k2_variants.txt
