#!/bin/bash
# round 6, call s: the walk kernels' parameters re-swept (variants wt_*: exit
# thresholds, fetch chunk, LDS stack entries) on the K5 proxy and at full size
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06s
ROUNDS=2 LIMIT=120 bash scripts/variants.sh wt_ python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06s/k5.txt
ROUNDS=1 LIMIT=200 bash scripts/variants.sh wt_ python3 scripts/prof_k5.py 2 1024 256 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06s/k5_full.txt
