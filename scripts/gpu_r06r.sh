#!/bin/bash
# round 6, call r: timing ablation of the shade step — the fused pass over the
# uniform (Cornell) units skipped (variant ab_nounits; its frame is wrong by design)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06r
ROUNDS=2 LIMIT=120 bash scripts/variants.sh ab_ python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06r/k5.txt
