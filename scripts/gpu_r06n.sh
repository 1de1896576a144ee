#!/bin/bash
# round 6, call n: K5 512^2 proxy, own kernel times, against the built library:
# the walk kernels under the iterative min-register / max-occupancy schedulers
# (ws_iterative-*, every unit), the shade step at >= 4 waves/SIMD (ws_shade4),
# the shadow walks' list in per-XCD segments (ws_xcd; its frame checked)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06n
PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB=pathtracerpython_amd/_lib/variants/ws_xcd.so timeout -k 10 120 python3 scripts/k5_parity.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06n/parity.txt
ROUNDS=2 LIMIT=120 bash scripts/variants.sh ws_ python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06n/k5.txt
