#!/bin/bash
# round 6, call f: K2 launch parameters on the round-6 kernel: the tail rows'
# share and lane multiplier (PT_TAIL_FRAC / PT_TAIL_MUL), lanes per pixel 16
set -o pipefail
mkdir -p gpurun_out/r06f
ROUNDS=3 bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06f/k2_variants.txt || exit 3
for l in 16 8 16 8; do echo "== main --lanes $l"; timeout -k 10 120 python3 scripts/prof_k2.py 20 --lanes $l 2>&1 | grep -v amdgpu.ids; done | tee gpurun_out/r06f/k2_lanes.txt
