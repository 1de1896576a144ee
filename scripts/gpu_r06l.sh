#!/bin/bash
# round 6, call l: the shade step in its own translation unit under the ILP
# scheduler (main) vs in the library (variant shade_in_lib), K5 proxy and full
# size; K2 at 3 waves/SIMD under the ILP scheduler (variant k2w_3)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06l
timeout -k 10 200 python3 scripts/k5_parity.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06l/parity.txt
ROUNDS=2 bash scripts/variants.sh shade_ python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06l/k5.txt
ROUNDS=1 bash scripts/variants.sh shade_ python3 scripts/prof_k5.py 2 1024 256 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06l/k5_full.txt
ROUNDS=2 bash scripts/variants.sh k2w_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06l/k2.txt
