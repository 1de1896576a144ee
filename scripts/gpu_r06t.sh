#!/bin/bash
# round 6, call t: K2 dispatch knobs re-checked under the ILP scheduler
# (variants k2b_/k2t_: 2-wave render blocks, the tail rows' share and lane factor)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06t
ROUNDS=2 LIMIT=120 bash scripts/variants.sh k2 python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06t/k2.txt
