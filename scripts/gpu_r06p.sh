#!/bin/bash
# round 6, call p: the final refresh, part A (scripts/gpu_r06_refresh_a.sh), then
# K2 variants k2v_* against it (PT_MICRO 6 under the ILP scheduler)
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/gpu_r06_refresh_a.sh || exit $?
mkdir -p gpurun_out/r06p
ROUNDS=2 LIMIT=120 bash scripts/variants.sh k2v_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r06p/k2.txt
