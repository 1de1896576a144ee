#!/bin/bash
# round 6, call k: scheduler knobs for the K2 unit (variants k2s_*) A/B on prof_k2
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06k
ROUNDS=2 bash scripts/variants.sh k2s_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06k/k2.txt
