#!/bin/bash
# round 6, call o: K2 code-generation flags on top of the ILP scheduler (variants k2f_*)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06o
ROUNDS=2 LIMIT=120 bash scripts/variants.sh k2f_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06o/k2.txt
