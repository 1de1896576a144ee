#!/bin/bash
# round 6, call i: compiler scheduling strategies (-mllvm -amdgpu-sched-strategy=...)
# on K2 (prof_k2) and the K5 512^2 proxy, A/B against the built library
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06i
ROUNDS=2 bash scripts/variants.sh s_ python3 scripts/prof_k2.py 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06i/k2.txt
ROUNDS=2 bash scripts/variants.sh s_ python3 scripts/prof_k5.py 3 512 64 --times 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06i/k5.txt
