#!/bin/bash
# round 6, call m: K2 under the ILP scheduler — lanes per pixel (8 / 16 auto / 32)
# and the primary ray shared from 8 or 32 lanes (variants k2p_*)
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r06m
{
for r in 1 2; do
    for l in 8 32; do echo "== main --lanes $l"; timeout -k 10 200 python3 scripts/prof_k2.py 20 --lanes $l; done
    ROUNDS=1 bash scripts/variants.sh k2p_ python3 scripts/prof_k2.py 20
done
} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06m/k2.txt
