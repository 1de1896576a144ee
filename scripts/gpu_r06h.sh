#!/bin/bash
# Round 6, call h: f16 grid codes in the 4-wide nodes (PT_QNODE16) — K5 512^2
# proxy with walk counts and own kernel times, parity, and the full K5 render,
# for the built library and the variants (old 8-bit nodes; f16 codes on the
# 8-bit grid).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
{
echo "== main"
timeout -k 10 200 python3 scripts/prof_k5.py 3 512 64 --counts --times
timeout -k 10 200 python3 scripts/k5_parity.py
for v in pathtracerpython_amd/_lib/variants/*.so; do
    echo "== $(basename "$v")"
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 200 python3 scripts/prof_k5.py 3 512 64 --counts --times
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 200 python3 scripts/k5_parity.py
done
bash scripts/variants_k5_full.sh
} 2>&1 | tee gpurun_out/r06h.log
