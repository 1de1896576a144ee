#!/bin/bash
# Dev tool: the full K5 render (1024^2 x 256 spp, 2 launches) of the built library and of
# every variant under pathtracerpython_amd/_lib/variants (PT_HIP_LIB).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
echo "== main"; timeout -k 10 300 python3 "$R/scripts/prof_k5.py" 2 1024 256
for v in "$R"/pathtracerpython_amd/_lib/variants/*.so; do
    echo "== $(basename "$v")"
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 300 python3 "$R/scripts/prof_k5.py" 2 1024 256
done
