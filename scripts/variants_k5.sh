#!/bin/bash
# Dev tool: K5 render time (prof_k5.py: 512^2 x 64 spp, 3 launches) of the
# built library and of every variant under pathtracerpython_amd/_lib/variants.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
echo "== main"; timeout -k 10 200 python3 "$R/scripts/prof_k5.py" 3 512 64
timeout -k 10 200 python3 "$R/scripts/k5_parity.py"
for v in "$R"/pathtracerpython_amd/_lib/variants/*.so; do
    [ -e "$v" ] || continue
    echo "== $(basename "$v")"
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 200 python3 "$R/scripts/prof_k5.py" 3 512 64
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 200 python3 "$R/scripts/k5_parity.py"
done
