#!/bin/bash
# Dev tool: run one timing command against the built library and every
# variant build pathtracerpython_amd/_lib/variants/PREFIX*.so (PT_HIP_LIB),
# the whole list ROUNDS times (default 2) so box drift shows.  Each run has its
# own time limit (LIMIT s, default 300); stops at the first failure.
#   bash scripts/variants.sh k2_ python3 scripts/prof_k2.py 20
#   bash scripts/variants.sh k5_ python3 scripts/prof_k5.py 2 1024 256 --times
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
prefix=$1; shift
for round in $(seq 1 "${ROUNDS:-2}"); do
    echo "== main"; timeout -k 10 "${LIMIT:-300}" "$@"
    for v in "$R"/pathtracerpython_amd/_lib/variants/"$prefix"*.so; do
        [ -e "$v" ] || continue
        echo "== $(basename "$v")"
        PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 "${LIMIT:-300}" "$@"
    done
done
