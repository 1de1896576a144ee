#!/bin/bash
# Dev tool: K2 kernel time (prof_k2.py, 20 launches) of the built library and
# of every variant build under pathtracerpython_amd/_lib/variants/*.so
# (compile-time -D experiments, loaded through PT_HIP_LIB), the whole list
# ROUNDS times (default 2) so box drift shows.  Each run has its own time
# limit; stops at the first failure.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
for round in $(seq 1 "${ROUNDS:-2}"); do
    echo "== main"; timeout -k 10 120 python3 "$R/scripts/prof_k2.py" 20
    for v in "$R"/pathtracerpython_amd/_lib/variants/*.so; do
        [ -e "$v" ] || continue
        echo "== $(basename "$v")"
        PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 120 python3 "$R/scripts/prof_k2.py" 20
    done
done
