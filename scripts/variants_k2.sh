#!/bin/bash
# Dev tool: K2 kernel time (prof_k2.py, 10 launches) of the built library and
# of every variant build under pathtracerpython_amd/_lib/variants/*.so
# (compile-time -D experiments, loaded through PT_HIP_LIB).  Each run has its
# own time limit; stops at the first failure.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
echo "== main"; timeout -k 10 120 python3 "$R/scripts/prof_k2.py" 10
for v in "$R"/pathtracerpython_amd/_lib/variants/*.so; do
    [ -e "$v" ] || continue
    echo "== $(basename "$v")"
    PT_HIP_LIB="$v" timeout -k 10 120 python3 "$R/scripts/prof_k2.py" 10
done
