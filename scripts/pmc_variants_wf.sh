#!/bin/bash
# Per-kernel counters of the K5 wavefront kernels (scripts/pmc_wf.sh) for the
# built library and every variant _lib/variants/${PREFIX:-k5_}*.so (dev tool).
# Usage: bash scripts/pmc_variants_wf.sh TAG
set -uo pipefail
R=$PWD; TAG=${1:-var}
bash "$R/scripts/pmc_wf.sh" "${TAG}_main" || exit 1
for v in "$R"/pathtracerpython_amd/_lib/variants/${PREFIX:-k5_}*.so; do
    [ -e "$v" ] || continue
    cd "$R" && bash "$R/scripts/pmc_wf.sh" "${TAG}_$(basename "$v" .so)" "$v" || exit 1
done
