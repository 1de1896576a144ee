#!/bin/bash
# Dev tool: rocprofv3 kernel stats of the K5 wavefront render (prof_k5.py,
# 512^2 x 64 spp, 2 launches) for the built library and every variant under
# pathtracerpython_amd/_lib/variants -> gpurun_out/pc_<name>/k5_kernel_stats.csv
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pc_main" -o k5 \
    -- python3 "$R/scripts/prof_k5.py" 2 512 64 > "$R/gpurun_out/pc_main.log" 2>&1
for v in "$R"/pathtracerpython_amd/_lib/variants/*.so; do
    [ -e "$v" ] || continue
    n=$(basename "$v" .so)
    PT_ALLOW_FOREIGN_BUILD=1 PT_HIP_LIB="$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/pc_$n" -o k5 -- python3 "$R/scripts/prof_k5.py" 2 512 64 > "$R/gpurun_out/pc_$n.log" 2>&1
done
