#!/bin/bash
# Per-kernel times of the K5 wavefront render (dev tool): rocprofv3 kernel
# trace + stats of scripts/prof_k5.py 3.  Usage: bash scripts/prof_k5_wf.sh [W] [spp]
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/prof_k5_wf; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k5 -- python3 $R/scripts/prof_k5.py 3 ${1:-512} ${2:-64} > $OUT/run.log 2>&1
cat $OUT/k5_kernel_stats.csv
