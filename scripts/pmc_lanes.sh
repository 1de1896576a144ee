#!/bin/bash
# VALU lane utilisation of the K2 and K5 render kernels (dev tool).
# Usage: bash scripts/pmc_lanes.sh [lib.so]
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_lanes; mkdir -p $OUT
if [ -n "${1:-}" ]; then export PT_HIP_LIB=$(readlink -f "$1") PT_DEV_OLD_LIB=1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/k2 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/k2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/k5 -o p -- python3 $R/scripts/prof_k5.py 2 > $OUT/k5.log 2>&1
python3 $R/scripts/summarize_pmc.py $OUT/k2.json $OUT/k2 > /dev/null
python3 $R/scripts/summarize_pmc.py $OUT/k5.json $OUT/k5 > /dev/null
