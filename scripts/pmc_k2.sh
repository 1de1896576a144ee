#!/bin/bash
# Instruction-mix / stall counters of the K2 render kernel (dev tool).
# Usage: bash scripts/pmc_k2.sh TAG [lib.so]   -> gpurun_out/pmc_k2_TAG/k2_pmc.json
set -euo pipefail
R=$PWD; TAG=${1:-base}; OUT=$R/gpurun_out/pmc_k2_$TAG; mkdir -p $OUT
if [ -n "${2:-}" ]; then export PT_HIP_LIB=$(readlink -f "$2") PT_ALLOW_FOREIGN_BUILD=1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $OUT/p2 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/p2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $OUT/p3 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/p3.log 2>&1 || echo "pass 3 failed (see p3.log)"
python3 $R/scripts/summarize_pmc.py $OUT/k2_pmc.json $OUT/p1 $OUT/p2 $OUT/p3 > /dev/null
cat $OUT/k2_pmc.json
