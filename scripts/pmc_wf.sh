#!/bin/bash
# Per-kernel PMC counters of the K5 wavefront kernels (dev tool; 512^2 x 64 spp,
# prof_k5.py).  Usage: bash scripts/pmc_wf.sh TAG [lib.so] -> gpurun_out/pmc_wf_TAG/{shade,shadow,closest}.json
set -euo pipefail
R=$PWD; TAG=${1:-base}; OUT=$R/gpurun_out/pmc_wf_$TAG; mkdir -p $OUT
if [ -n "${2:-}" ]; then export PT_HIP_LIB=$(readlink -f "$2"); fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/prof_k5.py 1 512 64 > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o p -- python3 $R/scripts/prof_k5.py 1 512 64 > $OUT/p2.log 2>&1
for k in shade shadow closest; do
    PMC_KERNEL="k_wf_$k" python3 $R/scripts/summarize_pmc.py $OUT/$k.json $OUT/p1 $OUT/p2 > /dev/null
done
