#!/bin/bash
# Memory counters of the K5 wavefront walk kernels (dev tool).
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_wf2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/k5_modes.py ${1:-256} ${2:-16} > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_SMEM SQ_INSTS_FLAT --output-format csv -d $OUT/p2 -o p -- python3 $R/scripts/k5_modes.py ${1:-256} ${2:-16} > $OUT/p2.log 2>&1
for k in k_wf_shadow k_wf_closest; do
  PMC_KERNEL=$k python3 $R/scripts/summarize_pmc.py $OUT/$k.json $OUT/p1 $OUT/p2 > /dev/null
  python3 -c "
import json; d=json.load(open('$OUT/$k.json')); m=d['per_dispatch_median']; print('$k', d['dispatches'].get('SQ_WAVES'), {k: '%.3g' % v for k, v in m.items()})"
done
