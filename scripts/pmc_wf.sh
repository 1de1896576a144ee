#!/bin/bash
# Counters of the K5 wavefront kernels (dev tool): lane utilisation, issue and
# wait cycles per kernel.  Usage: bash scripts/pmc_wf.sh [W] [spp]
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_wf; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/k5_modes.py ${1:-256} ${2:-16} > $OUT/p1.log 2>&1
for k in k_wf_shadow k_wf_closest k_wf_shade; do
  PMC_KERNEL=$k python3 $R/scripts/summarize_pmc.py $OUT/$k.json $OUT/p1 > /dev/null
  python3 -c "
import json; d=json.load(open('$OUT/$k.json')); m=d['per_dispatch_median']; n=d['dispatches']
print('$k', d['kernel'].get('VGPR_Count'), 'lane util %.3f' % (m['SQ_THREAD_CYCLES_VALU']/(m['SQ_ACTIVE_INST_VALU']*64)), 'valu/wave-cycle %.3f' % (m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES']), 'wait %.3f' % (m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES']), 'waitinst %.3f' % (m['SQ_WAIT_INST_ANY']/m['SQ_WAVE_CYCLES']), 'salu/valu %.2f' % (m['SQ_INSTS_SALU']/m['SQ_INSTS_VALU']), m)"
done
