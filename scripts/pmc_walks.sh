#!/bin/bash
# Memory-pipeline counters of the K5 walk kernels (dev tool): one rocprofv3
# --pmc pass per counter group on the 512^2 x 16 spp K5 proxy
# (scripts/prof_k5.py), summarised per kernel into
# gpurun_out/pmc_walks/<kernel>.json.  With LIST=1 it first writes the
# counters this box offers to gpurun_out/pmc_walks/avail.txt.
# Usage: gpurun -- bash scripts/pmc_walks.sh "CTRS1" "CTRS2" ...
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_walks; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "${LIST:-0}" = 1 ]; then
    timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
fi
dirs=()
i=0
for ctr in "$@"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
        -d $OUT/p$i -o p -- python3 $R/scripts/prof_k5.py 2 512 16 > $OUT/p$i.log 2>&1
    dirs+=($OUT/p$i)
done
if [ $i -gt 0 ]; then
    for k in k_wf_shadow k_wf_closest k_wf_shade; do
        PMC_KERNEL=$k python3 $R/scripts/summarize_pmc.py $OUT/$k.json "${dirs[@]}" > /dev/null
    done
    grep -h -A30 per_dispatch_median $OUT/k_wf_*.json
fi
