#!/bin/bash
# Per-kernel times of the K5 wavefront render for several library builds (dev
# tool).  Usage: bash scripts/wf_lib_sweep.sh W SPP lib1.so [lib2.so ...]
set -euo pipefail
R=$PWD; W=$1; SPP=$2; shift 2
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so); OUT=$R/gpurun_out/wfsweep_$n; mkdir -p $OUT
  PT_HIP_LIB=$(readlink -f $R/$lib) PT_DEV_OLD_LIB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k -- python3 $R/scripts/k5_modes.py $W $SPP > $OUT/run.log 2>&1
  echo "== $n"; grep -E "wavefront|single" $OUT/run.log; grep -E "k_wf|k_render" $OUT/k_kernel_stats.csv | awk -F, '{printf "%s calls %s total %.1f ms\n", substr($1,1,40), $2, $3/1e6}'
done
