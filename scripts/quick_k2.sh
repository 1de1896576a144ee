#!/bin/bash
# Dev loop on a GPU box: GPU tests, K2 timing of the given builds, HBM write
# bytes of the first build.  Usage: bash scripts/quick_k2.sh TAG lib1.so [lib2.so ...]
set -euo pipefail
R=$PWD; TAG=$1; shift; OUT=$R/gpurun_out/quick_$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 400 python3 scripts/variant_sweep.py "$@" > $OUT/sweep.log 2>&1
export PT_HIP_LIB=$(readlink -f "$1") PT_DEV_OLD_LIB=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/pw.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/pf.log 2>&1
python3 $R/scripts/summarize_pmc.py $OUT/traffic.json $OUT/pw $OUT/pf > /dev/null
tail -1 $OUT/pytest.log; cat $OUT/sweep.log | grep -v amdgpu.ids; python3 -c "import json; d=json.load(open('$OUT/traffic.json')); print('hbm bytes/launch', d['hbm_bytes_per_launch'], d['per_dispatch_median'])"
