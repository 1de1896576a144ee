#!/bin/bash
# HBM traffic and L2 hit rate of the K5 wavefront kernels (dev tool): separate
# rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; TCC hit/miss + wait cycles),
# kernel trace only, then per-kernel medians.  Usage: bash scripts/pmc_wf_traffic.sh [W] [spp]
set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_wf_traffic; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pf -o p -- python3 $R/scripts/prof_k5.py 1 ${1:-512} ${2:-64} > $OUT/pf.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pw -o p -- python3 $R/scripts/prof_k5.py 1 ${1:-512} ${2:-64} > $OUT/pw.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/ph -o p -- python3 $R/scripts/prof_k5.py 1 ${1:-512} ${2:-64} > $OUT/ph.log 2>&1
for k in k_wf_shade k_wf_shadow k_wf_closest; do
  PMC_KERNEL=$k python3 $R/scripts/summarize_pmc.py $OUT/$k.json $OUT/pf $OUT/pw $OUT/ph > /dev/null
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for k in ("k_wf_shade", "k_wf_shadow", "k_wf_closest"):
    d = json.load(open(f"{out}/{k}.json"))
    m = d["per_dispatch_median"]
    print(k, json.dumps({"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
                         "l2_hit": round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3),
                         "wait_frac": round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3),
                         "dispatches": d.get("dispatches")}))
PY
