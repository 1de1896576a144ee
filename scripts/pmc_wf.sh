#!/bin/bash
# Per-kernel PMC counters of the K5 wavefront kernels (dev tool; 512^2 x 64 spp,
# prof_k5.py).  Usage: bash scripts/pmc_wf.sh TAG [lib.so] -> gpurun_out/pmc_wf_TAG/{shade,shadow,closest}.json
set -euo pipefail
R=$PWD; TAG=${1:-base}; OUT=$R/gpurun_out/pmc_wf_$TAG; mkdir -p $OUT
if [ -n "${2:-}" ]; then export PT_HIP_LIB=$(readlink -f "$2") PT_ALLOW_FOREIGN_BUILD=1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/prof_k5.py 1 512 64 > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o p -- python3 $R/scripts/prof_k5.py 1 512 64 > $OUT/p2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p3 -o p -- python3 $R/scripts/prof_k5.py 1 512 64 > $OUT/p3.log 2>&1
for k in shade shadow closest; do
    PMC_KERNEL="k_wf_$k" python3 $R/scripts/summarize_pmc.py $OUT/$k.json $OUT/p1 $OUT/p2 $OUT/p3 > /dev/null
    python3 - "$OUT/$k.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["per_dispatch_median"]
w = d["SQ_WAVE_CYCLES"]
print(sys.argv[1].split("/")[-2], sys.argv[1].split("/")[-1], json.dumps({
    "issue_frac": round(d["SQ_ACTIVE_INST_ANY"] / w, 4), "wait_any_frac": round(d["SQ_WAIT_ANY"] / w, 4),
    "wait_inst_any_frac": round(d["SQ_WAIT_INST_ANY"] / w, 4), "valu_insts": d["SQ_INSTS_VALU"],
    "vmem_rd": d.get("SQ_INSTS_VMEM_RD"), "waves": d["SQ_WAVES"], "busy_cycles": d["SQ_BUSY_CYCLES"],
    "l2_hit": round(d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"]), 4)
    if "TCC_HIT_sum" in d else None}))
PY
done
