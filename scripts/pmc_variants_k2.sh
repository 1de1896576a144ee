#!/bin/bash
# SQ counters (busy / wait / instruction mix, scripts/pmc_k2.sh) of the built
# K2 kernel and of every variant build under pathtracerpython_amd/_lib/variants
# (dev tool).  Usage: bash scripts/pmc_variants_k2.sh TAG
set -uo pipefail
R=$PWD; TAG=${1:-var}
bash "$R/scripts/pmc_k2.sh" "${TAG}_main" > /dev/null 2>&1 || exit 1
for v in "$R"/pathtracerpython_amd/_lib/variants/${PREFIX:-k2_}*.so; do
    [ -e "$v" ] || continue
    b=$(basename "$v" .so)
    cd "$R" && bash "$R/scripts/pmc_k2.sh" "${TAG}_$b" "$v" > /dev/null 2>&1 || exit 1
done
for d in "$R"/gpurun_out/pmc_k2_${TAG}_*; do
    python3 - "$d/k2_pmc.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["per_dispatch_median"]
w = d["SQ_WAVE_CYCLES"]
print(sys.argv[1].split("/")[-2], json.dumps({
    "issue_frac": round(d["SQ_ACTIVE_INST_ANY"] / w, 4), "wait_any_frac": round(d["SQ_WAIT_ANY"] / w, 4),
    "wait_inst_any_frac": round(d["SQ_WAIT_INST_ANY"] / w, 4), "valu_insts": d["SQ_INSTS_VALU"],
    "salu_insts": d["SQ_INSTS_SALU"], "smem_insts": d["SQ_INSTS_SMEM"],
    "lds_insts": d.get("SQ_INSTS_LDS"), "wave_cycles": w}))
PY
done
