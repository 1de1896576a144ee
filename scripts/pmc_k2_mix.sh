#!/bin/bash
# VALU instruction mix of the K2 render kernel (dev tool; two --pmc passes).
# Usage: bash scripts/pmc_k2_mix.sh TAG [lib.so] -> gpurun_out/pmc_k2mix_TAG/k2_mix.json
set -euo pipefail
R=$PWD; TAG=${1:-base}; OUT=$R/gpurun_out/pmc_k2mix_$TAG; mkdir -p $OUT
if [ -n "${2:-}" ]; then export PT_HIP_LIB=$(readlink -f "$2") PT_ALLOW_FOREIGN_BUILD=1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d $OUT/m1 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/m1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_SCA --output-format csv -d $OUT/m2 -o p -- python3 $R/scripts/prof_k2.py 2 > $OUT/m2.log 2>&1
python3 $R/scripts/summarize_pmc.py $OUT/k2_mix.json $OUT/m1 $OUT/m2 > /dev/null
cat $OUT/k2_mix.json
