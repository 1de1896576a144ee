set -euo pipefail
R=$PWD; OUT=$R/gpurun_out/pmc_k5; mkdir -p $OUT
if [ -n "${PT_HIP_LIB:-}" ]; then export PT_HIP_LIB=$(readlink -f "$PT_HIP_LIB") PT_ALLOW_FOREIGN_BUILD=1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d $OUT/p1 -o p -- python3 $R/scripts/prof_k5.py 2 > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p2 -o p -- python3 $R/scripts/prof_k5.py 2 > $OUT/p2.log 2>&1
python3 $R/scripts/summarize_pmc.py $OUT/k5_pmc.json $OUT/p1 $OUT/p2 > /dev/null
cat $OUT/k5_pmc.json
