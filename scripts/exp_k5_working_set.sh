#!/bin/bash
# exp_k5_working_set.py at each size, plain (times) and under one rocprofv3
# --pmc pass (TCC_HIT_sum TCC_MISS_sum: the walks' L2 hit rate), summarised
# per walk kernel (dev tool).  Usage: bash scripts/exp_k5_working_set.sh OUTDIR
set -uo pipefail
R=$PWD; OUT=$(readlink -f "${1:-$R/gpurun_out/k5ws}"); mkdir -p "$OUT"
timeout -k 10 400 python3 "$R/scripts/exp_k5_working_set.py" > "$OUT/times.jsonl" 2> "$OUT/times.err" || exit 1
grep -v amdgpu "$OUT/times.jsonl"
cd /tmp && export TMPDIR=/tmp
for n in 25000 50000 100000 200000; do
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
        -d "$OUT/pmc_$n" -o p -- python3 "$R/scripts/exp_k5_working_set.py" $n > "$OUT/pmc_$n.log" 2>&1 || exit 2
    for k in k_wf_shadow k_wf_closest k_wf_shade; do
        echo -n "$n $k "
        PMC_KERNEL=$k python3 "$R/scripts/summarize_pmc.py" "$OUT/pmc_${n}_$k.json" "$OUT/pmc_$n" \
            | python3 -c "import json,sys; d=json.load(sys.stdin)['sum_over_dispatches']; h,m=d['TCC_HIT_sum'],d['TCC_MISS_sum']; print(json.dumps({'l2_hit': round(h/(h+m),4), 'l2_miss_req': m}))"
    done
done
