#!/bin/bash
# Re-measure every artifact under profiles/ that bench.py and DESIGN.md cite,
# on a GPU box (dev tool).  gpurun merges back only gpurun_out/, so the files
# are staged under their final profiles/ names in
#   gpurun_out/refresh_TAG/profiles/
# and installed here with `python3 scripts/install_profiles.py TAG`, which
# checks that every traffic stamp matches the current kernel sources
# (tests/test_profiles.py fails on a stale stamp).
#   1. k_render (K2) HBM traffic: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE
#      (separate passes, kernel trace only; FETCH doubled, gfx950)
#      -> TAG_pmc_k2_traffic.json, traffic_k2.json (stamped)
#   2. k_render SQ counters (busy, stalls, instruction mix) -> TAG_pmc_k2_sq.json
#   3. kernel trace + stats of the K2 bench command -> TAG_k2_kernel_stats.csv
#   4. the K2 bench line -> TAG_bench_k2.json
#   5. K5: kernel stats of the bench render and of a serialised-walks render
#      (each walk's own time), HBM traffic of the shadow walks
#      (traffic_k5.json, stamped) and of the closest walks, the K5 bench line
# Usage (from the repo root): gpurun -- bash scripts/refresh_profiles.sh TAG
# Every GPU step runs under its own time limit; the script stops at the first
# failure.
set -euo pipefail
TAG=${1:-r04}
R=$PWD
OUT=$R/gpurun_out/refresh_$TAG
P=$OUT/profiles
mkdir -p "$P"
cd /tmp && export TMPDIR=/tmp
pmc() {   # pmc NAME "COUNTERS" driver args...
    local name=$1 ctr=$2; shift 2
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv \
        -d "$OUT/$name" -o p -- python3 "$@" > "$OUT/$name.log" 2>&1
}
# PARTS: "k2 k5" (default), or one of them (two gpurun calls)
PARTS=${PARTS:-k2 k5}
if [[ " $PARTS " == *" k2 "* ]]; then
# 1-2. K2 counters (3 launches each)
pmc k2_fetch FETCH_SIZE "$R/scripts/prof_k2.py" 3
pmc k2_write WRITE_SIZE "$R/scripts/prof_k2.py" 3
PMC_NOTE="algorithmic bytes: the framebuffer, 512x512x3 f32 = 3,145,728 B written" \
    python3 "$R/scripts/summarize_pmc.py" "$P/${TAG}_pmc_k2_traffic.json" "$OUT/k2_fetch" "$OUT/k2_write" > /dev/null
python3 "$R/scripts/stamp_traffic.py" "$P/${TAG}_pmc_k2_traffic.json" "$P/traffic_k2.json" median \
    "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), k_render<false,false,false>, 512x512 64spp 4b, median over 3 dispatches; profiles/${TAG}_pmc_k2_traffic.json; FETCH doubled (gfx950)"
pmc k2_sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "$R/scripts/prof_k2.py" 2
pmc k2_sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH" "$R/scripts/prof_k2.py" 2
pmc k2_sq3 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32" "$R/scripts/prof_k2.py" 2
python3 "$R/scripts/summarize_pmc.py" "$P/${TAG}_pmc_k2_sq.json" "$OUT/k2_sq1" "$OUT/k2_sq2" "$OUT/k2_sq3" > /dev/null
cd "$R"
# the box's copy of the repo reads the new stamp, so this run's bench lines
# carry the traffic just measured (profiles/ here is a scratch copy: the
# staged files are installed by install_profiles.py)
cp "$P/traffic_k2.json" "$R/profiles/traffic_k2.json"
# 3-4. K2 bench: rocprof stats of the bench command, then the line itself
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_k2" -o k2 \
    -- python3 "$R/bench.py" --steps 50 --no-cpu-baseline --no-check > "$OUT/trace_k2.log" 2>&1
cp "$OUT/trace_k2/k2_kernel_stats.csv" "$P/${TAG}_k2_kernel_stats.csv"
timeout -k 10 400 python3 "$R/bench.py" > "$P/${TAG}_bench_k2.json" 2> "$OUT/bench_k2.err"
cat "$P/${TAG}_bench_k2.json"
fi
if [[ " $PARTS " == *" k5 "* ]]; then
cd "$R"
# 5. K5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_k5" -o k5 \
    -- python3 "$R/bench.py" --config k5 --steps 1 --warmup 0 --no-cpu-baseline --no-check \
    > "$OUT/trace_k5.log" 2>&1
cp "$OUT/trace_k5/k5_kernel_stats.csv" "$P/${TAG}_k5_kernel_stats.csv"
cd /tmp
# the walks' own times (bench.py's k5 roofline: a PT_FLAG_KERNEL_TIMES render,
# the two walks of a step one after the other)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_k5s" -o k5 \
    -- python3 "$R/scripts/prof_k5_serial.py" 1 > "$OUT/trace_k5s.log" 2>&1
cp "$OUT/trace_k5s/k5_kernel_stats.csv" "$P/${TAG}_k5_kernel_stats_serial.csv"
pmc k5_fetch FETCH_SIZE "$R/scripts/prof_k5.py" 1 1024 256
pmc k5_write WRITE_SIZE "$R/scripts/prof_k5.py" 1 1024 256
PMC_KERNEL=k_wf_shadow PMC_NOTE="k_wf_shadow (K5 one-ray shadow walks, 1024x1024 256 spp): bytes beyond L2 of the BVH node / leaf records and the shadow query records (Infinity Cache hits included)" \
    python3 "$R/scripts/summarize_pmc.py" "$P/${TAG}_pmc_k5_traffic.json" "$OUT/k5_fetch" "$OUT/k5_write" > /dev/null
PMC_KERNEL=k_wf_closest PMC_NOTE="k_wf_closest (K5 closest-hit walks, 1024x1024 256 spp): bytes beyond L2 of the BVH node / leaf records and the closest query records (Infinity Cache hits included)" \
    python3 "$R/scripts/summarize_pmc.py" "$P/${TAG}_pmc_k5_closest_traffic.json" "$OUT/k5_fetch" "$OUT/k5_write" > /dev/null
python3 "$R/scripts/stamp_traffic.py" "$P/${TAG}_pmc_k5_traffic.json" "$P/traffic_k5.json" median \
    "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), k_wf_shadow, 1024x1024 256spp 4b, median over its dispatches; profiles/${TAG}_pmc_k5_traffic.json; FETCH doubled (gfx950)" \
    "$P/${TAG}_pmc_k5_closest_traffic.json"
cd "$R"
cp "$P/traffic_k5.json" "$R/profiles/traffic_k5.json"
timeout -k 10 400 python3 "$R/bench.py" --config k5 > "$P/${TAG}_bench_k5.json" 2> "$OUT/bench_k5.err"
cat "$P/${TAG}_bench_k5.json"
fi
