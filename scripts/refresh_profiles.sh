#!/bin/bash
# Re-measure the artifacts under profiles/ on a GPU box (dev tool):
#   1. HBM traffic of k_render (K2): rocprofv3 --pmc FETCH_SIZE, then
#      WRITE_SIZE (separate passes, kernel trace only), stamped with the
#      kernel-source hash bench.py checks -> gpurun_out/refresh_TAG/traffic_k2.json
#   2. kernel trace + stats of bench.py (the command the bench line uses)
#   3. the K2 bench line itself (with the CPU baseline)
#   4. the kernel stats of the K5 wavefront kernels, the HBM traffic of its
#      shadow walks (-> traffic_k5.json) and the K5 bench line
# Usage (from the repo root): gpurun -- bash scripts/refresh_profiles.sh TAG
# Every GPU step runs under its own time limit; the script stops at the first
# failure.  Copy what is to be kept from gpurun_out/refresh_TAG to profiles/.
set -euo pipefail
TAG=${1:-r02}
R=$PWD
OUT=$R/gpurun_out/refresh_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc_fetch" -o p -- python3 "$R/scripts/prof_k2.py" 3 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
    -d "$OUT/pmc_write" -o p -- python3 "$R/scripts/prof_k2.py" 3 > "$OUT/pmc_write.log" 2>&1
python3 "$R/scripts/summarize_pmc.py" "$OUT/pmc_traffic.json" "$OUT/pmc_fetch" "$OUT/pmc_write" > /dev/null
python3 - "$R" "$OUT/pmc_traffic.json" "$OUT/traffic_k2.json" "$TAG" <<'EOF'
import json, sys
root, src, dst, tag = sys.argv[1:]
sys.path.insert(0, root)
import bench
d = json.load(open(src))
m = d["per_dispatch_median"]
t = {"hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
     "fetch_kib_raw": m.get("FETCH_SIZE"), "write_kib": m.get("WRITE_SIZE"),
     "source_sha": bench.source_sha(),
     "source": ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), k_render, "
                "512x512 64spp 4b; profiles/%s_pmc_k2_traffic.json; FETCH doubled (gfx950)" % tag)}
json.dump(t, open(dst, "w"), indent=1)
print(json.dumps(t))
EOF
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o k2 \
    -- python3 "$R/bench.py" --steps 50 --no-cpu-baseline --no-check > "$OUT/trace_bench.log" 2>&1
cp "$OUT/traffic_k2.json" "$R/profiles/traffic_k2.json"
timeout -k 10 400 python3 "$R/bench.py" > "$OUT/bench_k2.json" 2> "$OUT/bench_k2.err"
cat "$OUT/bench_k2.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_k5" -o k5 \
    -- python3 "$R/bench.py" --config k5 --steps 1 --warmup 0 --no-cpu-baseline --no-check \
    > "$OUT/trace_k5.log" 2>&1
# HBM traffic of the K5 shadow walks (k_wf_shadow, the K5 line's roofline
# kernel) at the bench shape, mean over its dispatches (as the line averages)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc5_fetch" -o p -- python3 "$R/scripts/prof_k5.py" 1 1024 256 > "$OUT/pmc5_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
    -d "$OUT/pmc5_write" -o p -- python3 "$R/scripts/prof_k5.py" 1 1024 256 > "$OUT/pmc5_write.log" 2>&1
PMC_KERNEL=k_wf_shadow python3 "$R/scripts/summarize_pmc.py" "$OUT/pmc_k5_traffic.json" \
    "$OUT/pmc5_fetch" "$OUT/pmc5_write" > /dev/null
python3 "$R/scripts/stamp_traffic.py" "$OUT/pmc_k5_traffic.json" "$OUT/traffic_k5.json" mean \
    "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), k_wf_shadow, 1024x1024 256spp 4b, mean over its dispatches; profiles/${TAG}_pmc_k5_traffic.json; FETCH doubled (gfx950)"
cd "$R"
cp "$OUT/traffic_k5.json" "$R/profiles/traffic_k5.json"
timeout -k 10 400 python3 "$R/bench.py" --config k5 > "$OUT/bench_k5.json" 2> "$OUT/bench_k5.err"
cat "$OUT/bench_k5.json"
