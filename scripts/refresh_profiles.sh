#!/bin/bash
# Re-measure the K2 artifacts under profiles/ on a GPU box (dev tool):
#   1. HBM traffic of k_render: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE
#      (separate passes, kernel trace only) -> gpurun_out/traffic_k2.json
#   2. kernel trace + stats of bench.py (the same command the bench line uses)
#   3. the bench line itself (with the CPU baseline) -> gpurun_out/bench_k2.json
# Usage (from the repo root): gpurun -- bash scripts/refresh_profiles.sh TAG
# Every GPU step runs under its own time limit; the script stops at the first
# failure.
set -euo pipefail
TAG=${1:-r01}
R=$PWD
OUT=$R/gpurun_out/refresh_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc_fetch" -o p -- python3 "$R/scripts/prof_k2.py" 3 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv \
    -d "$OUT/pmc_write" -o p -- python3 "$R/scripts/prof_k2.py" 3 > "$OUT/pmc_write.log" 2>&1
python3 "$R/scripts/summarize_pmc.py" "$OUT/pmc_traffic.json" "$OUT/pmc_fetch" "$OUT/pmc_write" > /dev/null
python3 - "$OUT/pmc_traffic.json" "$R/profiles/traffic_k2.json" "$OUT/traffic_k2.json" "$TAG" <<'EOF'
import json, sys
src, *dst, tag = sys.argv[1:]
d = json.load(open(src))
m = d["per_dispatch_median"]
t = {"hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
     "fetch_kib_raw": m.get("FETCH_SIZE"), "write_kib": m.get("WRITE_SIZE"),
     "source": ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), k_render, "
                "512x512 64spp 4b; profiles/%s_pmc_k2_traffic.json; FETCH doubled (gfx950)" % tag)}
for p in dst:
    json.dump(t, open(p, "w"), indent=1)
print(json.dumps(t))
EOF
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o k2 \
    -- python3 "$R/bench.py" --steps 10 --no-cpu-baseline --no-check > "$OUT/trace_bench.log" 2>&1
timeout -k 10 400 python3 "$R/bench.py" > "$OUT/bench_k2.json" 2> "$OUT/bench_k2.err"
cat "$OUT/bench_k2.json"
