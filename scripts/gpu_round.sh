#!/bin/bash
# One GPU-box pass over everything the round's claims rest on (dev tool):
#   1. the GPU test suite (parity) -> gpurun_out/round_TAG/gputest.log
#   2. the band-scaling sweep (scripts/prof_scaling.py) -> scaling.jsonl
#   3. the profile refresh (scripts/refresh_profiles.sh TAG), staged for
#      scripts/install_profiles.py
#   4. every single-GPU BASELINE config at full size (scripts/run_configs.py)
#      -> staged as profiles/TAG_configs.jsonl
# Usage: gpurun -- bash scripts/gpu_round.sh TAG
# Each GPU step has its own time limit; a failed test run stops before the
# measurements, a fault or timeout stops everything.
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/round_$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    > "$OUT/gputest.log" 2>&1
rc=$?
tail -3 "$OUT/gputest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/prof_scaling.py 20 2>&1 | grep -v amdgpu.ids > "$OUT/scaling.jsonl" || exit 3
cat "$OUT/scaling.jsonl"
bash scripts/refresh_profiles.sh "$TAG" > "$OUT/refresh.log" 2>&1
rc=$?
tail -4 "$OUT/refresh.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u scripts/run_configs.py 2>&1 | grep -v amdgpu.ids \
    | tee "gpurun_out/refresh_$TAG/profiles/${TAG}_configs.jsonl"
