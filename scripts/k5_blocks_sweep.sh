#!/bin/bash
# K5 wavefront render time over (shadow, closest) walk grid sizes (dev tool).
# Usage: bash scripts/k5_blocks_sweep.sh W SPP "sh,cl" ["sh,cl" ...]
set -euo pipefail
W=$1; SPP=$2; shift 2
for p in "$@"; do
  PT_WF_SHADOW_BLOCKS=${p%,*} PT_WF_CLOSEST_BLOCKS=${p#*,} timeout -k 10 120 python3 scripts/k5_env_sweep.py $W $SPP PT_WF_CLOSEST_BLOCKS ${p#*,} 2>&1 | grep -v amdgpu.ids | sed "s/^/sh=${p%,*} /"
done
