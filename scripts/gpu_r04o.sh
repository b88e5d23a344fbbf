#!/bin/bash
# Headline tick kernel compiled for 7 waves per SIMD (72 VGPRs) vs 6 (79): A/B on the 8-tile form.
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-r04o}"
mkdir -p "$OUT"
timeout -k 10 600 python -u scripts/ab_scale_tiles.py 3 base: w7:GSP_LIB_VARIANT=w7 > "$OUT/ab.txt" 2>&1
rc=$?; cat "$OUT/ab.txt"; exit $rc
