#!/bin/bash
# Once-per-tick segment order (segment_sort_kernel) A/B on the headline form, then the scale
# parity tests.   bash scripts/gpu_r04i.sh <tag>
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-r04i}"
mkdir -p "$OUT"
timeout -k 10 600 python -u scripts/ab_scale_tiles.py 3 base: noearly:GSP_LIB_VARIANT=noearly nopre:GSP_LIB_VARIANT=nopresort > "$OUT/ab.txt" 2>&1 || exit $?
cat "$OUT/ab.txt"
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py tests/test_policy_gpu.py tests/test_events_gpu.py tests/test_scale_rules_vs_reference.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; exit $rc
