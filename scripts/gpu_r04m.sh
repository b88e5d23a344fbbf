#!/bin/bash
# vectorized key and value LDS writes A/B + pview parity tests.  bash scripts/gpu_r04k.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04k}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_pview_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_pview_pmc.sh "$TAG/ab" base scalarkeys
