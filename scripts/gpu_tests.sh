#!/bin/bash
# GPU session: the whole -m gpu suite (one process), then optionally a bench line.
#   bash scripts/gpu_tests.sh <tag> [bench]
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tests}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit $rc
if [ "$2" = bench ]; then
    timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?
    tail -c 600 "$OUT/bench.json"
    exit $rc
fi
