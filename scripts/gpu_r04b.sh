#!/bin/bash
# Round 4: full-view long rows as a deferred list + scale_long_kernel (tests + headline A/B),
# the parallel receipt kernel (partial-view tests + CSR/receipt time over ticks 6-105).
#   bash scripts/gpu_r04b.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04b}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_policy_gpu.py tests/test_pview_gpu.py tests/test_events_gpu.py tests/test_scale_gpu.py
bash scripts/ab_scale.sh "$TAG/ab" base nolong base nolong || exit 1
step pv100 400 python -u scripts/bench_pview.py --steps 100 --warmup 5 --no-cpu-baseline
echo done
