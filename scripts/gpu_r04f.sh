#!/bin/bash
# Round 4: partial-view parity with the merged-orphan survivor slots (product library), the
# same suite on the predicated-pass variant (GSP_LIB_VARIANT=mow), then the A/B of both against
# the one-multiply-hash library of r04c ("hash").
#   bash scripts/gpu_r04f.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04f}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -1 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
T="tests/test_pview_gpu.py tests/test_events_gpu.py tests/test_policy_gpu.py -k pview_or_partial"
step tests_base 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pview_gpu.py tests/test_events_gpu.py tests/test_policy_gpu.py -k "pview or partial"
GSP_LIB_VARIANT=mow step tests_mow 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pview_gpu.py tests/test_events_gpu.py tests/test_policy_gpu.py -k "pview or partial"
bash scripts/ab_pview_pmc.sh "$TAG/ab" base mow hash
