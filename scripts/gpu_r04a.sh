#!/bin/bash
# Round 4, first GPU session: the new tests (full-view join burst, pview forms with events and
# the rows-run counter), an A/B of the full-view headline kernel with / without the long-segment
# path, then the whole -m gpu suite.
#   bash scripts/gpu_r04a.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04a}
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
step newtests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_policy_gpu.py::test_full_view_join_burst_past_1024_messages" \
    "tests/test_pview_gpu.py::test_pview_kernel_forms_events_and_rows_run" \
    "tests/test_pview_gpu.py::test_pview_rows_run_queued_ticks" \
    "tests/test_pview_gpu.py::test_pview_rows_run_needs_the_env" \
    tests/test_scale_gpu.py -k "capacity or join_burst or rows_run or events_and_rows"
bash scripts/ab_scale.sh "$TAG/ab" base nolong base nolong || exit 1
step tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
