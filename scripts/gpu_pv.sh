#!/bin/bash
# GPU session: partial-view tests + config-5 bench (+ kernel trace)
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pv}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step tests 600 python -u -m pytest tests/test_pview_gpu.py -x -v --timeout 300 --timeout-method thread
tail -3 "$OUT/tests.log"
step bench 300 python -u scripts/bench_pview.py
tail -1 "$OUT/bench.log"
cd /tmp
step trace 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_pview.py" --steps 10 --warmup 3 --no-cpu-baseline
echo done
