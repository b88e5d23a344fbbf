#!/bin/bash
# Round 3 final-tree evidence, part 1: the whole -m gpu suite, smoke(), the default bench line
# and a rocprofv3 kernel trace of the bench (part 2, the PMC passes: scripts/gpu_r03_pmc.sh).
#   bash scripts/gpu_r03_final.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03final}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -1 "$OUT/tests.log"
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 "$OUT/smoke.log"
step bench 420 python -u bench.py
tail -c 400 "$OUT/bench.log"
cd /tmp
step trace 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
