#!/bin/bash
# Round 4 final-tree evidence: the whole -m gpu suite, smoke(), the default bench line and a
# rocprofv3 kernel trace of the default bench run.
#   bash scripts/gpu_r04_final.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04final}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -1 "$OUT/$name.log" | head -c 1500; echo
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python -u bench.py
cd /tmp
step trace 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
