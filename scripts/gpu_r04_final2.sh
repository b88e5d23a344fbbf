#!/bin/bash
# Round 4 final tree (after the receive-path work): the whole -m gpu suite, smoke(), the default
# bench line, then one rocprofv3 kernel trace per config (3, 4, 5) so each line's kernel time
# reads from one CSV line.   bash scripts/gpu_r04_final2.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04final2}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -1 "$OUT/$name.log" | head -c 600; echo
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python -u bench.py
cd /tmp
R=$GRAFT_REPO_ROOT
step trace_c3 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c3" -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events
step trace_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c4" -o run --output-format csv -- python3 $R/scripts/bench_full.py --nodes 262144 --steps 8 --warmup 2
step trace_c5 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c5" -o run --output-format csv -- python3 $R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
