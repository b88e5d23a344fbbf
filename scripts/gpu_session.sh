#!/bin/bash
# One GPU session, steps in order, stopping at the first failure / crash / timeout:
#   bash scripts/gpu_session.sh <tag> <step>...
# steps: tests (the whole -m gpu suite), tests:<pytest -k expr>, smoke, bench,
#        trace3 / trace5 (rocprofv3 kernel trace of config 3 / config 5 alone, ticks 1-25),
#        bench5 (config 5 alone, default window), cmd:<shell command> (anything else, 600 s)
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() {   # step <name> <timeout> cmd...
    local name=$1 to=$2; shift 2
    ( cd /tmp && timeout -k 10 "$to" "$@" ) > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "$OUT/$name.log" | cut -c1-600
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in "$@"; do
    case $s in
        tests) step tests 1100 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
        tests:*) step tests_k 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${s#tests:}" ;;
        smoke) step smoke 200 python -u -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python -u $R/bench.py ;;
        bench5) step bench5 300 python -u $R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline ;;
        trace3) step trace3 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace3" -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events ;;
        trace5) step trace5 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace5" -o run --output-format csv -- python3 $R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline ;;
        cmd:*) step cmd 600 bash -c "cd $R && ${s#cmd:}" ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo done
