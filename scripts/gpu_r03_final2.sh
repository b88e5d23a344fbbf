#!/bin/bash
# Round 3 final tree: the whole -m gpu suite, an A/B of the partial-view tick (AB="name:ENV ..."),
# smoke(), the default bench line and a rocprofv3 kernel trace of the bench.
#   AB="base: noown:GSP_LIB_VARIANT=noown" bash scripts/gpu_r03_final2.sh <tag>
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
for i in 1 2; do
    for spec in ${AB:-}; do
        name=${spec%%:*}
        envs=${spec#*:}
        step ab_${name}_$i 150 env $envs python3 -u scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
        echo "$name $i $(tail -1 "$OUT/ab_${name}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f csr_ms=%.3f step_ms=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["exchange_csr_ms"], d["ms_per_step"]))')"
    done
done
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 "$OUT/smoke.log"
step bench 420 python -u bench.py
tail -c 300 "$OUT/bench.log"
cd /tmp
step trace 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
