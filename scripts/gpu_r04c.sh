#!/bin/bash
# Round 4: evict_order tests, the 8-row-shard full-size test, the RCCL rank program's capacity
# cases (one rank), the in-degree skew per eviction order, and one rocprofv3 kernel trace per
# config (3, 4, 5) of the final kernels.
#   bash scripts/gpu_r04c.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04c}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp GSP_TEST_RECORD_DIR="$OUT"
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi.py \
    tests/test_pview_gpu.py tests/test_rccl_multi_gpu.py tests/test_events_gpu.py
step skew 300 python -u scripts/pview_skew.py --ticks 100 --out "$OUT/skew.json"
cd /tmp
R=$GRAFT_REPO_ROOT
step trace_c3 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c3" -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events
step trace_c4 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c4" -o run --output-format csv -- python3 $R/scripts/bench_full.py --nodes 262144 --steps 8 --warmup 2
step trace_c5 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c5" -o run --output-format csv -- python3 $R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
echo done
