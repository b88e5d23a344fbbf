#!/bin/bash
# Round 3: GPU suite, partial-view A/B (persistent grids vs exact grids + host sync), TLB
# counters per full-view tile width, config-4 tile-count probe.
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03e}
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
step tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -2 "$OUT/tests.log"
for i in 1 2; do
    for v in exact:GSP_PV_SPLITSYNC=1 persist:GSP_PV_SPLITSYNC=0; do
        name=${v%%:*}
        step ab_${name}_$i 150 env ${v#*:} python3 -u scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline
        echo "$name $i $(tail -1 "$OUT/ab_${name}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms=%.3f csr_ms=%.3f step_ms=%.3f" % (d["roofline"]["kernel_ms_per_tick"], d["exchange_csr_ms"], d["ms_per_step"]))')"
    done
done
step pvprof 150 env GSP_PV_PROFILE=1 python3 -u scripts/bench_pview.py --steps 10 --warmup 5 --no-cpu-baseline
grep "pview phases" "$OUT/pvprof.log"
cd /tmp
for G in 1 8 16; do
    step tlb_g$G 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d "$OUT/tlb_g$G" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tile_run.py $G
    step lat_g$G 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d "$OUT/lat_g$G" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tile_run.py $G
done
cd "$GRAFT_REPO_ROOT"
for G in 16 32 64; do
    step c4_g$G 200 python3 -u scripts/tile_run.py $G --nodes 262144 --ticks 4 --warmup 2
    tail -1 "$OUT/c4_g$G.log"
done
for G in 1 8 16; do
    python3 scripts/pmc_by_kernel.py scale_tick_kernel $(ls "$OUT"/tlb_g$G/*counter_collection.csv) $(ls "$OUT"/lat_g$G/*counter_collection.csv) --json "$OUT/tlb_g$G.json" > "$OUT/tlb_g$G.txt"
done
echo done
