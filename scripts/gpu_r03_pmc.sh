#!/bin/bash
# Round 3 final-tree evidence, part 2: PMC passes (one rocprofv3 run per counter group, each
# under its own time limit) -- full-view HBM traffic per tick (8 column tiles), partial-view HBM
# traffic and SQ instruction counts per tick; summaries in the files bench.py reads.
#   bash scripts/gpu_r03_pmc.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03pmc}
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
cd /tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events"
if [ "${PV_ONLY:-0}" = 0 ]; then
step pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $BENCH
step pmc_write 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $BENCH
fi
PVB="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 30 --warmup 5 --no-cpu-baseline"   # bench.py's pview window
step pv_fetch 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pv_fetch" -o run --output-format csv -- python3 $PVB
step pv_write 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pv_write" -o run --output-format csv -- python3 $PVB
step pv_sq 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/pv_sq" -o run --output-format csv -- python3 $PVB
cd "$GRAFT_REPO_ROOT"
[ "${PV_ONLY:-0}" = 0 ] && python3 scripts/pmc_traffic.py $(ls "$OUT"/pmc_fetch/*counter_collection.csv) $(ls "$OUT"/pmc_write/*counter_collection.csv) "$OUT/pmc_traffic.json" --tiles 8
python3 scripts/pmc_traffic.py $(ls "$OUT"/pv_fetch/*counter_collection.csv) $(ls "$OUT"/pv_write/*counter_collection.csv) "$OUT/pmc_traffic_pview.json" --pview
python3 scripts/pmc_summary.py "pview_tick_split_kernel<0, " $(ls "$OUT"/pv_sq/*counter_collection.csv) \
    --per-tick "pview_tick_split_kernel<0, 128, 0, 3," --json "$OUT/pmc_sq_pview.json"
echo done
