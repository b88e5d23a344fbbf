#!/bin/bash
# Round 4 PMC passes (one rocprofv3 run per counter group, each under its own time limit),
# every figure over the driver's bench window (ticks 6-25) via scripts/pmc_window.py:
#   config 5: FETCH_SIZE, WRITE_SIZE, SQ instruction counts of the tick kernels;
#   config 3: FETCH_SIZE, WRITE_SIZE of the 8 tile launches per tick;
#   VERDICT r03 item 8, config 3 (8 tiles) against config 4 (32 tiles): address translation,
#   L2-miss latency and memory-side read requests (all / DRAM) per tick.
#   bash scripts/gpu_r04d.sh <tag>
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04d}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() {   # step <name> <timeout> cmd...; stop the session on a failure / crash / timeout
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
cd /tmp
PVB="$R/scripts/bench_pview.py --steps 20 --warmup 5 --no-cpu-baseline"
C3B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pview --no-262k --no-events"
pmc() {   # pmc <name> <timeout> <program args...> -- counters given in PMC
    local name=$1 to=$2; shift 2
    step $name $to rocprofv3 --pmc $PMC -d "$OUT/$name" -o run --output-format csv -- python3 "$@"
}
PMC="FETCH_SIZE" pmc pv_fetch 200 $PVB
PMC="WRITE_SIZE" pmc pv_write 200 $PVB
PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" pmc pv_sq 200 $PVB
PMC="FETCH_SIZE" pmc c3_fetch 200 $C3B
PMC="WRITE_SIZE" pmc c3_write 200 $C3B
for cfg in "c3 8 65536 6 4" "c4 32 262144 3 2"; do
    set -- $cfg
    name=$1 G=$2 N=$3 T=$4 W=$5
    PMC="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" pmc ${name}_tlb 300 $R/scripts/tile_run.py $G --nodes $N --ticks $T --warmup $W
    PMC="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" pmc ${name}_lat 300 $R/scripts/tile_run.py $G --nodes $N --ticks $T --warmup $W
    PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" pmc ${name}_ea 300 $R/scripts/tile_run.py $G --nodes $N --ticks $T --warmup $W
done
cd "$R"
W5="--anchor pview_receipt_kernel --ticks 6 25 --kernels pview_tick"
python3 scripts/pmc_window.py $(ls "$OUT"/pv_*/*counter_collection.csv) $W5 --json "$OUT/pv_window.json" > /dev/null
W3="--anchor tile_sum_kernel --ticks 6 25 --kernels scale_tick_kernel"
python3 scripts/pmc_window.py $(ls "$OUT"/c3_fetch/*counter_collection.csv "$OUT"/c3_write/*counter_collection.csv) $W3 --json "$OUT/c3_window.json" > /dev/null
python3 scripts/pmc_window.py $(ls "$OUT"/c3_tlb/*counter_collection.csv "$OUT"/c3_lat/*counter_collection.csv "$OUT"/c3_ea/*counter_collection.csv) --anchor tile_sum_kernel --ticks 5 10 --kernels scale_tick_kernel --json "$OUT/c3_mem.json" > /dev/null
python3 scripts/pmc_window.py $(ls "$OUT"/c4_tlb/*counter_collection.csv "$OUT"/c4_lat/*counter_collection.csv "$OUT"/c4_ea/*counter_collection.csv) --anchor tile_sum_kernel --ticks 3 5 --kernels scale_tick_kernel --json "$OUT/c4_mem.json" > /dev/null
echo done
