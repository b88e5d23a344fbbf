#!/bin/bash
# Two PMC passes of the drain-all config-5 run (scripts/bench_pview.py --inbox 0, ticks 1-25):
# SQ issue / wait / LDS counters per kernel instance (scripts/pmc_by_kernel.py), for the drain
# kernels and the split kernels.  [DRAIN_VARIANT=<tag>: GSP_LIB_VARIANT]
#   bash scripts/pmc_drain.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:?usage: $0 <tag>}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp || exit 2
pass() {   # pass <name> <counters...>
    local name=$1; shift
    GSP_LIB_VARIANT=${DRAIN_VARIANT:-} timeout -k 10 240 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv -- \
        python3 "$R/scripts/bench_pview.py" --steps 20 --warmup 5 --no-cpu-baseline --inbox 0 > "$OUT/pmc_$name.log" 2>&1
    local rc=$?
    echo "pmc $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
    python3 "$R/scripts/pmc_by_kernel.py" pview_drain,pview_tick_split $(ls "$OUT"/pmc_$name/*counter_collection.csv) --json "$OUT/pmc_$name.json" > "$OUT/pmc_$name.txt"
}
pass a SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU
pass b SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES
echo done
