#!/bin/bash
# GPU session: partial-view phase profile (GSP_PV_PROFILE) + SQ PMC passes of the tick kernel
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pvprof}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 env GSP_PV_PROFILE=1 python3 -u scripts/bench_pview.py --steps 10 --warmup 5 --no-cpu-baseline > "$OUT/phases.log" 2>&1
rc=$?; echo "phases rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep "pview phases" "$OUT/phases.log"; tail -1 "$OUT/phases.log" | cut -c1-400
BENCH="$GRAFT_REPO_ROOT/scripts/bench_pview.py --steps 3 --warmup 5 --no-cpu-baseline"
cd /tmp
pass() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 $BENCH > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS
pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VALU
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_summary.py "pview_tick_kernel<8, 0>" $(ls "$OUT"/*/run_counter_collection.csv) --json "$OUT/summary.json"
echo done
